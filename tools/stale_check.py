"""Diagnostic: decoder fwd+bwd on fresh random modules -- parameter checksum, error vs the oracle, and
whether a second run on the same module is bitwise equal (python tools/stale_check.py)."""
import ctypes
import sys

sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/seq2seq-attention-asr_amd")
import numpy as np
import torch
assert torch.cuda.is_available()
import s2s_amd  # noqa: E402
from oracle import s2s_oracle as orc  # noqa: E402

B, L, Tn, A, Sc, S, O, M, K = (int(a) for a in sys.argv[1:10]) if len(sys.argv) > 9 else (21, 50, 9, 128, 128, 64, 29, 4, 7)
pen = float(sys.argv[10]) if len(sys.argv) > 10 else 0.2
names = ("V", "Ws", "bs", "we", "Wy", "by", "Wc", "bc", "Wd", "bd", "dec.Wz", "dec.Wr", "dec.Wh", "Wm", "bm", "Wo", "bo")
cfg = orc.ModelConfig(inputFrameSize=8, hiddenFrameSize=16, outputFrameSize=A // 2, scoreDepth=Sc, stateDepth=S,
                      outputDepth=O, mlpDepth=M, maxoutWindow=K, penalty=pen, numLayers=1)
for trial in range(8):
    rng = np.random.default_rng(L * 7 + Tn)
    att = s2s_amd.Attention(s2s_amd.GRU(S, S), s2s_amd.MaxoutMLP(S + A, M, K, O), Sc, 10, 0, S, A, O, True, pen).cuda()
    P = {n: t.cpu().double().numpy() for n, t in zip(names, att.parameters()[0])}
    csum = sum(float(v.sum()) for v in P.values())
    h = rng.standard_normal((B, L, A)) * 0.5
    labels = rng.integers(0, O, (B, Tn)).astype(np.int32)
    hs = torch.tensor(h, dtype=torch.float32, device="cuda")
    ls = torch.tensor(labels, dtype=torch.int32, device="cuda")
    lref, cache = orc.attention_fwd(h, labels, P, cfg)
    dlogp = rng.standard_normal(lref.shape)
    G = orc.zeros_like_params(P)
    dhr = orc.attention_bwd(P, cfg, cache, dlogp, G, 0.5)
    outs = []
    for rep in range(3):
        logp = att.forward([hs, ls]).clone()
        al = att.alpha().clone()
        att.zeroGradParameters()
        dh = att.backward([hs, None], torch.tensor(dlogp, dtype=torch.float32, device="cuda"), 0.5)[0].clone()
        g = [t.clone() for t in att.parameters()[1]]
        torch.cuda.synchronize()
        outs.append((logp, al, dh, g))
    e = np.abs(outs[0][2].cpu().numpy() - dhr).max() / np.abs(dhr).max()
    same = [torch.equal(outs[0][2], o[2]) and all(torch.equal(a, b) for a, b in zip(outs[0][3], o[3])) for o in outs[1:]]
    samef = [torch.equal(outs[0][0], o[0]) for o in outs[1:]]
    gerr = {n: np.abs(outs[0][3][i].cpu().double().numpy() - G[n]).max() / max(np.abs(G[n]).max(), 1e-30)
            for i, n in enumerate(names)}
    worst = sorted(gerr.items(), key=lambda kv: -kv[1])[:3]
    # MonotonicAlignment indicator decisions (diff_t > 0) from the GPU's and the oracle's alphas
    wl = (L - np.arange(L))[None, None, :]
    def diffs(a):
        prev = np.concatenate([np.zeros_like(a[:, :1]), a[:, :-1]], 1)
        return (wl * (a - prev)).sum(-1)
    dg, dr = diffs(outs[0][1].cpu().double().numpy()), diffs(cache["alpha"])
    flips = int((np.sign(dg) != np.sign(dr)).sum())
    print(f"    indicator flips {flips}, min |diff| {np.abs(dr).min():.2e}", flush=True)
    print(f"trial {trial} csum {csum:.6f} dh err {e:.2e} fwd-same {samef} bwd-same {same} worst grads "
          + " ".join(f"{n}:{v:.1e}" for n, v in worst), flush=True)
