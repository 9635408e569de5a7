"""Diagnostic: run the attention decoder fwd+bwd repeatedly (XCD-local kernels, both hand-off forms)
and report whether outputs are bitwise stable and their error vs the oracle.
python tools/dec_determinism.py B L T A Sc S O pen"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
import s2s_amd  # noqa: E402
from s2s_amd import _lib  # noqa: E402
from oracle import s2s_oracle as orc  # noqa: E402

B, L, T, A, Sc, S, O = (int(a) for a in sys.argv[1:8])
pen = float(sys.argv[8])
M, K = 4, 7
fn = _lib.lib.s2s_debug_dec_local
fn.argtypes = [ctypes.c_int]
rng = np.random.default_rng(L * 7 + T)
cfg = orc.ModelConfig(inputFrameSize=8, hiddenFrameSize=16, outputFrameSize=A // 2, scoreDepth=Sc, stateDepth=S,
                      outputDepth=O, mlpDepth=M, maxoutWindow=K, penalty=pen, numLayers=1)
att = s2s_amd.Attention(s2s_amd.GRU(S, S), s2s_amd.MaxoutMLP(S + A, M, K, O), Sc, 10, 0, S, A, O, True, pen).cuda()
NAMES = ("V", "Ws", "bs", "we", "Wy", "by", "Wc", "bc", "Wd", "bd", "dec.Wz", "dec.Wr", "dec.Wh", "Wm", "bm", "Wo", "bo")
P = {n: t.cpu().double().numpy() for n, t in zip(NAMES, att.parameters()[0])}
h = rng.standard_normal((B, L, A)) * 0.5
labels = rng.integers(0, O, (B, T)).astype(np.int32)
hs = torch.tensor(h, dtype=torch.float32, device="cuda")
ls = torch.tensor(labels, dtype=torch.int32, device="cuda")
lref, cache = orc.attention_fwd(h, labels, P, cfg)
dlogp = rng.standard_normal(lref.shape)
G = orc.zeros_like_params(P)
dhr = orc.attention_bwd(P, cfg, cache, dlogp, G, 0.5)
first = None
W = [t.clone() for t in att.parameters()[0]]
for local in (1, 0, 1, 0):
    fn(local)
    for rep in range(2):
        if os.environ.get("NEW_MODULE"):
            att = s2s_amd.Attention(s2s_amd.GRU(S, S), s2s_amd.MaxoutMLP(S + A, M, K, O), Sc, 10, 0, S, A, O, True,
                                    pen).cuda()
            for dst, src in zip(att.parameters()[0], W):
                dst.copy_(src)
        logp = att.forward([hs, ls]).clone()
        att.zeroGradParameters()
        dh = att.backward([hs, None], torch.tensor(dlogp, dtype=torch.float32, device="cuda"), 0.5)[0].clone()
        torch.cuda.synchronize()
        e_l = np.abs(logp.cpu().numpy() - lref).max() / np.abs(lref).max()
        e_h = np.abs(dh.cpu().numpy() - dhr).max() / np.abs(dhr).max()
        same = first is not None and torch.equal(first[0], logp) and torch.equal(first[1], dh)
        if first is None:
            first = (logp, dh)
        print(f"local={local} rep={rep} logp err {e_l:.2e} dh err {e_h:.2e} bitwise-same-as-first {same}")
fn(1)
