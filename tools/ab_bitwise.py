"""Bitwise A/B of one conv + BiLSTM model step (timit/timit.lua:106-145: LSTM encoder, LSTM decoder, hybrid
attention) and a beam search between two builds: run once per library (S2S_HIP_LIB), then compare.
  S2S_HIP_LIB=.../ab/base.so python tools/ab_bitwise.py save gpurun_out/ab_base.pt
  S2S_HIP_LIB=.../ab/new.so  python tools/ab_bitwise.py save gpurun_out/ab_new.pt
  python tools/ab_bitwise.py cmp gpurun_out/ab_base.pt gpurun_out/ab_new.pt"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))


def save(path):
    import s2s_amd
    g = torch.Generator().manual_seed(3)
    B, L, T = 8, 128, 12
    x = torch.randn((B, L, 123), generator=g).cuda()
    labels = torch.randint(0, 61, (B, T), generator=g).to(torch.int32).cuda()
    m = s2s_amd.ConvBiLSTMAttentionModel(generator=torch.Generator().manual_seed(1), penalty=0.1).cuda()
    m.zeroGradParameters()
    nll, logp = m.step(x, labels)
    out = {"nll": nll, "logp": logp, "grads": [t.clone() for t in m.parameters()[1]]}
    h = m.encoder.forward(x)
    toks, lens, scores = m.decoder.BeamSearch(h, 1, K=3, maxseqlength=6)
    out.update(beam_toks=toks, beam_scores=scores)
    torch.save({k: (v.cpu() if torch.is_tensor(v) else [t.cpu() for t in v]) for k, v in out.items()}, path)
    print("saved", path)


def cmp(a, b):
    A, Bd = torch.load(a, weights_only=True), torch.load(b, weights_only=True)
    bad = []
    for k in A:
        if isinstance(A[k], list):
            bad += [f"{k}[{i}]" for i, (x, y) in enumerate(zip(A[k], Bd[k])) if not torch.equal(x, y)]
        elif not torch.equal(A[k], Bd[k]):
            bad.append(k)
    print("bitwise equal" if not bad else f"DIFFER: {bad}")


if __name__ == "__main__":
    save(sys.argv[2]) if sys.argv[1] == "save" else cmp(sys.argv[2], sys.argv[3])
