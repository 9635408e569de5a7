"""Diagnostic: per-tensor relative error (max|gpu - oracle| / max|oracle|) of one model step, for the
decoder path selected by S2S_DEC_MODE (default / persist / step).  python tools/step_errs.py B L T F O"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
import s2s_amd  # noqa: E402
from oracle import s2s_oracle as orc  # noqa: E402

B, L, T, F, O = (int(a) for a in sys.argv[1:6])
kw = dict(inputFrameSize=F, outputDepth=O)
cfg_o = orc.ModelConfig(**kw)
model = s2s_amd.ChorowskiBaseline(s2s_amd.ModelConfig(**kw))
P = orc.unflatten(model.params.cpu().double().numpy(), cfg_o)
x, labels = orc.synthetic_batch(cfg_o, B, L, T, seed=7, pad=min(10, L // 4), eos=min(23, O - 1))
nll, logp = model.step(torch.tensor(x, dtype=torch.float32, device="cuda"),
                       torch.tensor(labels, dtype=torch.int32, device="cuda"))
torch.cuda.synchronize()
nll_ref, G, lref, enc = orc.training_step(x, labels, P, cfg_o)
Gg = orc.unflatten(model.grads.cpu().double().numpy(), cfg_o)
mode = os.environ.get("S2S_DEC_MODE", "default")
out = [f"logp {np.abs(logp.cpu().numpy() - lref).max() / np.abs(lref).max():.2e}"]
for k in G:
    out.append(f"{k} {np.abs(Gg[k] - G[k]).max() / max(np.abs(G[k]).max(), 1e-30):.2e}")
print(mode, " ".join(out))
