"""Diagnostic: fused x-projection of the persistent GRU forward vs the per-step path (GPU box)."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
import s2s_amd  # noqa: E402

B, L, D, H = (int(v) for v in sys.argv[1:5]) if len(sys.argv) > 4 else (32, 16, 64, 256)
rng = np.random.default_rng(3)
x = torch.tensor(rng.standard_normal((B, L, D)), dtype=torch.float32, device="cuda")
f, b = s2s_amd.GRU(D, H), s2s_amd.GRU(D, H)
out = {}
for mode in ("step", "persistent"):
    os.environ["S2S_GRU_MODE"] = mode
    mod = s2s_amd.BiRNN(f, b).cuda()
    t0 = time.time()
    y = mod.forward(x).clone()
    torch.cuda.synchronize()
    print(mode, "fwd done in", round(time.time() - t0, 3), "s", flush=True)
    out[mode] = y
d = (out["step"] - out["persistent"]).abs().max().item()
print("max abs diff", d, "equal", torch.equal(out["step"], out["persistent"]), flush=True)
