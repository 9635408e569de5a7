"""Diagnostic: a few conv + BiLSTM model steps (timit/timit.lua:106-145 sizes) for rocprofv3."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "seq2seq-attention-asr_amd")]
import torch  # noqa: E402

import s2s_amd  # noqa: E402

torch.manual_seed(0)
m = s2s_amd.ConvBiLSTMAttentionModel(123).cuda()
x = torch.randn(32, 512, 123, device="cuda")
lab = torch.randint(0, 61, (32, 40), device="cuda", dtype=torch.int32)
for _ in range(4):
    m.zeroGradParameters()
    m.step(x, lab)
torch.cuda.synchronize()
print("done")
