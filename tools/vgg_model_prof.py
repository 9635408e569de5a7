"""Diagnostic: a few VGG model steps (BASELINE config 5 shape) for rocprofv3."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "seq2seq-attention-asr_amd")]
import torch  # noqa: E402

import s2s_amd  # noqa: E402

torch.manual_seed(0)
m = s2s_amd.VGGAttentionModel(40, outputFrameSize=512, hidden=2048, outputDepth=29).cuda()
x = torch.randn(16, 3, 1024, 40, device="cuda")
lab = torch.randint(0, 28, (16, 200), device="cuda", dtype=torch.int32)
for _ in range(3):
    m.zeroGradParameters()
    m.step(x, lab)
torch.cuda.synchronize()
print("done")
