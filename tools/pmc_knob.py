"""Workload for a rocprofv3 --pmc pass with a library debug knob set: three eager config-2 training steps.
rocprofv3 --pmc FETCH_SIZE -- python tools/pmc_knob.py s2s_debug_gru_fused_dy 0
(The knob separates a kernel's traffic streams: e.g. the BPTT launch with and without its fused dy producers.)"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
import s2s_amd  # noqa: E402
from s2s_amd import _lib  # noqa: E402


def main():
    if len(sys.argv) > 2:
        fn = getattr(_lib.lib, sys.argv[1])
        fn.argtypes = [ctypes.c_int]
        fn(int(sys.argv[2]))
    cfg = s2s_amd.ModelConfig()
    model = s2s_amd.ChorowskiBaseline(cfg, graph=False)
    B, L, T = 32, 128, 40
    x = torch.randn(B, L, cfg.inputFrameSize, device="cuda")
    lab = torch.randint(0, cfg.outputDepth, (B, T), device="cuda", dtype=torch.int32)
    for _ in range(3):
        model.step(x, lab)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
