"""A/B a library debug knob on the config-2 training step (graph replay), alternating arms in one process.
python tools/ab_debug_knob.py s2s_debug_dec_u4 1 0 [rounds]"""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
import s2s_amd  # noqa: E402
from s2s_amd import _lib  # noqa: E402


def main():
    name, a, b = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    fn = getattr(_lib.lib, name)
    fn.argtypes = [ctypes.c_int]
    cfg = s2s_amd.ModelConfig()
    model = s2s_amd.ChorowskiBaseline(cfg, graph=False)  # a knob is a kernel argument: no captured graphs
    B, L, T = 32, 128, 40
    x = torch.randn(B, L, cfg.inputFrameSize, device="cuda")
    lab = torch.randint(0, cfg.outputDepth, (B, T), device="cuda", dtype=torch.int32)
    res = {a: [], b: []}
    for r in range(rounds):
        for v in (a, b):
            fn(v)
            for _ in range(3):
                model.step(x, lab)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(30):
                model.step(x, lab)
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / 30 * 1e3)
    for v in (a, b):
        xs = sorted(res[v])
        print(f"{name}={v}: median {xs[len(xs) // 2]:.3f} ms/step  all {' '.join(f'{t:.3f}' for t in res[v])}")


if __name__ == "__main__":
    main()
