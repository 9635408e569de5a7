"""Diagnostic: the XCDs' shader-clock frequency across a config-2 training step.  A bounded probe kernel
(s2s_debug_clock_probe, one single-lane workgroup per XCD) records (100 MHz real-time, shader-clock) counter pairs
every microsecond on a second stream while the step replays on the first; the clock rate over each 20 us bin is
printed beside the step's timeline.  Run on a GPU box:  python tools/clock_probe.py [steps]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
sys.path.insert(0, ROOT)
import s2s_amd  # noqa: E402
from s2s_amd import _lib  # noqa: E402
from bench import CONFIGS  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    kw, B, L, T = CONFIGS["timit_chorowski_b32"]
    cfg = s2s_amd.ModelConfig(**kw)
    model = s2s_amd.ChorowskiBaseline(cfg, graph=True, seed=1234)
    g = torch.Generator(device="cpu").manual_seed(1234)
    x = torch.randn((B, L, cfg.inputFrameSize), generator=g).cuda()
    lab = torch.randint(0, cfg.outputDepth - 1, (B, T), generator=g).to(torch.int32).cuda()
    stream, side = torch.cuda.Stream(), torch.cuda.Stream()
    for _ in range(3):
        model.step(x, lab, stream=stream)
    torch.cuda.synchronize()
    fn = _lib.lib.s2s_debug_clock_probe
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    nwg, period = 8, 100
    n = int((300 + steps * 3400) / (period / 100.0))
    out = torch.zeros(nwg * n * 2, dtype=torch.int64, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    _lib.check(fn(ctypes.c_void_p(side.cuda_stream), nwg, n, period, ctypes.c_void_p(out.data_ptr())))
    with torch.cuda.stream(stream):
        ev[0].record()
        for i in range(steps):
            model.step(x, lab, stream=stream)
            ev[i + 1].record()
    torch.cuda.synchronize()
    print("step times (ms):", [round(ev[i].elapsed_time(ev[i + 1]), 3) for i in range(steps)])
    a = out.cpu().numpy().reshape(nwg, n, 2).astype(np.float64)
    r0 = a[:, 0, 0].min()
    binw = 20.0
    print(f"per-XCD shader clock (MHz) in {binw:.0f} us bins, t from the first sample")
    rows = {}
    for w in range(nwg):
        t = (a[w, :, 0] - r0) * 0.01
        dr = np.diff(a[w, :, 0]) * 0.01  # us
        dc = np.diff(a[w, :, 1])
        f = dc / np.maximum(dr, 1e-9)  # cycles per us = MHz
        b = (t[1:] // binw).astype(int)
        for k in np.unique(b):
            rows.setdefault(k, [np.nan] * nwg)[w] = f[b == k].mean()
    for k in sorted(rows):
        print(f"{k * binw:8.0f} " + " ".join(f"{v:6.0f}" for v in rows[k]))
    allf = np.array([v for r in rows.values() for v in r if np.isfinite(v)])
    print(f"clock min {allf.min():.0f} median {np.median(allf):.0f} max {allf.max():.0f} MHz")


if __name__ == "__main__":
    main()
