"""Diagnostic: per-phase latency of the persistent decoder kernels from in-kernel s_memrealtime
stamps (100 MHz).  Run on a GPU box:  python tools/dec_stamps.py [B L T]"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
import s2s_amd  # noqa: E402
from s2s_amd import _lib  # noqa: E402


def phase_ends(st, T, parts):
    """st: (grid, T, 8) stamps; parts[ph] = list of workgroup indices (per tile) taking part."""
    nt = st.shape[0] // 128
    ends = np.zeros((nt, T, 8))
    for m in range(nt):
        for ph in range(8):
            ws = [m * 128 + w for w in parts[ph]]
            ends[m, :, ph] = st[ws, :, ph].max(0)
    return ends


def report(name, st, T, parts, labels):
    ends = phase_ends(st.astype(np.float64) * 10.0 / 1000.0, T, parts)  # -> microseconds
    lat = np.zeros((ends.shape[0], T, 8))
    for t in range(T):
        for ph in range(1, 8):
            prev = ends[:, t, ph - 1] if ph > 1 else (ends[:, t - 1, 7] if t > 0 else ends[:, t, 0])
            lat[:, t, ph] = ends[:, t, ph] - prev
    m = lat[:, 1:, 1:].mean((0, 1))
    total = (ends[:, -1, 7] - ends[:, 0, 0]).mean()
    print(f"{name}: total {total:.1f} us, {total / T:.2f} us/step")
    for lab, v in zip(labels, m):
        print(f"   {lab:28s} {v:7.2f} us")


def main():
    B, L, T = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (32, 128, 40)
    cfg = s2s_amd.ModelConfig()
    model = s2s_amd.ChorowskiBaseline(cfg)
    x = torch.randn(B, L, cfg.inputFrameSize, device="cuda")
    lab = torch.randint(0, cfg.outputDepth, (B, T), device="cuda", dtype=torch.int32)
    grid = 128 * ((B + 15) // 16)
    sf = torch.zeros(grid * T * 8, dtype=torch.int64, device="cuda")
    sb = torch.zeros_like(sf)
    fn = _lib.lib.s2s_debug_dec_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    fn(sf.data_ptr(), sb.data_ptr())
    model.step(x, lab)
    torch.cuda.synchronize()
    fn(None, None)
    S, A, Sc = cfg.stateDepth, cfg.annotationDepth, cfg.scoreDepth
    allw = list(range(128))
    fparts = {0: allw, 1: list(range(Sc // 16)), 2: allw, 3: list(range(32, 32 + 16 * ((A + 255) // 256))),
              4: list(range(64, 64 + S // 16)), 5: list(range(80, 80 + S // 16)), 6: list(range(96, 96 + 2 * S // 16)),
              7: list(range(96, 96 + S // 16))}
    bparts = {0: allw, 1: list(range(S // 16)), 2: list(range(S // 16)) + list(range(16, 16 + S // 16)),
              3: list(range(32, 32 + 2 * S // 16)), 4: list(range(64, 64 + A // 16)), 5: allw,
              6: list(range(96, 96 + 16 * ((Sc + 255) // 256))), 7: list(range(S // 16))}
    report("decoder forward", sf.cpu().numpy().reshape(grid, T, 8), T, fparts,
           ["P1 ws", "P2 attention", "P3 combine", "P4 c_in", "P5 d", "P6 z|r", "P7 hh,s"])
    report("decoder backward", sb.cpu().numpy().reshape(grid, T, 8)[:, ::-1, :].copy(), T, bparts,
           ["Q1 dq", "Q2 ds|dd", "Q3 Wd^T", "Q4 Wc^T", "Q5 attention", "Q6 dws", "Q7 Ws^T+gates"])


if __name__ == "__main__":
    main()
