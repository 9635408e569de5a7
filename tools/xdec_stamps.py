"""Diagnostic: per-phase latency of the XCD-local decoder kernels (dec_xcd.inc) from in-kernel
s_memrealtime stamps (100 MHz).  Run on a GPU box:  python tools/xdec_stamps.py [B L T]
Phase end = latest stamp over the chain's 32 workgroups; phase time = end - previous phase's end."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
import s2s_amd  # noqa: E402
from s2s_amd import _lib  # noqa: E402


def report(name, st, nph, labels):
    # st: (chains, 32, T, 8) stamps in processing order along axis 2
    ends = st[..., :nph].max(axis=1) * 0.01  # (chains, T, nph) microseconds
    T = ends.shape[1]
    lat = np.zeros((ends.shape[0], T, nph))
    for t in range(1, T):
        lat[:, t, 1:] = ends[:, t, 1:] - ends[:, t, :-1]
        lat[:, t, 0] = ends[:, t, 0] - ends[:, t - 1, nph - 1]
    m = lat[:, 1:].mean((0, 1))
    total = (ends[:, -1, nph - 1] - ends[:, 0, 0]).mean()
    print(f"{name}: {total:.1f} us over {T} steps = {total / T:.2f} us/step")
    t0 = ends[:, 0, 0].min()
    print("   per chain (start, end after the earliest loop start): " +
          ", ".join(f"{a - t0:.0f}-{b - t0:.0f}" for a, b in zip(ends[:, 0, 0], ends[:, -1, nph - 1])))
    for lab, v in zip(labels, m):
        print(f"   {lab:24s} {v:7.2f} us")


def prologue(name, st):
    # slots 11-15 of the first processed step: entry (15), sentinel slots re-armed (13), chain census (12), chunk rows
    # staged (11), loop start (14); times from the launch's first workgroup entry, latest workgroup per mark
    p = st[:, :, 0, :]
    if not (p[..., 15] > 0).all():
        return
    t0 = p[..., 15].min()
    marks = [("entry", 15), ("re-armed", 13), ("census", 12), ("staged", 11), ("loop start", 14)]
    print(f"{name} prologue (us after the first workgroup's entry, latest workgroup): " +
          ", ".join(f"{lab} {(p[..., s].max() - t0) * 0.01:.1f}" for lab, s in marks))


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    B, L, T = (int(a) for a in args[:3]) if len(args) > 2 else (32, 128, 40)

    cfg = s2s_amd.ModelConfig()
    model = s2s_amd.ChorowskiBaseline(cfg)
    x = torch.randn(B, L, cfg.inputFrameSize, device="cuda")
    lab = torch.randint(0, cfg.outputDepth, (B, T), device="cuda", dtype=torch.int32)
    nst = 8 * 32 * T * 16
    sf = torch.zeros(nst, dtype=torch.int64, device="cuda")
    sb = torch.zeros_like(sf)
    fn = _lib.lib.s2s_debug_dec_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    model.step(x, lab)  # warm
    torch.cuda.synchronize()
    fn(sf.data_ptr(), sb.data_ptr())
    model.step(x, lab)
    torch.cuda.synchronize()
    fn(None, None)
    U = (B + 7) // 8  # attn.hip dec_xcd_plan
    nch = (B + U - 1) // U
    f = sf.cpu().numpy().reshape(8 * 32, T, 16)[: nch * 32].reshape(nch, 32, T, 16).astype(np.float64)
    b = sb.cpu().numpy().reshape(8 * 32, T, 16)[: nch * 32].reshape(nch, 32, T, 16)[:, :, ::-1].astype(np.float64)
    prologue("decoder forward", f)
    report("decoder forward", f, 6, ["(loop)", "F1 ws,us", "F2 attention", "F3 combine", "F4 gx,z,r,q", "F5 hh,s"])
    prologue("decoder backward", b)
    report("decoder backward", b, 7, ["(loop)", "G gate grads", "B2 dq,da_r", "B3 dc,us'", "B4 attention",
                                       "B45 dws", "B5 ds"])


if __name__ == "__main__":
    main()
