"""Diagnostic: sub-phases of the XCD-local decoder forward's attention (F2 / F3), per workgroup means
from the in-kernel stamps (slot 6 = ws_t arrived, slot 7 = scores done).  python tools/xdec_substamps.py"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
import s2s_amd  # noqa: E402
from s2s_amd import _lib  # noqa: E402


def main():
    B, L, T = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (32, 128, 40)
    cfg = s2s_amd.ModelConfig()
    model = s2s_amd.ChorowskiBaseline(cfg)
    x = torch.randn(B, L, cfg.inputFrameSize, device="cuda")
    lab = torch.randint(0, cfg.outputDepth, (B, T), device="cuda", dtype=torch.int32)
    sf = torch.zeros(8 * 32 * T * 16, dtype=torch.int64, device="cuda")
    sb = torch.zeros_like(sf)
    fn = _lib.lib.s2s_debug_dec_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    model.step(x, lab)
    torch.cuda.synchronize()
    fn(sf.data_ptr(), sb.data_ptr())
    model.step(x, lab)
    torch.cuda.synchronize()
    fn(None, None)
    U = (B + 7) // 8
    nch = (B + U - 1) // U
    st = sf.cpu().numpy().reshape(8 * 32, T, 16)[: nch * 32].reshape(nch, 32, T, 16).astype(np.float64) * 0.01
    st = st[:, :, 1:]  # skip step 0
    d = lambda a, b: (st[..., a] - st[..., b]).mean()  # noqa: E731
    print(f"F1 (all wgs)            {d(1, 0):6.2f} us  (step start -> ws/us published)")
    print(f"F2 wait ws_t            {d(6, 1):6.2f} us")
    print(f"F2 scores (tanh sums)   {d(7, 6):6.2f} us")
    print(f"F2 softmax+context+pub  {d(2, 7):6.2f} us")
    c = st[:, :8]
    print(f"F3 (combine wgs)        {(c[..., 3] - c[..., 2]).mean():6.2f} us  (poll partials + combine + publish c)")
    print(f"F4 (all wgs)            {d(4, 3):6.2f} us")
    print(f"F5 (all wgs)            {d(5, 4):6.2f} us")
    print(f"next step start         {(st[:, :, 1:, 0] - st[:, :, :-1, 5]).mean():6.2f} us")
    # backward: stamps in processing order p = 0.. (t = T-1-p); slot 7 = dc_t arrived in B4
    bt = sb.cpu().numpy().reshape(8 * 32, T, 16)[: nch * 32].reshape(nch, 32, T, 16)[:, :, ::-1].astype(np.float64) * 0.01
    bt = bt[:, :, 1:]
    db = lambda a, b: (bt[..., a] - bt[..., b]).mean()  # noqa: E731
    print(f"B2 (all wgs)            {db(2, 1):6.2f} us")
    print(f"B3 (all wgs)            {db(3, 2):6.2f} us")
    print(f"B4 pre + wait dc        {db(7, 3):6.2f} us")
    print(f"B4 de (dots, DE)        {db(8, 7):6.2f} us")
    print(f"B4 barrier              {db(9, 8):6.2f} us")
    print(f"B4 dws partials + pub   {db(4, 9):6.2f} us")
    print(f"B45 (all wgs)           {db(5, 4):6.2f} us")
    print(f"B5 (all wgs)            {db(6, 5):6.2f} us")


if __name__ == "__main__":
    main()
