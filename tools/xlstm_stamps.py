"""Diagnostic: per-phase latency of the XCD-local LSTM / hybrid decoder kernels (dec_xcd_lstm.inc) of the conv +
BiLSTM model (timit/timit.lua:106-155) from in-kernel s_memrealtime stamps (100 MHz).  Run on a GPU box:
python tools/xlstm_stamps.py [B L T]   (L = input frames; the decoder sees (L - 8) / 8 annotation frames)"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import s2s_amd  # noqa: E402
from s2s_amd import _lib  # noqa: E402
from xdec_stamps import report  # noqa: E402


def main():
    B, L, T = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (32, 512, 40)
    g = torch.Generator().manual_seed(3)
    x = torch.randn((B, L, 123), generator=g).cuda()
    labels = torch.randint(0, 61, (B, T), generator=g).to(torch.int32).cuda()
    model = s2s_amd.ConvBiLSTMAttentionModel(generator=torch.Generator().manual_seed(1)).cuda()
    nst = 8 * 32 * T * 16
    sf = torch.zeros(nst, dtype=torch.int64, device="cuda")
    sb = torch.zeros_like(sf)
    fn = _lib.lib.s2s_debug_dec_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    model.zeroGradParameters()
    model.step(x, labels)  # warm
    torch.cuda.synchronize()
    fn(sf.data_ptr(), sb.data_ptr())
    model.zeroGradParameters()
    model.step(x, labels)
    torch.cuda.synchronize()
    fn(None, None)
    U = (B + 7) // 8
    nch = (B + U - 1) // U
    f = sf.cpu().numpy().reshape(8 * 32, T, 16)[: nch * 32].reshape(nch, 32, T, 16).astype(np.float64)
    b = sb.cpu().numpy().reshape(8 * 32, T, 16)[: nch * 32].reshape(nch, 32, T, 16)[:, :, ::-1].astype(np.float64)
    report("LSTM decoder forward", f, 5, ["(loop)", "F1 ws", "F2 attention+hybrid", "F3 combine", "F4 gates,cell"])
    report("LSTM decoder backward", b, 6, ["(loop)", "G gate grads", "B3 dc,us'", "B4 attention+hybrid", "B45 dws",
                                           "B5 ds"])
    st = f[:, :, 1:].astype(np.float64) * 0.01
    d = lambda a, c: (st[..., a] - st[..., c]).mean()  # noqa: E731
    print(f"  F2 sub: wait ws + alpha halo {d(6, 1):6.2f} us, scores {d(7, 6):6.2f} us, softmax+context+pub {d(2, 7):6.2f} us")
    bt = b[:, :, 1:] * 0.01
    db = lambda a, c: (bt[..., a] - bt[..., c]).mean()  # noqa: E731
    print(f"  B4 sub: pre + wait dc {db(7, 2):6.2f} us, de {db(8, 7):6.2f} us, dws/dG/q {db(3, 9):6.2f} us")


if __name__ == "__main__":
    main()
