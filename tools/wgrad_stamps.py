"""Diagnostic: the first encoder layer's BPTT with its in-launch weight-gradient workers (S2S_BPTT_WGRAD=1,
gru_persist.hip bptt_wgrad) -- chain steps (member stamps) against the workers' progress (worker stamps), from
s_memrealtime (100 MHz).  Run on a GPU box:  S2S_BPTT_WGRAD=1 python tools/wgrad_stamps.py [B]"""
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
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 32
    L, H = 128, 256
    cfg = s2s_amd.ModelConfig()
    ndir, MT = 2, (B + 15) // 16
    nch, nmem, nw = ndir * MT, H // 16, 3 * H // 64
    model = s2s_amd.ChorowskiBaseline(cfg, graph=False)
    x = torch.randn(B, L, cfg.inputFrameSize, device="cuda")
    lab = torch.randint(0, cfg.outputDepth, (B, 40), device="cuda", dtype=torch.int32)
    sb = torch.zeros(nch * nmem * L * 8, dtype=torch.int64, device="cuda")
    sw = torch.zeros(nch * nw * (L + 4), dtype=torch.int64, device="cuda")
    st_fn = _lib.lib.s2s_debug_gru_stamps
    st_fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    ws_fn = _lib.lib.s2s_debug_gru_wg_stamps
    ws_fn.argtypes = [ctypes.c_void_p]
    model.step(x, lab)
    torch.cuda.synchronize()
    st_fn(None, sb.data_ptr())
    ws_fn(sw.data_ptr())
    model.step(x, lab)  # the stamps keep the last BPTT launch's: layer 1's
    torch.cuda.synchronize()
    st_fn(None, None)
    ws_fn(None)
    tb = sb.cpu().numpy().reshape(nch * nmem, L, 8).astype(np.float64) * 0.01
    tw = sw.cpu().numpy().reshape(nch, nw, L + 4).astype(np.float64) * 0.01
    tbp = tb[:, ::-1, :]  # processing order
    t0 = tbp[:, 0, 6].min()
    if not (tw > 0).any():
        print("no worker stamps (S2S_BPTT_WGRAD=0 or the shape does not fit the workers)")
    print(f"B={B}: chain entry {tbp[:, 0, 6].max() - t0:.1f}, first step starts {tbp[:, 0, 0].min() - t0:.1f}, "
          f"last step ends {tbp[:, -1, 5].max() - t0:.1f} us; step {np.diff(tbp[:, :, 5].max(0)).mean():.2f} us")
    for c in range(nch):
        e = tw[c, :, 0] - t0
        cen = tw[c, :, 1] - t0
        steps = tw[c, :, 2:L + 2] - t0
        print(f" chain {c}: workers entry {e.min():.1f}..{e.max():.1f}, census {cen.min():.1f}..{cen.max():.1f}, "
              f"step 0 done {steps[:, 0].min():.1f}..{steps[:, 0].max():.1f}, step {L // 2} "
              f"{steps[:, L // 2].min():.1f}..{steps[:, L // 2].max():.1f}, last {steps[:, -1].min():.1f}.."
              f"{steps[:, -1].max():.1f}, loop end {tw[c, :, L + 2].max() - t0:.1f}")
    ch_end = tbp[:, :, 5].max(0) - t0  # chain's step p end (max over members)
    lag = steps.max(0) - ch_end
    print(" worker lag behind the chain (last chain's workers, us) at steps 0, 16, 32, 64, 96, 127:",
          [round(lag[i], 1) for i in (0, 16, 32, 64, 96, L - 1)])
    dur = np.diff(tw[:, :, 2:L + 2], axis=2)
    print(f" worker per-step time: median {np.median(dur):.2f} us, p90 {np.percentile(dur, 90):.2f}")


if __name__ == "__main__":
    main()
