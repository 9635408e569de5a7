"""Diagnostic: the fused producers of the persistent GRU backward (the layer above's dX as this layer's
dy) against the recurrence that consumes their slices, from in-kernel s_memrealtime stamps (100 MHz).
Run on a GPU box:  python tools/gru_prod_stamps.py [B L H]
Two encoder layers: the lower layer's BPTT launch (the last one) produces its own dy (the upper layer's dX);
S2S_GRU_LAYERS=1: the top layer's, whose dy is the decoder's dh (context term + dVh V)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
import s2s_amd  # noqa: E402
from s2s_amd import _lib  # noqa: E402

ITEMS = 32  # kProdStampItems


def main():
    B, L, H = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (32, 128, 256)
    D = 2 * H
    ndir, ntile = 2, (B + 15) // 16
    nchains, nmem_b, nmem_f = ndir * ntile, H // 16, 2 * H // 16
    gch = 8 * ((nchains + 7) // 8)
    nprod_b, nprod_f = (gch - nchains) * nmem_b, (gch - nchains) * nmem_f
    nf, nb = nchains * nmem_f, nchains * nmem_b
    sf = torch.zeros(nf * L * 8, dtype=torch.int64, device="cuda")
    sb = torch.zeros(nb * L * 8, dtype=torch.int64, device="cuda")
    pf = torch.zeros(max(nprod_f, 1) * ITEMS * 2, dtype=torch.int64, device="cuda")
    pb = torch.zeros(max(nprod_b, 1) * ITEMS * 2, dtype=torch.int64, device="cuda")
    st_fn = _lib.lib.s2s_debug_gru_stamps
    st_fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    ps_fn = _lib.lib.s2s_debug_gru_prod_stamps
    ps_fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    nl = int(os.environ.get("S2S_GRU_LAYERS", "2"))
    cfg = s2s_amd.ModelConfig(inputFrameSize=D, hiddenFrameSize=H, outputFrameSize=H, numLayers=nl)
    model = s2s_amd.ChorowskiBaseline(cfg, graph=False)
    x = torch.randn(B, L, D, device="cuda")
    lab = torch.randint(0, cfg.outputDepth, (B, 40), device="cuda", dtype=torch.int32)
    if os.environ.get("S2S_XP_SPLIT") == "0":
        _lib.lib.s2s_debug_gru_xp_split(0)
    model.step(x, lab)  # warm-up (first-launch costs)
    torch.cuda.synchronize()
    st_fn(sf.data_ptr(), sb.data_ptr())
    ps_fn(pf.data_ptr(), pb.data_ptr())
    model.step(x, lab)
    torch.cuda.synchronize()
    st_fn(None, None)
    ps_fn(None, None)
    tb = sb.cpu().numpy().reshape(nb, L, 8).astype(np.float64) * 0.01
    prod = pb.cpu().numpy().reshape(max(nprod_b, 1), ITEMS, 2).astype(np.float64) * 0.01
    tbp = tb[:, ::-1, :]  # processing order
    t0 = tbp[:, 0, 6].min()
    print(f"backward (B={B} L={L} H={H}), times in us from the first consumer workgroup's entry:")
    print(f"  consumer entry spread {tbp[:, 0, 6].max() - t0:.1f}, census done {tbp[:, 0, 7].max() - t0:.1f}, "
          f"first step starts {tbp[:, 0, 0].min() - t0:.1f} .. {tbp[:, 0, 0].max() - t0:.1f}, "
          f"last step ends {tbp[:, -1, 5].max() - t0:.1f}")
    tpt = 64 // B
    nslices = (L + tpt - 1) // tpt
    per_s = ndir * (H // 64)
    # the producers' work units (gru_persist.hip xunit / xproj_split): slice of each unit
    K = 3 * ndir * H if nl > 1 else cfg.scoreDepth
    split = os.environ.get("S2S_XP_SPLIT", "1") != "0" and (K // 32) % 16 == 0
    sA = max(1, nprod_b // (per_s * 4)) if split else 0
    sB = min(nslices, sA + max(1, nprod_b // (per_s * 2))) if split else 0
    unit_slice = [i // per_s for i in range(sA * per_s) for _ in range(4)]
    unit_slice += [sA + i // per_s for i in range((sB - sA) * per_s) for _ in range(2)]
    unit_slice += [sB + i // per_s for i in range((nslices - sB) * per_s)]
    nwork = len(unit_slice)
    print(f"  ({nl} encoder layer(s); the stamped launch is layer 1's; split start: slices < {sA} in 4 K-parts, "
          f"< {sB} in 2)")
    per = (nwork + nprod_b - 1) // nprod_b
    used = min(per, ITEMS)
    st, en = prod[:, :used, 0], prod[:, :used, 1]
    valid = en > 0
    dur = (en - st)[valid]
    print(f"  producers: {nprod_b}, {per} items each; first item start {st[:, 0].min() - t0:.1f} .. "
          f"{st[:, 0].max() - t0:.1f}, end {en[:, 0].min() - t0:.1f} .. {en[:, 0].max() - t0:.1f}; "
          f"item duration mean {dur.mean():.1f} (min {dur.min():.1f}, max {dur.max():.1f}); last item end "
          f"{en[valid].max() - t0:.1f}")
    ready = {}
    for p in range(nprod_b):
        for i in range(used):
            w = p + i * nprod_b
            if w >= nwork or en[p, i] == 0:
                continue
            sl = unit_slice[w]
            ready[sl] = max(ready.get(sl, 0.0), en[p, i] - t0)
    print("  slice: ready / consumer step start (slice 0 .. 9, 15, 31)")
    for sl in list(range(10)) + [15, 31]:
        if sl in ready and sl * tpt < L:
            print(f"    {sl:3d}: {ready[sl]:7.1f} / {tbp[:, sl * tpt, 0].min() - t0:7.1f}")


if __name__ == "__main__":
    main()
