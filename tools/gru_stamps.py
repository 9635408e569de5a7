"""Diagnostic: hand-off vs compute latency inside the persistent GRU layer kernels, from in-kernel
s_memrealtime stamps (100 MHz).  Run on a GPU box:  python tools/gru_stamps.py [B L H]

Per step of one chain (direction, 16-row tile):
  forward   h_{t-1} -> [z|r] (p1, 2H/16 workgroups)  ->  q = r*h -> hh, h_t (p2, H/16 workgroups)
  backward  da_h -> dq, da_r (p1, H/16)  ->  [da_z; da_r] -> dh_{t-1}, gates (p2, H/16)
hand-off = consumer sweep done - last producer's phase end; compute = phase end - sweep done.
S2S_GRU_DIAG=1 with a diagnostic build (tools/ab_variant.sh diag "-DS2S_GRU_DIAG=1", S2S_HIP_LIB=...): 16 stamp slots;
each seam is split into the producers' publication skew, the consumers' poll passes and the sweep of data that is
already there (the backward's da_z sweep)."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
import s2s_amd  # noqa: E402
from s2s_amd import _lib  # noqa: E402


def analyse(name, st, nwg, ndir, ntile, prod1, cons1, prod2, cons2):
    """st: (grid, L, 8) stamps in us; prodX / consX: workgroup offsets within a chain."""
    L = st.shape[1]
    rows = []
    for d in range(ndir):
        for m in range(ntile):
            base = d * nwg + m * (nwg // ntile)
            c = st[base:base + nwg // ntile]
            for s in range(2, L):
                h1 = c[cons1, s, 1].mean() - c[prod1, s - 1, 5].max()
                k1 = c[prod2, s, 2].max() - c[cons1, s, 1].mean()
                h2 = c[cons2, s, 4].mean() - c[prod2, s, 2].max()
                k2 = c[prod1, s, 5].max() - c[cons2, s, 4].mean()
                per = c[prod1, s, 5].max() - c[prod1, s - 1, 5].max()
                rows.append((per, h1, k1, h2, k2))
    r = np.array(rows).mean(0)
    print(f"{name}: step {r[0]:.2f} us = hand-off1 {r[1]:.2f} + compute1 {r[2]:.2f} + hand-off2 {r[3]:.2f} "
          f"+ compute2 {r[4]:.2f}")


def seams(name, st, nwg, ndir, ntile, specs):
    """specs: (label, producers, producer stamp slot, producer step offset, consumers, start slot, done slot,
    polls slot).  Per seam and step: producers' publication spread (last - first), consumer start relative to
    the last publication (negative: the consumer was already polling), done - last publication, poll passes."""
    L = st.shape[1]
    for label, prod, pslot, poff, cons, s0, s1, pc in specs:
        sk, st0, dn, pol, sw = [], [], [], [], []
        for d in range(ndir):
            for m in range(ntile):
                base = d * nwg + m * (nwg // ntile)
                c = st[base:base + nwg // ntile]
                for s in range(2, L):
                    pub = c[prod, s + poff, pslot]
                    last, first = pub.max(), pub.min()
                    sk.append(last - first)
                    st0.append(c[cons, s, s0].mean() - last)
                    dn.append(c[cons, s, s1].mean() - last)
                    sw.append(c[cons, s, s1].mean() - c[cons, s, s0].mean())
                    pol.append(c[cons, s, pc].mean() * 100.0)  # stamps were scaled by 0.01
        print(f"  {name} {label}: publication spread {np.mean(sk):.2f} us; consumers start {np.mean(st0):+.2f} us "
              f"from the last publication, done {np.mean(dn):+.2f} us after it (sweep {np.mean(sw):.2f} us, "
              f"{np.mean(pol):.1f} poll passes)")


def main():
    B, L, H = (int(a) for a in sys.argv[1:4]) if len(sys.argv) > 3 else (32, 128, 256)
    # S2S_GRU_LAYERS=2: the stamped backward is the lower layer's, whose dy (the upper layer's dX) the
    # BPTT launch produces itself (fused dy)
    nl = int(os.environ.get("S2S_GRU_LAYERS", "1"))
    D = 2 * H
    ndir = 2
    ntile = (B + 15) // 16
    nf, nb = ndir * (2 * H // 16) * ntile, ndir * (H // 16) * ntile
    K = 16 if os.environ.get("S2S_GRU_DIAG") == "1" else 8
    sf = torch.zeros(nf * L * K, dtype=torch.int64, device="cuda")
    sb = torch.zeros(nb * L * K, dtype=torch.int64, device="cuda")
    fn = _lib.lib.s2s_debug_gru_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    x = torch.randn(B, L, D, device="cuda")
    cfg = s2s_amd.ModelConfig(inputFrameSize=D, hiddenFrameSize=H, outputFrameSize=H, numLayers=nl)
    model = s2s_amd.ChorowskiBaseline(cfg, graph=False)
    lab = torch.randint(0, cfg.outputDepth, (B, 8), device="cuda", dtype=torch.int32)
    if os.environ.get("S2S_GRU_FUSED") == "0":  # separate x-projection / dX GEMMs (A/B)
        _lib.lib.s2s_debug_gru_fused_xproj(0)
    if os.environ.get("S2S_GRU_LOCAL") == "0":  # force the tagged-granule hand-offs (A/B)
        _lib.lib.s2s_debug_gru_local(0)
    fn(sf.data_ptr(), sb.data_ptr())
    model.step(x, lab)
    torch.cuda.synchronize()
    fn(None, None)
    tf = sf.cpu().numpy().reshape(nf, L, K).astype(np.float64) * 0.01
    tb = sb.cpu().numpy().reshape(nb, L, K).astype(np.float64) * 0.01
    z = list(range(H // 16))
    zr = list(range(2 * H // 16))
    r = list(range(H // 16, 2 * H // 16))
    analyse("gru forward ", tf, nf // ndir, ndir, ntile, prod1=z, cons1=zr, prod2=r, cons2=z)
    t = tf[:, 2:]  # per-workgroup means of the forward p1 sub-phases
    print(f"  p1 per workgroup: MFMA {(t[..., 6] - t[..., 1]).mean():.2f}  reduce {(t[..., 7] - t[..., 6]).mean():.2f}"
          f"  gate + publish {(t[..., 2] - t[..., 7]).mean():.2f} us")
    # backward stamps are indexed by time step s (processed L-1 .. 0): flip to processing order
    tbp = tb[:, ::-1, :].copy()
    allc = list(range(H // 16))
    analyse("gru backward", tbp, nb // ndir, ndir, ntile, prod1=allc, cons1=allc, prod2=allc, cons2=allc)
    t0 = tbp[:, 0, 0].min()
    ends = tbp[:, :, 5].max(0)  # per processing step: the last workgroup's end
    per = np.diff(ends)
    q = len(per) // 4
    print("  backward step time by quarter of the sweep: " + ", ".join(f"{per[i * q:(i + 1) * q].mean():.2f}"
                                                                    for i in range(4)) + " us")
    print(f"  backward: first step starts at +0, step 8 at {tbp[:, 8, 0].mean() - t0:.1f} us, last step ends at "
          f"{tbp[:, -1, 5].max() - t0:.1f} us")
    if K == 16:
        print("seam decomposition (diagnostic build):")
        seams("forward", tf, nf // ndir, ndir, ntile, [
            ("h   -> [z|r]", z, 5, -1, zr, 0, 1, 8),
            ("q   -> hh   ", r, 2, 0, z, 3, 4, 9)])
        seams("backward", tbp, nb // ndir, ndir, ntile, [
            ("da_h -> dq  ", allc, 5, -1, allc, 0, 1, 8),
            ("da_z (ready)", allc, 5, -1, allc, 3, 10, 9),
            ("da_r -> dh  ", allc, 2, 0, allc, 10, 4, 11)])


if __name__ == "__main__":
    main()
