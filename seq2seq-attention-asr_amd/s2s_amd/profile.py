"""Live per-kernel timing (HIP events inside libs2s_hip.so, s2s_prof_*) for bench.py's roofline."""
import ctypes

from ._lib import check, lib
from .nn import Context

# kernel family -> roofline it is priced against
BOUND = {"gemm_f32": "mfma", "gru_fwd_persist": "mfma", "gru_bwd_persist": "mfma"}
# the persistent recurrences that hold every CU and make up the step's critical path.  The roofline
# kernel is the one of these with the largest live time: their event brackets match rocprofv3's
# dispatch durations (within 1 %, profiles/r01), whereas a side-stream GEMM's bracket also counts
# the time it waits for CU residency behind them (117 us by events vs 90 us by rocprofv3).
CRITICAL = ("gru_bwd_persist", "gru_fwd_persist")
DECODER = ("dec_fwd_xcd", "dec_bwd_xcd")


def collect():
    buf = ctypes.create_string_buffer(1 << 16)
    check(lib.s2s_prof_collect(buf, len(buf)))
    out = {}
    for line in buf.value.decode().splitlines():
        name, n, us, flops, nbytes = line.split("\t")
        out[name] = {"launches": int(n), "total_us": float(us), "flops": float(flops), "bytes": float(nbytes)}
    return out


def profile_step(model, x, labels, stream, reps=3):
    """Eager (un-captured) training steps with event timing on; returns per-family aggregates
    averaged over `reps` steps."""
    graph_ctx = model.ctx
    # same stream layout as the timed steps (weight-gradient GEMMs on the side stream), eager so the
    # library can bracket every launch with events
    model.ctx = Context(model.device.index, graph=False, overlap=True)
    model.ctx.set_precision(getattr(model, "precision", "fp32"))
    try:
        model.step(x, labels, stream=stream)  # warm
        stream.synchronize()
        check(lib.s2s_prof_enable(1))
        collect()
        for _ in range(reps):
            model.step(x, labels, stream=stream)
        stream.synchronize()
        agg = collect()
    finally:
        lib.s2s_prof_enable(0)
        model.ctx = graph_ctx
    for v in agg.values():
        for k in ("launches", "total_us", "flops", "bytes"):
            v[k] = v[k] / reps
    return agg


def dominant_kernel_roofline(model, x, labels, stream, peak_tflops, peak_gbs):
    agg = profile_step(model, x, labels, stream)
    kernels = {k: {"launches_per_step": round(v["launches"], 2), "us_per_step": round(v["total_us"], 2),
                   "avg_us": round(v["total_us"] / max(v["launches"], 1e-9), 3)} for k, v in agg.items()}
    single = {k: v for k, v in agg.items() if not k.endswith("_steps") and v["flops"] > 0 and k not in DECODER}
    if not single:
        return None, kernels, []
    crit = {k: v for k, v in single.items() if k in CRITICAL}
    name, v = max((crit or single).items(), key=lambda kv: kv[1]["total_us"])
    avg_us = v["total_us"] / v["launches"]
    bound = BOUND.get(name, "hbm")
    if bound == "mfma":
        achieved = v["flops"] / v["launches"] / (avg_us * 1e-6) / 1e12
        peak, unit = peak_tflops, "TFLOP/s"
    else:
        achieved = v["bytes"] / v["launches"] / (avg_us * 1e-6) / 1e9
        peak, unit = peak_gbs, "GB/s"
    roof = {"kernel": name, "bound": bound, "achieved": round(achieved, 3), "peak": peak, "unit": unit,
            "frac": round(achieved / peak, 4), "traffic": None, "avg_launch_us": round(avg_us, 2),
            "selection": ("largest live time among the critical-path persistent recurrences" if crit
                          else "largest live time"),
            "algorithmic_flops_per_launch": v["flops"] / v["launches"],
            "algorithmic_bytes_per_launch": v["bytes"] / v["launches"]}
    # the decoder recurrences are latency-bound chains of hand-offs (bench.py adds the latency floor and the
    # HBM bytes the PMC counters saw).  Their attention operand stream (Vh and h rows every step) is read
    # from LDS, where the XCD-local kernels keep it resident for the whole launch, so it is reported as an
    # LDS rate and never priced against HBM.
    dec = []
    for k in DECODER:
        if k not in agg or agg[k]["launches"] <= 0 or agg[k]["bytes"] <= 0:
            continue
        d = agg[k]
        us = d["total_us"] / d["launches"]
        lds = d["bytes"] / d["launches"]
        dec.append({"kernel": k, "bound": "latency", "avg_launch_us": round(us, 2),
                    "lds_operand_stream": {"bytes_per_launch": lds, "GB_s": round(lds / (us * 1e-6) / 1e9, 1),
                                           "what": "T B L (Sc + A) 4 B per pass, read from LDS (resident Vh and "
                                                   "h rows), not HBM"},
                    "algorithmic_flops_per_launch": d["flops"] / d["launches"],
                    "tflops": round(d["flops"] / d["launches"] / (us * 1e-6) / 1e12, 3),
                    "mfma_frac": round(d["flops"] / d["launches"] / (us * 1e-6) / 1e12 / peak_tflops, 4)})
    return roof, kernels, dec
