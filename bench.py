"""Throughput of the attention-seq2seq training step (forward + NLL seed + backward) on MI355X.

Metric (BASELINE.json): log-mel frames/s fwd+bwd, Chorowski TIMIT baseline; frames = N_gpu * B * L
per step.  Workload = BASELINE config 2: B=32 utterances/GPU, L=128 frames,
T=40 labels, F=123 (40 log-mel + energy, +d +dd), 3 x BiGRU(256), scoreDepth 512, GRU(256) decoder,
Maxout(768 -> 64, 7), 62 classes, fp32 (random-init weights, synthetic N(0,1) features).
Data parallel: one process per GPU, each its own B utterances (weak scaling); the flat fp32
gradient is summed over ranks with RCCL all-reduce inside the timed step (§8e).  The optimizer
step is excluded (§8d).

  python bench.py [--gpus N] [--steps K] [--warmup W]
  (N > 1: python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N)
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "seq2seq-attention-asr_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

CONFIGS = {
    # name: (model kwargs, B per GPU, L, T)
    "timit_chorowski_b32": (dict(), 32, 128, 40),
    "librispeech_chorowski_b32": (dict(inputFrameSize=80, outputDepth=29), 32, 400, 200),
    # BASELINE config 3 class: model_chorowski_baseline_dropout.lua (p = 0.5), B = 64 (bf16 hoisted GEMMs: PRECISION)
    "timit_chorowski_dropout_b64": (dict(dropout=0.5), 64, 128, 40),
    # config 2's model on TIMIT-like variable-length utterances (oracle.timit_like_lengths): length-sorted
    # minibatches of 32, each padded to its longest utterance, masked (s2s_model_dims.frame_lengths /
    # label_lengths); frames = the utterances' real frames (padding not counted).  L / T: the cap.
    "timit_ragged_b32": (dict(), 32, 264, 98),
    # BASELINE config 5 single-GPU shape: librispeech/model_vgg.lua (VGG conv stack on (B, 3, 1024, 40),
    # 1x1 layers 2048, A = 512, S = 256, Sc = 512, two-Maxout decoder_mlp, 29 chars), B = 16 per GPU
    "librispeech_vgg_b16": (dict(inputFrameSize=40, outputDepth=29), 16, 1024, 200),
}
CONFIG_DESC = {
    "timit_chorowski_b32": ("BASELINE config 2", "timit/model_chorowski_baseline.lua"),
    "librispeech_chorowski_b32": ("BASELINE config 4 shape (1 GPU)", "librispeech/model_chorowski_baseline.lua"),
    "timit_chorowski_dropout_b64": ("BASELINE config 3 (bf16)", "timit/model_chorowski_baseline_dropout.lua"),
    "timit_ragged_b32": ("BASELINE config 2 model, TIMIT-like variable lengths", "timit/model_chorowski_baseline.lua"),
    "librispeech_vgg_b16": ("BASELINE config 5 (1 GPU)", "librispeech/model_vgg.lua"),
}
# operand precision of the hoisted GEMMs per config (BASELINE.json: configs 3 and 5 are bf16 MFMA); the
# recurrences (GRU / attention steps) stay fp32 in every config
# (config 5: bf16-all = bf16 operands in every GEMM including the weight gradients, the usual bf16 mixed
# precision; at config 5 its gradient error equals bf16's -- both are set by forward decision flips,
# tests/test_gpu_bf16.py -- so nothing is gained by fp32 weight gradients there)
PRECISION = {"timit_chorowski_dropout_b64": "bf16", "librispeech_vgg_b16": "bf16-all"}


def precision_note(p, what):
    if p == "fp32":
        return "fp32 everywhere (exact f32 MFMA)"
    wg = ("weight gradients bf16 too" if p == "bf16-all" else "weight-gradient GEMMs fp32")
    return f"bf16 operands / fp32 accumulation in {what}; {wg}; recurrences fp32; fp32 master weights"
PEAK_BF16_MFMA_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense BF16 matrix peak
RAGGED_BATCHES = 8  # length-sorted minibatches cycled by the ragged workload (one captured graph each)
PEAK_FP32_MFMA_TFLOPS = 157.3   # MI355X_MICROARCH.md: F32 matrix peak (v_mfma_f32_32x32x2_f32)
PEAK_HBM_GBS = 8000.0           # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
SIMDS = 1024                    # 256 CUs x 4 SIMDs (MfmaUtil's SIMD_NUM)
HOP_US = 0.22                   # one XCD-local hand-off, measured (tools/pingpong.hip)
# hand-off seams per recurrence step of each persistent kernel: the latency floor of a
# launch is seams x steps x HOP_US -- the recurrences are chains of dependent hand-offs
SEAMS = {"gru_fwd_persist": 2, "gru_bwd_persist": 2, "dec_fwd_xcd": 5, "dec_bwd_xcd": 5}
# PMC passes (one rocprofv3 run each; MI355X_MICROARCH.md: FETCH_SIZE and WRITE_SIZE cannot share a pass)
PMC_PASSES = (("FETCH_SIZE",), ("WRITE_SIZE",),
              ("SQ_INSTS_VALU_MFMA_MOPS_F32", "SQ_INSTS_VALU_MFMA_MOPS_BF16", "SQ_VALU_MFMA_BUSY_CYCLES",
               "GRBM_GUI_ACTIVE"))


def flops_per_utterance(cfg, L, T):
    """fwd = 2 [L (P_enc + A Sc) + T P_step + T L (2 Sc + A)], fwd+bwd = 3 x fwd."""
    H = [cfg.hiddenFrameSize] * (cfg.numLayers - 1) + [cfg.outputFrameSize]
    D = [cfg.inputFrameSize] + [2 * h for h in H[:-1]]
    p_enc = sum(2 * 3 * h * (h + d) for h, d in zip(H, D))
    A, Sc, S, O, M, k = cfg.annotationDepth, cfg.scoreDepth, cfg.stateDepth, cfg.outputDepth, cfg.mlpDepth, cfg.maxoutWindow
    p_step = S * Sc + O * S + A * S + 2 * S * S + 3 * S * 2 * S + (S + A) * M * k + M * O
    fwd = 2 * (L * (p_enc + A * Sc) + T * p_step + T * L * (2 * Sc + A))
    return 3 * fwd


def cpu_worker(args):
    """One reference-semantics utterance (B=1, 2-D, fp32) through the oracle on one core."""
    seed, L, T, kw = args
    import numpy as np
    from oracle import s2s_oracle as orc
    kw = dict(kw)
    p = kw.pop("dropout", 0.0)  # the oracle takes the dropout as a mask (nn.Dropout, scaled by 1/(1-p))
    cfg = orc.ModelConfig(**kw)
    P = orc.init_params(cfg, seed=1234, dtype=np.float32)
    x, lab = orc.synthetic_batch(cfg, 1, L, T, seed=seed, dtype=np.float32)
    t = time.perf_counter()
    mask = None
    if p > 0:
        rng = np.random.default_rng(seed)
        width = cfg.stateDepth + 2 * cfg.outputFrameSize
        mask = ((rng.random((1, T, width)) >= p) / (1.0 - p)).astype(np.float32)
    orc.training_step(x, lab, P, cfg, dropout_mask=mask)
    return time.perf_counter() - t


def cpu_baseline(kw, L, T, seconds_budget):
    """CPU baseline on the host's cores (at most 16, the GPU box's share): the C restatement of the training step
    (oracle/cpu_ref.c, fp32, reference semantics -- every utterance forwarded and back-propagated alone with
    per-time-step matrix-vector products, timit/timit.lua:240-295 -- OpenMP over the minibatch's utterances);
    the NumPy restatement in one process per core when the C library is not built."""
    try:
        return cpu_baseline_c(kw, L, T, seconds_budget)
    except (OSError, FileNotFoundError):
        return cpu_baseline_numpy(kw, L, T, seconds_budget)


def cpu_baseline_c(kw, L, T, seconds_budget):
    import numpy as np
    from oracle import cpu_ref
    from oracle import s2s_oracle as orc
    cores = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    kw = dict(kw)
    p = kw.pop("dropout", 0.0)
    cfg = orc.ModelConfig(**kw)
    flat = orc.flatten(orc.init_params(cfg, seed=1234, dtype=np.float32), cfg)
    rng = np.random.default_rng(11)

    def batch(n, seed):
        x, lab = orc.synthetic_batch(cfg, n, L, T, seed=seed, dtype=np.float32)
        m = None
        if p > 0:  # nn.Dropout masks of the decoder MLP input, scaled by 1/(1-p)
            m = ((rng.random((n, T, cfg.stateDepth + cfg.annotationDepth)) >= p) / (1.0 - p)).astype(np.float32)
        return x, lab, m

    x, lab, m = batch(cores, 1)
    t = time.perf_counter()
    cpu_ref.training_step(x, lab, flat, cfg, dropout_mask=m, threads=cores)  # one utterance per thread
    t1 = time.perf_counter() - t
    rounds = max(1, int(seconds_budget / max(t1, 1e-3)))
    n = rounds * cores
    x, lab, m = batch(n, 2)
    t = time.perf_counter()
    cpu_ref.training_step(x, lab, flat, cfg, dropout_mask=m, threads=cores)
    wall = time.perf_counter() - t
    return {"value": round(n * L / wall, 1), "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"one minibatch of {n} utterances (L={L}, T={T}, fp32) of the same model, each forwarded and "
                      f"back-propagated alone (reference semantics, per-time-step matrix-vector products), "
                      f"gradients summed: oracle/cpu_ref.c (C restatement of the Torch7 path, not Torch7), "
                      f"OpenMP over the utterances on {cores} threads, {wall:.1f} s wall"}


def cpu_baseline_numpy(kw, L, T, seconds_budget):
    """CPU restatement (oracle/, numpy fp32, per-utterance like timit/timit.lua:240-295) on the host's
    cores: one single-threaded worker process per core, each running whole utterances."""
    import multiprocessing as mp
    for v in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ[v] = "1"
    cores = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    ctx = mp.get_context("spawn")
    with ctx.Pool(cores) as pool:
        pool.map(cpu_worker, [(0, 16, 4, kw)] * cores)          # warm-up (imports)
        t1 = pool.map(cpu_worker, [(1, L, T, kw)])[0]            # one utterance alone -> size the sample
        per_core = max(1, int(seconds_budget / max(t1, 1e-3)))
        n = per_core * cores
        t = time.perf_counter()
        pool.map(cpu_worker, [(i + 2, L, T, kw) for i in range(n)])
        wall = time.perf_counter() - t
    return {"value": round(n * L / wall, 1), "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"{n} utterances (L={L}, T={T}, B=1 each, fp32) of the same model, oracle/s2s_oracle.py "
                      f"(numpy restatement of the Torch7 path, not Torch7), {cores} single-threaded processes, "
                      f"{wall:.1f} s wall"}


def pmc_counters(config, precision):
    """Per-kernel PMC counters from rocprofv3, one child pass per PMC_PASSES entry (FETCH_SIZE and WRITE_SIZE
    cannot share one pass: MI355X_MICROARCH.md, rocprofv3 PMC slots) of a short eager run of this same
    workload: HBM traffic and MFMA instruction / busy counts.  Called before this process touches the GPU.
    Returns {kernel name: {counter: value per dispatch}} or None."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3")
    if not exe:
        return None
    out = {}
    for ctrs in PMC_PASSES:
        d = tempfile.mkdtemp(prefix="s2s_pmc_", dir=os.environ.get("TMPDIR", "/tmp"))
        cmd = ["timeout", "-s", "KILL", "150", exe, "--pmc", *ctrs, "--output-format", "csv", "-d", d, "-o", "pmc",
               "--", sys.executable, os.path.abspath(__file__), "--steps", "2", "--warmup", "1", "--no-cpu",
               "--no-kernel-timing", "--no-pmc", "--no-graph", "--config", config, "--precision", precision]
        try:
            subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=170, check=True)
        except Exception:
            return None
        files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not files:
            return None
        acc = {}
        for f in files:
            for r in csv.DictReader(open(f)):
                ctr = r.get("Counter_Name")
                if ctr not in ctrs:
                    continue
                a = acc.setdefault((r["Kernel_Name"], ctr), {})
                # one row per dispatch and counter (values summed over the counter's instances); keyed by
                # dispatch so a counter reported in several rows of one dispatch adds up
                key = r.get("Dispatch_Id") or len(a)
                a[key] = a.get(key, 0.0) + float(r["Counter_Value"])
        for (k, ctr), per in acc.items():
            out.setdefault(k, {})[ctr] = sum(per.values()) / len(per)
        shutil.rmtree(d, ignore_errors=True)
    return out


def mfma_of(pmc, family, avg_us):
    """MFMA evidence per launch of a kernel family: MFMA flops executed ((F32 + BF16 MOPS) x 512), MFMA-busy SIMD cycles
    and the busy fraction of the SIMDs over the dispatch (GRBM_GUI_ACTIVE / 8 = the dispatch's cycles:
    rocprofv3 sums it over the 8 XCDs, MI355X_MICROARCH.md DVFS note)."""
    if not pmc:
        return None
    family = SYMBOL.get(family, family)
    rows = [v for k, v in pmc.items() if family in k and "SQ_INSTS_VALU_MFMA_MOPS_F32" in v]
    if not rows:
        return None
    mops = sum(v["SQ_INSTS_VALU_MFMA_MOPS_F32"] for v in rows) / len(rows)
    mops16 = sum(v.get("SQ_INSTS_VALU_MFMA_MOPS_BF16", 0.0) for v in rows) / len(rows)
    busy = sum(v.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0) for v in rows) / len(rows)
    grbm = sum(v.get("GRBM_GUI_ACTIVE", 0.0) for v in rows) / len(rows)
    cycles = grbm / 8.0
    out = {"SQ_INSTS_VALU_MFMA_MOPS_F32": round(mops), "SQ_INSTS_VALU_MFMA_MOPS_BF16": round(mops16),
           "mfma_flops_per_launch": round(512.0 * (mops + mops16)),
           "SQ_VALU_MFMA_BUSY_CYCLES": round(busy), "GRBM_GUI_ACTIVE": round(grbm),
           "mfma_busy_frac": round(busy / (cycles * SIMDS), 4) if cycles > 0 else None,
           "clock_GHz_from_GRBM": round(cycles / (avg_us * 1e3), 3) if avg_us else None,
           "source": "rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_INSTS_VALU_MFMA_MOPS_BF16 "
                     "SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE, eager run"}
    return out


def latency_floor(name, steps, avg_us):
    """The hand-off chain a persistent recurrence cannot beat: seams per step x steps x one measured hop."""
    seams = SEAMS.get(name)
    if not seams or not avg_us:
        return None
    floor = seams * steps * HOP_US
    return {"seams_per_step": seams, "steps": steps, "hop_us": HOP_US, "floor_us": round(floor, 1),
            "frac": round(floor / avg_us, 4),
            "what": "seams x steps x one XCD-local hand-off (tools/pingpong.hip); the compute inside each seam "
                    "is on top of it"}


# live-timing family -> the kernel symbol rocprofv3 reports
SYMBOL = {"dec_fwd_xcd": "dec_xcd_fwd", "dec_bwd_xcd": "dec_xcd_bwd"}
SYMBOL_VGG = {"gemm_bf16": "gemm_bf16_kernel", "gemm_big_bf16": "gemm_bf16_nt", "conv_fwd_bf16": "conv_bf16_kernel<false",
              "conv_dx_bf16": "conv_bf16_kernel<true", "conv_wgrad_bf16": "conv_wgrad_bf16_kernel"}


def traffic_of(pmc, family):
    """HBM bytes per launch of a kernel family: (2 * FETCH_SIZE + WRITE_SIZE) KB -- on gfx950 FETCH_SIZE
    counts half the bytes of 16-B-per-lane reads (cdna_hip_programming.md section 7, MI355X_MICROARCH.md
    HBM), so the read side is doubled."""
    if not pmc:
        return None, None
    family = SYMBOL.get(family, family)
    rows = [v for k, v in pmc.items() if family in k and "FETCH_SIZE" in v and "WRITE_SIZE" in v]
    if not rows:
        return None, None
    fetch = sum(v["FETCH_SIZE"] for v in rows) / len(rows)
    write = sum(v["WRITE_SIZE"] for v in rows) / len(rows)
    return (2.0 * fetch + write) * 1024.0, {"FETCH_SIZE_KB": round(fetch, 1), "WRITE_SIZE_KB": round(write, 1),
                                            "formula": "(2*FETCH_SIZE + WRITE_SIZE) KiB per launch",
                                            "source": "rocprofv3 --pmc, 2 passes, eager run"}


def cpu_vgg_baseline(L, T, seconds_budget):
    """CPU restatement of librispeech/model_vgg.lua (oracle/frontend_oracle.py, numpy fp32) on the host:
    one process, BLAS threads on every core, whole utterances (B = 1, the reference's per-utterance loop)."""
    import numpy as np
    cores = max(1, min(16, len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else os.cpu_count()))
    from oracle import frontend_oracle as fo
    P, layers, cfg = fo.vgg_random_case(seed=1234)
    rng = np.random.default_rng(5)
    n, t0 = 0, time.perf_counter()
    while True:
        x = rng.standard_normal((1, 3, L, 40)).astype(np.float32)
        lab = rng.integers(0, cfg.outputDepth - 1, (1, T)).astype(np.int32)
        fo.vgg_model_step(x, lab, P, layers, cfg)
        n += 1
        wall = time.perf_counter() - t0
        if wall >= seconds_budget:
            break
    return {"value": round(n * L / wall, 1), "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"{n} utterances (3 x {L} x 40 log-mel planes, T={T}, B=1 each, fp32) of librispeech/model_vgg.lua, "
                      f"oracle/frontend_oracle.py (numpy restatement, not Torch7), one process, BLAS on {cores} "
                      f"threads, {wall:.1f} s wall"}


def run_vgg(args, pmc, rank, world, torch, dist, s2s_amd, s2s_dist):
    """BASELINE config 5: librispeech/model_vgg.lua training step (VGG encoder -> attention decoder with the
    two-Maxout decoder_mlp -> loss seed -> backward), B = 16 utterances of 1024 frames per GPU, the whole
    step (gradient zeroing included) replayed from one captured HIP graph (VGGAttentionModel.graph_step;
    --no-graph: eager launches of the host-side Sequential), all-reduce of every gradient when N > 1."""
    kw, B, L, T = CONFIGS[args.config]
    g = torch.Generator().manual_seed(1234 + rank)
    model = s2s_amd.VGGAttentionModel(kw["inputFrameSize"], outputFrameSize=512, hidden=2048,
                                      outputDepth=kw["outputDepth"], generator=torch.Generator().manual_seed(1234),
                                      precision=args.precision).cuda()
    x = torch.randn((B, 3, L, kw["inputFrameSize"]), generator=g).cuda()
    labels = torch.randint(0, kw["outputDepth"] - 1, (B, T), generator=g)
    labels[:, -1] = kw["outputDepth"] - 1
    labels = labels.to(torch.int32).cuda()
    grads = model.parameters()[1]

    def step():
        if args.no_graph:
            model.zeroGradParameters()
            model.step(x, labels)
        else:
            model.graph_step(x, labels)
        if world > 1:  # one flat all-reduce per gradient tensor list (RCCL)
            for gt in grads:
                dist.all_reduce(gt)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = 1000.0 * elapsed / args.steps
    value = world * B * L / (ms / 1000.0)
    out = {"metric": "log-mel frames/sec fwd+bwd, librispeech/model_vgg.lua",
           "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
           "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
           "dtype": "fp32" if args.precision == "fp32" else "bf16", "precision": args.precision,
           "precision_note": precision_note(args.precision, "the VGG convolutions (implicit GEMM), 1x1 layers, Vh, "
                                            "decoder MLP and data-gradient GEMMs"),
           "data": "synthetic (N(0,1) 3-plane log-mel-shaped input, uniform char labels, random-init weights)",
           "config": {"workload": f"{CONFIG_DESC[args.config][0]}: {args.config}", "model": CONFIG_DESC[args.config][1],
                      "global_batch": B * world, "utterances_per_gpu": B, "seq_len": L, "label_len": T,
                      "feat_dim": kw["inputFrameSize"], "annotation_frames": (L - 8) // 2,
                      "parallelism": f"dp{world}", "launch": "eager" if args.no_graph else "hipGraph replay"}}
    if rank == 0 and not args.no_kernel_timing:
        from s2s_amd import _lib
        from s2s_amd import profile as s2s_profile
        _lib.check(_lib.lib.s2s_prof_enable(1))
        s2s_profile.collect()
        # the profiled steps keep the parameter gradients on the call's stream (model.overlap off): the timed steps run
        # them beside the next module's backward, where a launch's events would also time the kernels beside it
        overlap, model.overlap = model.overlap, False
        for _ in range(2):  # eager: the library brackets each launch with events
            model.zeroGradParameters()
            model.step(x, labels)
        torch.cuda.synchronize()
        model.overlap = overlap
        agg = s2s_profile.collect()
        _lib.lib.s2s_prof_enable(0)
        bf16 = args.precision != "fp32"
        out["kernels"] = {k: {"launches_per_step": v["launches"] / 2, "us_per_step": round(v["total_us"] / 2, 1)}
                          for k, v in agg.items()}
        # the MFMA-bound families of the step (the decoder recurrences beside them are latency-bound): the
        # 64 x 64 tile GEMM, the big-tile GEMM of the 1x1 layers / decoder products and the implicit convolutions
        fams = (("gemm_bf16", "gemm_big_bf16", "conv_fwd_bf16", "conv_dx_bf16", "conv_wgrad_bf16") if bf16
                else ("gemm_f32",))
        peak = PEAK_BF16_MFMA_TFLOPS if bf16 else PEAK_FP32_MFMA_TFLOPS
        rows = []
        for fam in fams:
            if fam not in agg or agg[fam]["launches"] <= 0:
                continue
            v = agg[fam]
            avg = v["total_us"] / v["launches"]
            ach = v["flops"] / v["launches"] / (avg * 1e-6) / 1e12
            rows.append({"kernel": fam, "bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
                         "frac": round(ach / peak, 4), "avg_launch_us": round(avg, 2),
                         "launches_per_step": v["launches"] / 2, "us_per_step": round(v["total_us"] / 2, 1)})
        if rows:
            r = dict(max(rows, key=lambda e: e["us_per_step"]))
            t, detail = traffic_of(pmc, SYMBOL_VGG.get(r["kernel"], r["kernel"]))
            r.update({"traffic": round(t) if t is not None else None, "traffic_detail": detail,
                      "selection": "the MFMA-bound family with the largest live time (the others in mfma_families); "
                                   "live times from eager profiled steps with the parameter gradients serial",
                      "mfma_counters": mfma_of(pmc, SYMBOL_VGG.get(r["kernel"], r["kernel"]), r["avg_launch_us"])})
            out["roofline"] = r
            out["mfma_families"] = rows
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_vgg_baseline(L, T, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="timit_chorowski_b32", choices=sorted(CONFIGS))
    ap.add_argument("--no-graph", action="store_true", help="eager launches instead of hipGraph replay")
    ap.add_argument("--no-overlap", action="store_true",
                    help="weight-gradient GEMMs on the main stream (default: S2S_CTX_OVERLAP, a side stream "
                         "beside the next layer's BPTT)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-kernel-timing", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    ap.add_argument("--precision", choices=("auto", "fp32", "bf16", "bf16-all"), default="auto",
                    help="operand precision of the hoisted GEMMs (auto: BASELINE's per config)")
    ap.add_argument("--flat-allreduce", action="store_true",
                    help="N>1: one all-reduce of the whole gradient after the step instead of the bucketed, "
                         "overlapped one")
    args = ap.parse_args()
    if args.precision == "auto":
        args.precision = PRECISION.get(args.config, "fp32")

    world0 = int(os.environ.get("WORLD_SIZE", "1"))
    pmc = None
    if world0 == 1 and not args.no_pmc and not args.no_kernel_timing:
        pmc = pmc_counters(args.config, args.precision)  # child processes, before this one initialises the GPU

    import torch
    import torch.distributed as dist

    import s2s_amd
    from s2s_amd import dist as s2s_dist
    from s2s_amd import profile as s2s_profile

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    kw, B, L, T = CONFIGS[args.config]
    if args.config == "librispeech_vgg_b16":
        return run_vgg(args, pmc, rank, world, torch, dist, s2s_amd, s2s_dist)
    cfg = s2s_amd.ModelConfig(**kw)
    model = s2s_amd.ChorowskiBaseline(cfg, graph=not args.no_graph, seed=1234,
                                     overlap=not args.no_overlap, precision=args.precision)
    g = torch.Generator(device="cpu").manual_seed(1234 + rank)
    eos = 23 if cfg.outputDepth > 23 else cfg.outputDepth - 1

    def make_batch(nb, Lb, Tb, flen=None, tlen=None):
        x = torch.randn((nb, Lb, cfg.inputFrameSize), generator=g)
        labels = torch.randint(0, cfg.outputDepth - 1, (nb, Tb), generator=g)
        labels[labels >= eos] += 1
        flen = flen if flen is not None else [Lb] * nb
        tlen = tlen if tlen is not None else [Tb] * nb
        for b in range(nb):  # 10 zero frames each side of the utterance, EOS last
            x[b, :10] = 0
            x[b, max(10, flen[b] - 10):flen[b]] = 0
            labels[b, tlen[b] - 1] = eos
        return x.cuda(), labels.to(torch.int32).cuda()

    ragged = args.config == "timit_ragged_b32"
    if ragged:
        # RAGGED_BATCHES length-sorted minibatches of B TIMIT-like utterances (oracle.timit_like_lengths's
        # distribution, restated here so the bench does not import the oracle)
        import numpy as np
        rs = np.random.default_rng(77 + rank)
        dur = np.clip(rs.normal(3.1, 0.9, B * RAGGED_BATCHES), 1.0, 7.8)
        fl = np.minimum(np.rint(dur * 16000 / 512).astype(int) + 20, L)
        tl = np.minimum(np.maximum(np.rint(dur * 12.3).astype(int), 1) + 1, T)
        order = np.argsort(fl, kind="stable")
        batches = []
        for i in range(RAGGED_BATCHES):
            idx = order[i * B:(i + 1) * B]
            flen, tlen = fl[idx].tolist(), tl[idx].tolist()
            xb, lb = make_batch(B, max(flen), max(tlen), flen, tlen)
            batches.append((xb, lb, flen, tlen))
        args.warmup = max(args.warmup, RAGGED_BATCHES)  # one capture per batch shape, outside the timing
    else:
        x, labels = make_batch(B, L, T)
    stream = torch.cuda.Stream()
    scale = s2s_dist.step_scale(B)
    real_frames = [0]

    comm = torch.cuda.Stream()
    buckets = model.grad_buckets()
    bucketed = world > 1 and not args.flat_allreduce

    it = [0]

    def step():
        if ragged:
            xb, lb, flen, tlen = batches[it[0] % RAGGED_BATCHES]
            it[0] += 1
            real_frames[0] += sum(flen)
            model.step(xb, lb, scale=scale, stream=stream, bucket_events=bucketed, frame_lengths=flen,
                       label_lengths=tlen)
        else:
            real_frames[0] += B * L
            model.step(x, labels, scale=scale, stream=stream, bucket_events=bucketed)
        if bucketed:
            # per-bucket RCCL all-reduce issued as each bucket's gradients become final (decoder,
            # then encoder layers top-down), overlapping the BPTT of the layers below
            s2s_dist.allreduce_buckets(model.grads, buckets, wait=model.wait_bucket, comm_stream=comm)
        elif world > 1:
            s2s_dist.allreduce_gradients(model.grads)

    with torch.cuda.stream(stream):
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        real_frames[0] = 0
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    # a persistent launch that timed out would have produced invalid gradients: fail instead of reporting
    model.ctx.check_status(stream)
    if world > 1:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    ms = 1000.0 * elapsed / args.steps
    # the optimizer (timit.lua:292-347: clip, adadelta, column-norm constraint) is outside t_step
    #  and reported on its own: device step on the flat buffers, HBM-bound
    opt = s2s_amd.optim.Adadelta(model, rho=0.95, eps=1e-8, colnormconstr=True)
    flag = torch.zeros(1, dtype=torch.float32, device="cuda")

    def opt_step():
        # data parallel: a failed persistent launch on ANY rank skips the update on every rank (the failure flag's MAX
        # over the ranks, s2s_amd.dist.reduce_failure_flag), or the replicas diverge; one rank: the plain update
        if world > 1:
            opt.failure_flag(stream, out=flag)
            s2s_dist.reduce_failure_flag(flag)
            opt.step(stream, skip_flag=flag)
        else:
            opt.step(stream)

    with torch.cuda.stream(stream):
        for _ in range(3):
            opt_step()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(20):
            opt_step()
        e1.record(stream)
    torch.cuda.synchronize()
    opt_us = 1000.0 * e0.elapsed_time(e1) / 20
    frames_per_step = world * real_frames[0] / args.steps  # every rank runs the same batch schedule
    value = frames_per_step / (ms / 1000.0)

    if ragged:  # algorithmic flops of the real (unpadded) utterances
        flop_step = sum(flops_per_utterance(cfg, f, t) for _, _, fls, tls in batches for f, t in zip(fls, tls))
        flop_step /= RAGGED_BATCHES
    else:
        flop_step = flops_per_utterance(cfg, L, T) * B
    out = {
        "metric": "log-mel frames/sec fwd+bwd, Chorowski TIMIT baseline",
        "value": round(value, 1), "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
        "dtype": "fp32" if args.precision == "fp32" else "bf16", "precision": args.precision,
        "precision_note": precision_note(args.precision, "the hoisted GEMMs (x-projections, Vh, MLP, dX)"),
        "data": "synthetic (N(0,1) log-mel-shaped features, uniform labels, random-init weights)",
        "config": {"workload": f"{CONFIG_DESC[args.config][0]}: {args.config}", "model": CONFIG_DESC[args.config][1],
                   "global_batch": B * world, "utterances_per_gpu": B, "seq_len": L, "label_len": T,
                   "feat_dim": cfg.inputFrameSize, "parallelism": f"dp{world}",
                   "allreduce": ("none" if world == 1 else "flat RCCL after the step" if not bucketed
                                 else f"{len(buckets)} RCCL buckets overlapped with encoder BPTT"),
                   "launch": "eager" if args.no_graph else "hipGraph replay",
                   "flop_per_step_per_gpu": flop_step},
        "step_tflops_per_gpu": round(flop_step / (ms / 1000.0) / 1e12, 3),
        "optimizer": {"us_per_step": round(opt_us, 2), "what": "adadelta (rho .95, eps 1e-8) + global-norm clip + "
                      "column-norm constraint on the flat buffers (s2s_optim_adadelta_step), not in ms_per_step; N > 1: "
                      "behind the failure flag's MAX over the ranks (skipped on every rank if any rank's step failed)"},
    }
    if ragged:
        out["config"]["ragged"] = {
            "batches": RAGGED_BATCHES, "utterances": B * RAGGED_BATCHES,
            "mean_frames": round(sum(sum(b[2]) for b in batches) / (B * RAGGED_BATCHES), 1),
            "padded_frames_per_step": sum(len(b[2]) * max(b[2]) for b in batches) / RAGGED_BATCHES,
            "lengths": "TIMIT-like: dur ~ N(3.1 s, 0.9 s) in [1, 7.8] s, hop 512 @ 16 kHz + 20 pad frames, "
                       "12.3 phones/s + EOS; length-sorted batches, padded + masked; value counts real frames"}
        x, labels = batches[RAGGED_BATCHES // 2][:2]  # the profiled steps (unmasked, median batch)
    # the profiled launches' own shape (the ragged line profiles its median batch, padded to that batch's longest
    # utterance: its L / T, not the workload's caps, price the rec_frac and the latency floors)
    Lp, Tp = int(x.shape[1]), int(labels.shape[1])
    if ragged:
        out["config"]["ragged"]["profiled_batch"] = {"L": Lp, "T": Tp, "what": "the median batch, padded, unmasked"}
    if rank == 0 and not args.no_kernel_timing:
        with torch.cuda.stream(stream):
            out["roofline"], out["kernels"], dec = s2s_profile.dominant_kernel_roofline(
                model, x, labels, stream, PEAK_FP32_MFMA_TFLOPS, PEAK_HBM_GBS)
        if out["roofline"]:
            r = out["roofline"]
            t, detail = traffic_of(pmc, r["kernel"])
            r["traffic"] = round(t) if t is not None else None
            r["traffic_detail"] = detail
            r["mfma_counters"] = mfma_of(pmc, r["kernel"], r["avg_launch_us"])
            r["latency_floor"] = latency_floor(r["kernel"], Lp, r["avg_launch_us"])
            if r["kernel"].startswith("gru_"):
                r["work"] = ("the launch's algorithmic flops: the recurrence (2 B L 3H^2 per direction) plus the "
                             "GEMM its spare-slot producers compute inside the launch (forward: the x-projection; "
                             "backward: dy = the layer above's dX, or for the top layer the decoder's dh = "
                             "dVh V + sum_t alpha dc), averaged over the step's launches")
                # the recurrence alone (what the persistent kernel exists for), priced the same way: rec_frac
                Hs = [cfg.hiddenFrameSize] * (cfg.numLayers - 1) + [cfg.outputFrameSize]
                rec = sum(2.0 * 2 * B * Lp * 3.0 * h * h for h in Hs) / len(Hs)
                rec_ach = rec / (r["avg_launch_us"] * 1e-6) / 1e12
                r["rec_flops_per_launch"] = rec
                r["rec_achieved"] = round(rec_ach, 3)
                r["rec_frac"] = round(rec_ach / r["peak"], 4)
                r["rec_what"] = ("the recurrence alone: 2 directions x 2 B L 3H^2 per launch (no in-launch GEMM) / the "
                                 "same live launch time, against the same fp32 MFMA peak")
        # the decoder recurrences (the attention path): priced against their own hand-off latency floor; the
        # HBM rate is the counters' bytes (the attention operands themselves stay in LDS, profile.py)
        out["roofline_decoder"] = []
        for e in dec:
            t, detail = traffic_of(pmc, e["kernel"])
            e["traffic"] = round(t) if t is not None else None
            e["traffic_detail"] = detail
            if t is not None:
                gbs = t / (e["avg_launch_us"] * 1e-6) / 1e9
                e["hbm"] = {"achieved": round(gbs, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
                            "frac": round(gbs / PEAK_HBM_GBS, 4), "source": "PMC traffic / live launch time"}
            e["mfma_counters"] = mfma_of(pmc, e["kernel"], e["avg_launch_us"])
            e["latency_floor"] = latency_floor(e["kernel"], Tp, e["avg_launch_us"])
            out["roofline_decoder"].append(e)
    if rank == 0 and world == 1 and not args.no_cpu:
        out["cpu_baseline"] = cpu_baseline(kw, L, T, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
