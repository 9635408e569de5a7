"""GPU: the bf16-operand MFMA GEMMs (S2S_PREC_BF16_GEMM, BASELINE configs 3 and 5).

Two kinds of checks:
* exactness of the kernel: every transpose form, guarded and unguarded tiles, split-K, against numpy
  on the SAME bf16-rounded operands (round-to-nearest-even, what v_cvt_pk_bf16_f32 does) accumulated in
  float64 -- only the fp32 accumulation order differs: max|gpu - ref| <= 2e-5 max|ref|;
* the accuracy bf16 buys at model level, against the float64 oracle (tests below state their bars).
"""
import ctypes

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def lib():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from s2s_amd import _lib
    fn = _lib.lib.s2s_debug_gemm
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float,
                   ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p, ctypes.c_long, ctypes.c_float, ctypes.c_void_p,
                   ctypes.c_long, ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
    return _lib


def bf16_round(a):
    """float32 -> nearest bf16 (ties to even), returned as float64."""
    u = np.ascontiguousarray(a, dtype=np.float32).view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    return r.astype(np.uint32).view(np.float32).astype(np.float64)


@pytest.mark.parametrize("tA,tB", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K", [(256, 384, 512), (77, 45, 133), (64, 64, 8192), (1000, 2048, 96), (64, 40000, 576)])
def test_bf16_gemm_exact_on_rounded_operands(lib, tA, tB, M, N, K):
    rng = np.random.default_rng(M + N + K + 7 * tA + 3 * tB)
    A = rng.standard_normal((K, M) if tA else (M, K)).astype(np.float32)
    B = rng.standard_normal((N, K) if tB else (K, N)).astype(np.float32)
    C0 = rng.standard_normal((M, N)).astype(np.float32)
    Ag, Bg, Cg = (torch.tensor(v, device="cuda") for v in (A, B, C0))
    ws = torch.empty(8 << 20, device="cuda")
    rc = lib.lib.s2s_debug_gemm(tA, tB, M, N, K, 0.5, Ag.data_ptr(), A.shape[1], Bg.data_ptr(), B.shape[1], 0.25,
                                Cg.data_ptr(), N, 1, ws.data_ptr(), ws.numel())
    assert rc == 0
    torch.cuda.synchronize()
    Ar, Br = bf16_round(A), bf16_round(B)
    ref = 0.5 * ((Ar.T if tA else Ar) @ (Br.T if tB else Br)) + 0.25 * C0.astype(np.float64)
    err = np.abs(Cg.cpu().numpy() - ref).max() / np.abs(ref).max()
    assert err <= 2e-5, err
    # and it is really bf16: the fp32 product differs from the rounded-operand one by far more
    exact = 0.5 * ((A.T if tA else A).astype(np.float64) @ (B.T if tB else B).astype(np.float64)) + 0.25 * C0
    assert np.abs(ref - exact).max() / np.abs(exact).max() > 1e-4


def _big_run(lib):
    fn = lib.lib.s2s_debug_gemm_big_run
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_void_p] + [ctypes.c_int] * 5 + [ctypes.c_float, ctypes.c_void_p, ctypes.c_long,
                   ctypes.c_void_p, ctypes.c_long, ctypes.c_float, ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p,
                   ctypes.c_int, ctypes.POINTER(ctypes.c_int)]
    return fn


@pytest.mark.parametrize("tA,tB", [(0, 0), (0, 1), (1, 0), (1, 1)])
@pytest.mark.parametrize("M,N,K,bias,relu,beta", [(2000, 4096, 96, True, True, 0.0),     # 256 x 256 tiles, ragged M and K
                                                  (300, 200, 1030, False, False, 0.25),  # 128 x 128, split-K, ragged K
                                                  (2048, 512, 8128, False, False, 1.0),  # weight-gradient shape, split-K
                                                  (77, 70, 133, True, False, 0.5)])      # small, every edge ragged
def test_big_bf16_gemm_exact_on_rounded_operands(lib, tA, tB, M, N, K, bias, relu, beta):
    """The big-tile bf16 GEMM (gemm_bf16.hip: operands staged to K-contiguous bf16, 256 x 256 / 128 x 128 MFMA
    tiles fed by LDS-DMA, split-K slabs summed in order): every transpose form, ragged M / N / K, split-K, bias /
    beta / ReLU epilogue, against the float64 product of the RNE-bf16-rounded operands (<= 2e-5 max|ref|), and
    two runs are bitwise equal."""
    import s2s_amd
    rng = np.random.default_rng(M + N + K + 7 * tA + 3 * tB)
    A = rng.standard_normal((K, M) if tA else (M, K)).astype(np.float32)
    B = rng.standard_normal((N, K) if tB else (K, N)).astype(np.float32)
    C0 = rng.standard_normal((M, N)).astype(np.float32)
    bv = rng.standard_normal(N).astype(np.float32) if bias else None
    Ag, Bg = torch.tensor(A, device="cuda"), torch.tensor(B, device="cuda")
    bg = torch.tensor(bv, device="cuda") if bias else None
    ctx = s2s_amd.nn.get_context(0)
    fn = _big_run(lib)
    outs = []
    for _ in range(2):
        Cg = torch.tensor(C0, device="cuda")
        done = ctypes.c_int(0)
        rc = fn(ctx.handle, s2s_amd.nn.stream_ptr(), tA, tB, M, N, K, 0.5, Ag.data_ptr(), A.shape[1], Bg.data_ptr(),
                B.shape[1], beta, Cg.data_ptr(), N, bg.data_ptr() if bias else None, int(relu), ctypes.byref(done))
        assert rc == 0 and done.value == 1
        outs.append(Cg)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    Ar, Br = bf16_round(A), bf16_round(B)
    ref = 0.5 * ((Ar.T if tA else Ar) @ (Br.T if tB else Br)) + beta * C0.astype(np.float64)
    if bias:
        ref = ref + bv.astype(np.float64)
    if relu:
        ref = np.maximum(ref, 0.0)
    err = np.abs(outs[0].cpu().numpy() - ref).max() / np.abs(ref).max()
    assert err <= 2e-5, err


@pytest.mark.parametrize("tA,tB", [(0, 1), (1, 0)])
def test_big_bf16_gemm_narrow_output_deep_split(lib, tA, tB):
    """The first VGG layer's weight gradient shape (64 x 27 outputs over ~600k pixels): one 128 x 128 tile split over
    up to 256 K-slices, the slabs summed in slice order -- exact on the bf16-rounded operands (<= 2e-5 max|ref|)."""
    import s2s_amd
    rng = np.random.default_rng(27 + tA)
    M, N, K = 64, 27, 200000
    A = rng.standard_normal((K, M) if tA else (M, K)).astype(np.float32)
    B = rng.standard_normal((N, K) if tB else (K, N)).astype(np.float32)
    Ag, Bg = torch.tensor(A, device="cuda"), torch.tensor(B, device="cuda")
    C = torch.zeros(M, N, device="cuda")
    done = ctypes.c_int(0)
    rc = _big_run(lib)(s2s_amd.nn.get_context(0).handle, s2s_amd.nn.stream_ptr(), tA, tB, M, N, K, 1.0, Ag.data_ptr(),
                       A.shape[1], Bg.data_ptr(), B.shape[1], 0.0, C.data_ptr(), N, None, 0, ctypes.byref(done))
    torch.cuda.synchronize()
    assert rc == 0 and done.value == 1
    Ar, Br = bf16_round(A), bf16_round(B)
    ref = (Ar.T if tA else Ar) @ (Br.T if tB else Br)
    err = np.abs(C.cpu().numpy() - ref).max() / np.abs(ref).max()
    assert err <= 2e-5, err


def _rel(a, r):
    """relative L2 error ||a - r|| / ||r||"""
    a = np.asarray(a, np.float64).ravel()
    r = np.asarray(r, np.float64).ravel()
    return float(np.linalg.norm(a - r) / max(np.linalg.norm(r), 1e-30))


# The bf16 tolerance (stated against the float64 oracle).  bf16 operands carry a unit roundoff of 2^-9 per
# operand; the forward outputs stay within ~1e-4.  The gradients move more: the forward's rounding flips
# near-tie DISCRETE decisions (which of a Maxout group's 7 units wins, which ReLU units are active), and a
# flipped decision routes a whole gradient row elsewhere -- for any bf16 implementation, not a kernel error
# (the bf16 GEMM kernel itself is exact on rounded operands: test_bf16_gemm_exact_on_rounded_operands).  So the
# bar is on relative L2 error: logp <= 1e-3, every gradient <= BF16_GRAD_RTOL, on every tensor that the fp32
# restatement itself gets to 1e-5 (measured: 1-6e-2 at config 3, <= 1.4e-1 at config 5).
BF16_LOGP_RTOL = 1e-3
BF16_GRAD_RTOL = 0.2


@pytest.mark.parametrize("prec", ["bf16", "bf16-all"])
def test_model_step_bf16_config3_dims(lib, prec):
    """BASELINE config 3 (model_chorowski_baseline_dropout.lua, bf16 MFMA): the whole step with bf16 GEMM
    operands (injected dropout masks, reduced L / T for the oracle) against the float64 oracle."""
    import s2s_amd
    from oracle import s2s_oracle as orc
    cfg_o = orc.ModelConfig()
    model = s2s_amd.ChorowskiBaseline(s2s_amd.ModelConfig(dropout=0.5), precision=prec)
    P = orc.unflatten(model.params.cpu().double().numpy(), cfg_o)
    B, L, T = 16, 48, 16
    x, labels = orc.synthetic_batch(cfg_o, B, L, T, seed=3, pad=10, eos=23)
    rng = np.random.default_rng(4)
    mask = (rng.random((B, T, cfg_o.stateDepth + 2 * cfg_o.outputFrameSize)) >= 0.5) / 0.5
    nll, logp = model.step(torch.tensor(x, dtype=torch.float32, device="cuda"),
                           torch.tensor(labels, dtype=torch.int32, device="cuda"),
                           dropout_mask=torch.tensor(mask, dtype=torch.float32, device="cuda"))
    torch.cuda.synchronize()
    _, G, lref, _ = orc.training_step(x, labels, P, cfg_o, dropout_mask=mask)
    errs = {"logp": _rel(logp.cpu().numpy(), lref)}
    Gg = orc.unflatten(model.grads.cpu().double().numpy(), cfg_o)
    errs.update({"grad " + k: _rel(Gg[k], G[k]) for k in G})
    print(f"config 3 {prec} max rel errs:", {k: f"{v:.1e}" for k, v in errs.items()})
    bad = {k: f"{v:.2e}" for k, v in errs.items() if not v <= (BF16_LOGP_RTOL if k == "logp" else BF16_GRAD_RTOL)}
    assert not bad, bad
    assert errs["logp"] > 1e-6  # bf16 really ran (fp32 reaches ~2e-7 here)


# With the Maxout decisions pinned (the oracle runs under the GPU's own winners, s2s_attn_maxout_argmax) the
# discrete flips are gone and what is left is bf16 operand rounding (unit roundoff 2^-9 = 2e-3 per operand) carried
# through the recurrences: the bars below are that, not the 0.2 of the unpinned comparison above.
BF16_PINNED_LOGP_RTOL = 1e-3
BF16_PINNED_GRAD_RTOL = 1e-2


@pytest.mark.parametrize("B,fused", [(64, False), (16, True)])
@pytest.mark.parametrize("prec", ["bf16", "bf16-all"])
def test_model_step_bf16_config3_decisions_pinned(lib, B, fused, prec):
    """BASELINE config 3 as benched (model_chorowski_baseline_dropout.lua:56, bf16 MFMA): B = 64 -- the BiGRU
    launches fill the chip, so the x-projections and dX run as separate bf16 GEMMs (asserted from the live kernel
    profile: the persistent launches carry only the recurrence's flops) -- and B = 16, where the persistent
    launches' spare slots compute them in fp32.  Reduced L / T for the float64 oracle, injected
    dropout masks; the oracle runs under the GPU's own Maxout decisions (Maxout.lua:14-18), so every tensor is
    held to the operand-rounding bar."""
    import s2s_amd
    from oracle import s2s_oracle as orc
    from s2s_amd import profile as prof
    cfg_o = orc.ModelConfig()
    model = s2s_amd.ChorowskiBaseline(s2s_amd.ModelConfig(dropout=0.5), precision=prec)
    P = orc.unflatten(model.params.cpu().double().numpy(), cfg_o)
    L, T = 40, 12
    x, labels = orc.synthetic_batch(cfg_o, B, L, T, seed=B, pad=10, eos=23)
    rng = np.random.default_rng(B + 1)
    mask = (rng.random((B, T, cfg_o.stateDepth + 2 * cfg_o.outputFrameSize)) >= 0.5) / 0.5
    xs = torch.tensor(x, dtype=torch.float32, device="cuda")
    ls = torch.tensor(labels, dtype=torch.int32, device="cuda")
    ms = torch.tensor(mask, dtype=torch.float32, device="cuda")
    lib.check(lib.lib.s2s_prof_enable(1))
    try:
        prof.collect()
        nll, logp = model.step(xs, ls, dropout_mask=ms)
        torch.cuda.synchronize()
        agg = prof.collect()
    finally:
        lib.lib.s2s_prof_enable(0)
    H = cfg_o.hiddenFrameSize
    rec = 2.0 * 2 * B * L * 3 * H * H  # both directions' recurrence of one layer
    fwd = agg["gru_fwd_persist"]
    assert fwd["launches"] == 3
    assert "gemm_bf16" in agg, sorted(agg)  # bf16 GEMMs ran
    per = fwd["flops"] / fwd["launches"]
    if fused:
        assert per > 1.5 * rec, (per, rec)  # the x-projections were computed inside the launches
    else:
        assert abs(per - rec) <= 1e-6 * rec, (per, rec)  # recurrence only: x-projections by separate GEMMs
        # dX too (the first layer's BPTT may carry its weight gradients, S2S_BPTT_WGRAD: counted, not a dX)
        bwd, wg = agg["gru_bwd_persist"], 2.0 * 2 * B * L * 3 * H * (H + cfg_o.inputFrameSize)
        assert bwd["flops"] <= 1.0001 * (bwd["launches"] * rec + wg), (bwd, rec, wg)
    am = model.decoder_maxout_argmax().cpu().numpy()
    assert am.shape == (B, T, cfg_o.mlpDepth) and am.min() >= 0 and am.max() < cfg_o.maxoutWindow
    _, G, lref, _ = orc.training_step(x, labels, P, cfg_o, dropout_mask=mask, maxout_idx=am)
    errs = {"logp": _rel(logp.cpu().numpy(), lref)}
    Gg = orc.unflatten(model.grads.cpu().double().numpy(), cfg_o)
    errs.update({"grad " + k: _rel(Gg[k], G[k]) for k in G})
    print(f"config 3 B={B} {prec} rel L2 errs (Maxout decisions pinned):", {k: f"{v:.1e}" for k, v in errs.items()})
    bad = {k: f"{v:.2e}" for k, v in errs.items()
           if not v <= (BF16_PINNED_LOGP_RTOL if k == "logp" else BF16_PINNED_GRAD_RTOL)}
    assert not bad, bad
    assert errs["logp"] > 1e-6  # bf16 really ran (fp32 reaches ~2e-7 here)


# bf16 operands move pre-activations by ~2^-9 of their scale per product, so a decision is "near a tie" within a
# few 1e-3 of its site's scale: flips there are adopted (measured: at most 5.2e-3 of the scale, pool3); a flip
# beyond this band would be a kernel error.
BF16_DECISION_BAND = 1e-2
# and at most this fraction of a site's decisions may be adopted flips (measured: at most 3.3e-3, pool3; 1.4e-3 the
# deepest conv ReLU).  (The local-scale margins are reported only: a pooling window's reaches 1.0 where an adopted
# ReLU flip -- a slightly negative oracle value under the GPU's "active" mask -- competes with a zero; that lead
# is the flip's own |u|, already bounded at its ReLU site.)
BF16_FLIP_FRACTION = 1e-2
# config 5 chains 12 bf16 products (8 encoder layers, the decoder, the decoder_mlp) against config 3's 4, so its
# pinned bar is twice config 3's (measured with decisions pinned: 1.8e-4 .. 1.05e-2, the deepest layer dvgg2 worst;
# 7-9e-2 before pinning)
BF16_PINNED_DEEP_GRAD_RTOL = 2e-2
# The attention score layer's gradients dV / dWs / dbs / dwe all hang off de_l = alpha_l (h_l - c) . dc: a projection
# of the context gradient dc (bf16 MLP data-gradient product upstream, ~6e-3 relative like every other tensor here)
# onto h_l - c, a direction nearly orthogonal to it in 512 dimensions, so dc's rounding error reaches de ~4x
# amplified -- measured 2.4-2.5e-2 on all four at the conditioned test point (vgg_case.condition; fp32 floor
# 0.6-3e-5, so the bar judges the kernels, not fp32 noise).  Held to 5e-2 (the round-5 bar was 0.1 on an unconditioned
# case whose fp32 floor reached 0.9).
BF16_ATTN_GRAD_RTOL = 5e-2


@pytest.mark.parametrize("prec", ["bf16", "bf16-all"])
def test_vgg_model_step_bf16_config5(lib, prec):
    """BASELINE config 5 (librispeech/model_vgg.lua:23-82, bf16): full width (1x1 layers 2048), B = 1, L = 256,
    T = 50, against the float64 oracle run under the GPU's own discrete decisions (the VGG and 1x1 ReLUs, both
    SpatialMaxPoolings and the two decoder_mlp Maxouts) -- each adopted flip must sit within BF16_DECISION_BAND of
    its tie -- so every tensor is held to the operand-rounding bar, as config 3 is (BF16_PINNED_DEEP_GRAD_RTOL).
    The parameters are the conditioned test point of tests/vgg_case.py (`condition`: at the default init the
    attention is uniform and the score layer's gradients dV / dWs / dbs / dwe cancel to ~1e-11, unjudgeable), so
    every tensor is judged: the attention score layer's four at BF16_ATTN_GRAD_RTOL (their de projection amplifies
    the context gradient's bf16 rounding, see there), the rest at the pinned bar.  bf16-all also takes the weight
    gradients in bf16."""
    import s2s_amd
    import vgg_case as vc
    from s2s_amd import frontend as fe
    g = torch.Generator().manual_seed(5)
    B, L, T = 1, 256, 50
    model = s2s_amd.VGGAttentionModel(40, outputFrameSize=512, hidden=2048, outputDepth=29, generator=g,
                                      precision=prec).cuda()
    vc.condition(model, fe)
    rng = np.random.default_rng(5)
    x = rng.standard_normal((B, 3, L, 40)).astype(np.float32).astype(np.float64)
    labels = np.append(rng.integers(0, 28, (B, T - 1)), np.full((B, 1), 28), axis=1).astype(np.int32)
    model.zeroGradParameters()
    nll, logp = model.step(torch.tensor(x, dtype=torch.float32, device="cuda"),
                           torch.tensor(labels, dtype=torch.int32, device="cuda"))
    torch.cuda.synchronize()
    decide, mx = vc.gpu_decisions(model, fe)
    raw = {}
    nll64, logp64, G64, mg64 = vc.oracle_step(model, fe, x, labels, np.float64, decide, mx, raw)
    nll32, logp32, G32, mg32 = vc.oracle_step(model, fe, x, labels, np.float32, decide, mx)
    margins = vc.decision_margins(decide, mx, raw)
    print(f"config 5 {prec} adopted flips (count, fraction, largest margin / layer scale, / local scale):", margins)
    wide = {k: v for k, v in margins.items() if v[2] > BF16_DECISION_BAND}
    assert not wide, wide
    # near-tie flips are rare: a kernel error that flips many small units stays inside the layer-wide band but not
    # inside this count bound
    many = {k: v for k, v in margins.items() if v[1] > BF16_FLIP_FRACTION}
    assert not many, many
    errs = {"logp": _rel(logp.cpu().numpy(), logp64)}
    floor = {"logp": _rel(logp32, logp64)}
    for (name, gpu, r64), (_, _, r32) in zip(vc.grad_pairs(model, fe, G64, mg64), vc.grad_pairs(model, fe, G32, mg32)):
        errs[name] = _rel(gpu.detach().cpu().numpy(), r64)
        floor[name] = _rel(r32, r64)
    print(f"config 5 {prec} rel L2 errs, decisions pinned (fp32 floor):",
          {k: f"{errs[k]:.1e} ({floor[k]:.1e})" for k in errs})
    # every tensor is judged; the attention score layer's gradients are conditioned here (fp32 floor <= 1e-4, measured
    # 0.6-3e-5 under the two variants' adopted decisions; the unconditioned case reached 0.9)
    attn = ("dV", "dWs", "dbs", "dwe")
    att = {k: f"{floor[k]:.1e}" for k in attn if not floor[k] <= 1e-4}
    assert not att, att
    bad = {k: f"{errs[k]:.2e}" for k in errs
           if not errs[k] <= (BF16_PINNED_LOGP_RTOL if k == "logp" else BF16_ATTN_GRAD_RTOL if k in attn else
                              BF16_PINNED_DEEP_GRAD_RTOL)}
    assert not bad, bad
    assert errs["logp"] > 1e-6  # bf16 really ran


@pytest.mark.parametrize("B,Cin,H,W,Cout,relu", [(2, 3, 20, 12, 64, True), (2, 64, 17, 11, 64, False),
                                                   (1, 128, 9, 13, 128, True), (3, 5, 7, 6, 7, False),
                                                   (2, 64, 40, 21, 128, False)])
def test_bf16_implicit_conv_exact_on_rounded_operands(lib, B, Cin, H, W, Cout, relu):
    """SpatialConvolutionMM under bf16 runs as implicit GEMMs (conv_bf16.inc: no im2col / col2im panels):
    the forward and the input gradient equal float64 convolutions of the bf16-rounded operands up to the
    fp32 accumulation order (<= 2e-5 max|ref|); ragged pixel tiles, K = 27 / 45 / 576 / 1152, two channel
    tiles, ReLU on and off."""
    import s2s_amd
    from s2s_amd import frontend as fe
    from numpy.lib.stride_tricks import sliding_window_view as win
    rng = np.random.default_rng(B * 1000 + Cin + H)
    conv = fe.SpatialConvolutionMM(Cin, Cout, 3, 3, relu=relu)
    x = rng.standard_normal((B, Cin, H, W)).astype(np.float32)
    Wt = (rng.standard_normal((Cout, Cin * 9)) * 0.2).astype(np.float32)
    bias = (rng.standard_normal(Cout) * 0.1).astype(np.float32)
    dy = rng.standard_normal((B, Cout, H - 2, W - 2)).astype(np.float32)
    conv.weight = torch.tensor(Wt, device="cuda")
    conv.bias = torch.tensor(bias, device="cuda")
    conv.gradWeight = torch.zeros_like(conv.weight)
    conv.gradBias = torch.zeros_like(conv.bias)
    xg, dyg = torch.tensor(x, device="cuda"), torch.tensor(dy, device="cuda")
    with s2s_amd.precision("bf16"):
        y = conv.forward(xg).clone()
        dx = conv.backward(xg, dyg).clone()
    torch.cuda.synchronize()
    xr, Wr = bf16_round(x), bf16_round(Wt).reshape(Cout, Cin, 3, 3)
    pre = np.einsum("bchwij,ocij->bohw", win(xr, (3, 3), axis=(2, 3)), Wr) + bias.astype(np.float64)[None, :, None, None]
    yref = np.maximum(pre, 0.0) if relu else pre
    err = np.abs(y.cpu().numpy() - yref).max() / np.abs(yref).max()
    assert err <= 2e-5, ("y", err)
    dyt = dy.astype(np.float64) * (pre > 0) if relu else dy.astype(np.float64)
    dyr = bf16_round(dyt.astype(np.float32))
    pad = np.pad(dyr, ((0, 0), (0, 0), (2, 2), (2, 2)))
    dxref = np.einsum("bohwij,ocij->bchw", win(pad, (3, 3), axis=(2, 3)), Wr[:, :, ::-1, ::-1])
    err = np.abs(dx.cpu().numpy() - dxref).max() / np.abs(dxref).max()
    assert err <= 2e-5, ("dx", err)


@pytest.mark.parametrize("implicit", [1, 0])
@pytest.mark.parametrize("B,Cin,H,W,Cout,relu", [(2, 64, 17, 11, 64, False), (1, 128, 9, 13, 128, True),
                                                   (2, 64, 40, 21, 128, True), (3, 5, 7, 6, 7, False),
                                                   (16, 64, 70, 38, 64, True)])
def test_bf16_conv_weight_gradient_exact_on_rounded_operands(lib, implicit, B, Cin, H, W, Cout, relu):
    """SpatialConvolutionMM weight / bias gradient under bf16-all: Cin % 64 == 0 takes the implicit bf16 weight
    gradient (conv_wgrad_bf16_kernel: channels-last gather, split pixel chunks summed in order; implicit=0 forces
    the im2col panel + bf16 GEMM for comparison), other Cin the panel.  gradWeight (accumulated onto a nonzero
    start, scale 0.5) equals the float64 product of the bf16-rounded ReLU-masked dy and input up to the fp32
    accumulation order (<= 2e-5 max|ref|); ragged pixel chunks, two output-channel tiles, 9 / 18 column tiles."""
    import s2s_amd
    from s2s_amd import frontend as fe
    from numpy.lib.stride_tricks import sliding_window_view as win
    knob = lib.lib.s2s_debug_sconv_wgrad_implicit
    knob.argtypes = [ctypes.c_int]
    rng = np.random.default_rng(B * 100 + Cin + W)
    conv = fe.SpatialConvolutionMM(Cin, Cout, 3, 3, relu=relu)
    x = rng.standard_normal((B, Cin, H, W)).astype(np.float32)
    Wt = (rng.standard_normal((Cout, Cin * 9)) * 0.2).astype(np.float32)
    bias = (rng.standard_normal(Cout) * 0.1).astype(np.float32)
    dy = rng.standard_normal((B, Cout, H - 2, W - 2)).astype(np.float32)
    gw0 = rng.standard_normal((Cout, Cin * 9)).astype(np.float32)
    conv.weight = torch.tensor(Wt, device="cuda")
    conv.bias = torch.tensor(bias, device="cuda")
    conv.gradWeight = torch.tensor(gw0, device="cuda")
    conv.gradBias = torch.zeros_like(conv.bias)
    xg, dyg = torch.tensor(x, device="cuda"), torch.tensor(dy, device="cuda")
    knob(implicit)
    try:
        with s2s_amd.precision("bf16-all"):
            conv.forward(xg)
            conv.backward(xg, dyg, 0.5)
        torch.cuda.synchronize()
    finally:
        knob(1)
    xr, Wr = bf16_round(x), bf16_round(Wt).reshape(Cout, Cin, 3, 3)
    pre = np.einsum("bchwij,ocij->bohw", win(xr, (3, 3), axis=(2, 3)), Wr) + bias.astype(np.float64)[None, :, None, None]
    dyt = dy.astype(np.float64) * (pre > 0) if relu else dy.astype(np.float64)
    dyr = bf16_round(dyt.astype(np.float32))
    gref = gw0 + 0.5 * np.einsum("bohw,bchwij->ocij", dyr, win(xr, (3, 3), axis=(2, 3))).reshape(Cout, Cin * 9)
    err = np.abs(conv.gradWeight.cpu().numpy() - gref).max() / np.abs(gref - gw0).max()
    assert err <= 2e-5, ("dW", err)
    bref = 0.5 * dyt.sum(axis=(0, 2, 3))
    err = np.abs(conv.gradBias.cpu().numpy() - bref).max() / np.abs(bref).max()
    assert err <= 2e-5, ("db", err)


@pytest.mark.parametrize("big", [1, 0])
@pytest.mark.parametrize("B,L,Din,Dout,relu", [(4, 508, 896, 2048, True), (3, 300, 2048, 512, False), (2, 50, 64, 40, True)])
def test_bf16_linear_layer_exact_on_rounded_operands(lib, big, B, L, Din, Dout, relu):
    """TemporalConvolution(Din, Dout, 1) (+ReLU) -- the VGG model's 1x1 layers and nn.Linear -- under bf16-all: one
    GEMM over the B L rows, on the big-tile bf16 kernel when large (gemm_bf16.hip; big=0 forces gemm_f32's 64 x 64
    bf16 tiles).  Forward, input gradient and weight / bias gradients equal float64 products of the RNE-bf16-rounded
    operands up to fp32 accumulation order (<= 2e-5 of max|ref|), and two runs are bitwise equal."""
    import s2s_amd
    from s2s_amd import frontend as fe
    knob = lib.lib.s2s_debug_gemm_big
    knob.argtypes = [ctypes.c_int]
    rng = np.random.default_rng(B + L + Din)
    m = fe.TemporalConvolution(Din, Dout, 1, relu=relu)
    x = rng.standard_normal((B, L, Din)).astype(np.float32)
    W = (rng.standard_normal((Dout, Din)) / np.sqrt(Din)).astype(np.float32)
    b = (rng.standard_normal(Dout) * 0.1).astype(np.float32)
    dy = rng.standard_normal((B, L, Dout)).astype(np.float32)
    m.weight, m.bias = torch.tensor(W, device="cuda"), torch.tensor(b, device="cuda")
    xg, dyg = torch.tensor(x, device="cuda"), torch.tensor(dy, device="cuda")
    calls = lib.lib.s2s_debug_gemm_big_calls
    calls.restype = ctypes.c_long
    n0 = calls()
    outs = []
    knob(big)
    try:
        for _ in range(2):
            m.gradWeight, m.gradBias = torch.zeros_like(m.weight), torch.zeros_like(m.bias)
            with s2s_amd.precision("bf16-all"):
                y = m.forward(xg).clone()
                dx = m.backward(xg, dyg, 0.5).clone()
            outs.append((y, dx, m.gradWeight.clone(), m.gradBias.clone()))
        torch.cuda.synchronize()
    finally:
        knob(1)
    for a, c in zip(outs[0], outs[1]):
        assert torch.equal(a, c)
    large = 2.0 * B * L * Din * Dout >= 1e9
    assert (calls() - n0 == 6) == (bool(big) and large), calls() - n0  # fwd, dx, dW per run
    y, dx, gw, gb = (t.double().cpu().numpy() for t in outs[0])
    xr, Wr = bf16_round(x).reshape(B * L, Din), bf16_round(W)
    pre = xr @ Wr.T + b.astype(np.float64)
    yref = np.maximum(pre, 0) if relu else pre
    assert np.abs(y.reshape(B * L, Dout) - yref).max() / np.abs(yref).max() <= 2e-5
    dyt = dy.reshape(B * L, Dout).astype(np.float64) * ((pre > 0) if relu else 1.0)
    dyr = bf16_round(dyt.astype(np.float32))
    dxref = dyr @ Wr
    assert np.abs(dx.reshape(B * L, Din) - dxref).max() / np.abs(dxref).max() <= 2e-5
    gref = 0.5 * dyr.T @ xr
    assert np.abs(gw - gref).max() / np.abs(gref).max() <= 2e-5
    bref = 0.5 * dyt.sum(0)
    assert np.abs(gb - bref).max() / np.abs(bref).max() <= 2e-5
