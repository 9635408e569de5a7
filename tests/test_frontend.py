"""Encoder front-ends: the conv + BiLSTM encoder (timit/timit.lua:108-125) and the VGG
stack (librispeech/model_vgg.lua:23-51).

CPU: the oracle's operator restatements (oracle/frontend_oracle.py) against torch.nn.functional autograd
(an independent formulation of the same Torch7 nn semantics), and the encoder-level backward against
central finite differences.  GPU: libs2s_hip.so through the host mirror (s2s_amd.frontend) against the
oracle, tolerance max|gpu - ref| <= 1e-4 * max|ref| per tensor (fp32 vs float64).
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import frontend_oracle as fo

RTOL = 1e-4
# ill-conditioned tensors: bar = max(RTOL, FLOOR_FACTOR x the fp32 restatement's own error), see
# tests/test_gpu_fullsize.py
FLOOR_FACTOR = 16


def rel_err(g, r):
    g = np.asarray(g, dtype=np.float64)
    r = np.asarray(r, dtype=np.float64)
    assert g.shape == r.shape, (g.shape, r.shape)
    return float(np.abs(g - r).max() / max(np.abs(r).max(), 1e-30))


def assert_rel(g, r, name, rtol=RTOL):
    e = rel_err(g, r)
    assert np.isfinite(np.asarray(g, dtype=np.float64)).all(), f"{name}: non-finite values"
    assert e <= rtol, f"{name}: max rel err {e:.3e} > {rtol:.0e}"


def t64(a, grad=False):
    return torch.tensor(a, dtype=torch.float64, requires_grad=grad)


# --------------------------------------------------------------------------- oracle vs torch autograd (CPU)

@pytest.mark.parametrize("B,L,Din,Dout,kW", [(2, 11, 5, 4, 3), (1, 7, 3, 6, 1), (3, 9, 4, 2, 4)])
def test_oracle_tconv_matches_torch(B, L, Din, Dout, kW):
    rng = np.random.default_rng(L)
    x, W, b = rng.standard_normal((B, L, Din)), rng.standard_normal((Dout, kW * Din)), rng.standard_normal(Dout)
    dy = rng.standard_normal((B, L - kW + 1, Dout))
    xt, Wt, bt = t64(x, True), t64(W, True), t64(b, True)
    # Torch7 weight (out, kW*in), frame-major -> conv1d weight (out, in, kW)
    yt = F.conv1d(xt.transpose(1, 2), Wt.reshape(Dout, kW, Din).transpose(1, 2), bt).transpose(1, 2)
    yt.backward(t64(dy))
    y = fo.tconv_fwd(x, W, b, kW)
    dx, dW, db = fo.tconv_bwd(x, W, dy, kW)
    for g, r, n in ((y, yt, "y"), (dx, xt.grad, "dx"), (dW, Wt.grad, "dW"), (db, bt.grad, "db")):
        assert_rel(g, r.detach().numpy(), n, 1e-12)


def test_oracle_sconv_notebook_known_answer():
    """Attention.ipynb cell 2 (the "Vh" cell): SpatialConvolutionMM(1, scoreDepth=4, kW=annotationDepth=5, kH=1)
    with every parameter filled with 1 (p:fill(1)), on ones(1, L=10, 5) -> a (4, 10, 1) output of 6s (5 ones
    + bias 1).  Pins the (out, in*kH*kW) weight / bias layout of the SpatialConvolutionMM restatement."""
    Wt = np.ones((4, 1 * 1 * 5))
    y = fo.sconv_fwd(np.ones((1, 1, 10, 5)), Wt, np.ones(4), kH=1, kW=5)
    assert y.shape == (1, 4, 10, 1)
    np.testing.assert_array_equal(y, np.full((1, 4, 10, 1), 6.0))


def test_oracle_tmaxpool_matches_torch():
    rng = np.random.default_rng(3)
    x = rng.standard_normal((2, 13, 5))
    y, idx = fo.tmaxpool_fwd(x, 2, 2)
    xt = t64(x, True)
    yt = F.max_pool1d(xt.transpose(1, 2), 2, 2).transpose(1, 2)
    dy = rng.standard_normal(y.shape)
    yt.backward(t64(dy))
    assert_rel(y, yt.detach().numpy(), "y", 0)
    assert_rel(fo.tmaxpool_bwd(idx, dy, 13, 2, 2), xt.grad.numpy(), "dx", 0)
    # first maximum wins on ties (THNN `if (val > maxval)`)
    y2, idx2 = fo.tmaxpool_fwd(np.zeros((1, 4, 1)), 2, 2)
    assert (idx2 == 0).all()


@pytest.mark.parametrize("B,C,H,W,O,k", [(2, 3, 9, 8, 4, 3), (1, 2, 5, 7, 3, 2)])
def test_oracle_sconv_matches_torch(B, C, H, W, O, k):
    rng = np.random.default_rng(H * W)
    x, Wt_, b = rng.standard_normal((B, C, H, W)), rng.standard_normal((O, C * k * k)), rng.standard_normal(O)
    xt, wt, bt = t64(x, True), t64(Wt_, True), t64(b, True)
    yt = F.conv2d(xt, wt.reshape(O, C, k, k), bt)
    dy = rng.standard_normal(yt.shape)
    yt.backward(t64(dy))
    y = fo.sconv_fwd(x, Wt_, b, k, k)
    dx, dW, db = fo.sconv_bwd(x, Wt_, dy, k, k)
    for g, r, n in ((y, yt, "y"), (dx, xt.grad, "dx"), (dW, wt.grad, "dW"), (db, bt.grad, "db")):
        assert_rel(g, r.detach().numpy(), n, 1e-12)


@pytest.mark.parametrize("kW,kH,dW,dH", [(2, 1, 2, 1), (2, 2, 2, 2), (3, 2, 2, 1)])
def test_oracle_smaxpool_matches_torch(kW, kH, dW, dH):
    rng = np.random.default_rng(kW * 10 + kH)
    x = rng.standard_normal((2, 3, 9, 11))
    y, idx = fo.smaxpool_fwd(x, kW, kH, dW, dH)
    xt = t64(x, True)
    yt = F.max_pool2d(xt, (kH, kW), (dH, dW))
    dy = rng.standard_normal(y.shape)
    yt.backward(t64(dy))
    assert_rel(y, yt.detach().numpy(), "y", 0)
    assert_rel(fo.smaxpool_bwd(idx, dy, 9, 11, kW, kH, dW, dH), xt.grad.numpy(), "dx", 1e-15)


def _vgg_params(rng, hidden=16, out=8, F_=16):
    P = {}
    for l, (ci, co) in enumerate(fo.VGG_CONVS):
        P[f"vgg{l}.W"] = rng.standard_normal((co, ci * 9)) / np.sqrt(ci * 9)
        P[f"vgg{l}.b"] = rng.standard_normal(co) * 0.1
    for l, (di, do) in enumerate(fo.vgg_dims(F_, hidden, out)):
        P[f"lin{l}.W"] = rng.standard_normal((do, di)) / np.sqrt(di)
        P[f"lin{l}.b"] = rng.standard_normal(do) * 0.1
    return P


def _fd_check(fwd, bwd, P, x, keys, rng, n=3, eps=1e-6):
    y, cache = fwd(x, P)
    dy = rng.standard_normal(y.shape)
    G = {k: np.zeros_like(v) for k, v in P.items()}
    bwd(P, cache, dy, G)
    for k in keys:
        for _ in range(n):
            i = tuple(rng.integers(0, s) for s in P[k].shape)
            old = P[k][i]
            P[k][i] = old + eps
            fp = (fwd(x, P)[0] * dy).sum()
            P[k][i] = old - eps
            fm = (fwd(x, P)[0] * dy).sum()
            P[k][i] = old
            fd = (fp - fm) / (2 * eps)
            assert abs(fd - G[k][i]) <= 1e-6 * max(1.0, abs(fd)), (k, i, fd, G[k][i])


def test_oracle_vgg_encoder_finite_differences():
    rng = np.random.default_rng(7)
    P = _vgg_params(rng)
    x = rng.standard_normal((1, 3, 14, 16))
    _fd_check(fo.vgg_fwd, fo.vgg_bwd, P, x, ["vgg0.W", "vgg3.b", "lin0.W", "lin3.b"], rng)


def test_oracle_conv_bilstm_finite_differences():
    rng = np.random.default_rng(8)
    D, Hd, Ho = 5, 6, 4
    P = {}
    for l in range(3):
        din = D if l == 0 else Hd
        P[f"conv{l}.W"] = rng.standard_normal((Hd, 3 * din)) / np.sqrt(3 * din)
        P[f"conv{l}.b"] = rng.standard_normal(Hd) * 0.1
    for d in ("f.", "b."):
        for q in "ifgo":
            P[f"{d}W{q}x"] = rng.standard_normal((Ho, Hd)) * 0.4
            P[f"{d}b{q}x"] = rng.standard_normal(Ho) * 0.1
            P[f"{d}W{q}h"] = rng.standard_normal((Ho, Ho)) * 0.4
            P[f"{d}b{q}h"] = rng.standard_normal(Ho) * 0.1
    x = rng.standard_normal((2, 40, D))
    _fd_check(fo.conv_bilstm_fwd, fo.conv_bilstm_bwd, P, x, ["conv0.W", "conv2.b", "f.Wix", "b.bfh"], rng)


# --------------------------------------------------------------------------- GPU parity

@pytest.fixture(scope="module")
def fe():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from s2s_amd import frontend
    return frontend


def cu(a, dtype=torch.float32):
    return torch.tensor(np.ascontiguousarray(a), dtype=dtype, device="cuda")


def _np(t):
    return t.double().cpu().numpy()


@pytest.mark.gpu
@pytest.mark.parametrize("B,L,Din,Dout,kW,relu", [(4, 64, 123, 256, 3, True), (3, 17, 256, 256, 3, True),
                                                  (2, 9, 896, 2048, 1, True), (5, 12, 7, 5, 4, False),
                                                  (8, 1024, 64, 1024, 1, True),  # 8.4M ReLU outputs
                                                  (1, 3, 40, 16, 3, False)])
def test_tconv_matches_oracle(fe, B, L, Din, Dout, kW, relu):
    rng = np.random.default_rng(B * 100 + L)
    m = fe.TemporalConvolution(Din, Dout, kW, relu=relu).cuda()
    x = rng.standard_normal((B, L, Din))
    W, b = _np(m.weight), _np(m.bias)
    y = m.forward(cu(x))
    u = fo.tconv_fwd(x, W, b, kW)
    yr = fo.relu_fwd(u) if relu else u
    assert_rel(_np(y), yr, "y")
    dy = rng.standard_normal(yr.shape)
    m.gradWeight.fill_(0.5)
    m.gradBias.fill_(-0.25)
    dx = m.backward(cu(x), cu(dy), 0.5)
    # the ReLU's gradient is discontinuous at 0: compare under the GPU's decisions (1[y > 0]), which can
    # differ from the float64 oracle's only where u is within fp32 rounding of 0
    du = np.where(_np(y) > 0, dy, 0.0) if relu else dy
    dxr, dWr, dbr = fo.tconv_bwd(x, W, du, kW)
    torch.cuda.synchronize()
    assert_rel(_np(dx), dxr, "dx")
    assert_rel(_np(m.gradWeight), 0.5 + 0.5 * dWr, "dW")
    assert_rel(_np(m.gradBias), -0.25 + 0.5 * dbr, "db")


@pytest.mark.gpu
@pytest.mark.parametrize("B,L,D,kW,dW", [(4, 62, 256, 2, 2), (3, 13, 5, 2, 2), (2, 10, 7, 3, 2), (2, 9, 3, 2, 1)])
def test_tmaxpool_matches_oracle(fe, B, L, D, kW, dW):
    rng = np.random.default_rng(L)
    x = rng.standard_normal((B, L, D)).astype(np.float32).astype(np.float64)  # exact ops: compare on fp32 inputs
    x[0, :2, 0] = 1.0  # a tie: the first maximum wins
    m = fe.TemporalMaxPooling(kW, dW)
    y = m.forward(cu(x))
    yr, idx = fo.tmaxpool_fwd(x, kW, dW)
    assert_rel(_np(y), yr, "y", 0)
    assert (m.indices.cpu().numpy() == idx).all()
    dy = rng.standard_normal(yr.shape)
    dx = m.backward(cu(x), cu(dy))
    assert_rel(_np(dx), fo.tmaxpool_bwd(idx, dy, L, kW, dW), "dx", 1e-6)


@pytest.mark.gpu
@pytest.mark.parametrize("B,C,H,W,O,k,relu", [(2, 3, 40, 40, 64, 3, True), (2, 64, 20, 18, 128, 3, True),
                                              (3, 5, 9, 11, 7, 2, False), (1, 1, 3, 3, 1, 3, False)])
def test_sconv_matches_oracle(fe, B, C, H, W, O, k, relu):
    rng = np.random.default_rng(H * W + C)
    m = fe.SpatialConvolutionMM(C, O, k, k, relu=relu).cuda()
    x = rng.standard_normal((B, C, H, W))
    Wt, b = _np(m.weight), _np(m.bias)
    y = m.forward(cu(x))
    u = fo.sconv_fwd(x, Wt, b, k, k)
    yr = fo.relu_fwd(u) if relu else u
    assert_rel(_np(y), yr, "y")
    dy = rng.standard_normal(yr.shape)
    m.gradWeight.fill_(0.5)
    dx = m.backward(cu(x), cu(dy), 2.0)
    du = np.where(_np(y) > 0, dy, 0.0) if relu else dy  # under the GPU's ReLU decisions (see above)
    dxr, dWr, dbr = fo.sconv_bwd(x, Wt, du, k, k)
    torch.cuda.synchronize()
    assert_rel(_np(dx), dxr, "dx")
    assert_rel(_np(m.gradWeight), 0.5 + 2.0 * dWr, "dW")
    assert_rel(_np(m.gradBias), 2.0 * dbr, "db")


@pytest.mark.gpu
def test_sconv_notebook_known_answer_on_gpu(fe):
    """Attention.ipynb cell 2 on the HIP SpatialConvolutionMM: every parameter 1, input ones(1, 10, 5) (3-D, one
    image), kW = 5, kH = 1 -> (4, 10, 1) of 6s, exactly."""
    conv = fe.SpatialConvolutionMM(1, 4, 5, 1).cuda()
    conv.weight.fill_(1.0)
    conv.bias.fill_(1.0)
    y = conv.forward(torch.ones(1, 10, 5, device="cuda"))
    torch.cuda.synchronize()
    assert tuple(y.shape) == (4, 10, 1)
    assert torch.equal(y.cpu(), torch.full((4, 10, 1), 6.0))


@pytest.mark.gpu
@pytest.mark.parametrize("kW,kH,dW,dH,H,W", [(2, 1, 2, 1, 36, 36), (2, 2, 2, 2, 33, 15), (3, 2, 2, 1, 9, 11)])
def test_smaxpool_matches_oracle(fe, kW, kH, dW, dH, H, W):
    rng = np.random.default_rng(H + W)
    x = rng.standard_normal((2, 3, H, W)).astype(np.float32).astype(np.float64)
    m = fe.SpatialMaxPooling(kW, kH, dW, dH)
    y = m.forward(cu(x))
    yr, idx = fo.smaxpool_fwd(x, kW, kH, dW, dH)
    assert_rel(_np(y), yr, "y", 0)
    assert (m.indices.cpu().numpy() == idx).all()
    dy = rng.standard_normal(yr.shape)
    assert_rel(_np(m.backward(cu(x), cu(dy))), fo.smaxpool_bwd(idx, dy, H, W, kW, kH, dW, dH), "dx", 1e-6)


@pytest.mark.gpu
def test_transpose2_relu(fe):
    rng = np.random.default_rng(5)
    x = rng.standard_normal((2, 4, 6, 3)).astype(np.float32).astype(np.float64)
    m = fe.Transpose2((1, 2), 3)
    y = m.forward(cu(x))
    assert_rel(_np(y), x.transpose(0, 2, 1, 3), "y", 0)
    dy = rng.standard_normal(y.shape).astype(np.float32).astype(np.float64)
    assert_rel(_np(m.backward(cu(x), cu(dy))), dy.transpose(0, 2, 1, 3), "dx", 0)
    r = fe.ReLU()
    assert_rel(_np(r.forward(cu(x))), fo.relu_fwd(x), "relu", 0)
    dy = rng.standard_normal(x.shape).astype(np.float32).astype(np.float64)
    assert_rel(_np(r.backward(cu(x), cu(dy))), fo.relu_bwd(x, dy), "drelu", 0)


def _assert_grads(pairs, rtol=RTOL):
    errs = {name: rel_err(_np(g), r) for name, g, r in pairs}
    bad = {k: f"{v:.2e}" for k, v in errs.items() if not v <= rtol}
    assert not bad, f"max rel err > {rtol:.0e}: {bad}"


def _adopt_conv_decisions(convs, pools, ccache, margin=1e-5):
    """The conv stack's ReLU (1[u > 0]) and TemporalMaxPooling (first maximum) decisions are discrete: where u
    or the gap between a window's two values sits within fp32 noise of 0, any fp32 implementation -- the
    reference's CudaTensor path too -- may decide differently from the float64 oracle, and a flipped decision
    reroutes a whole gradient entry.  Require the GPU's decisions to equal the oracle's wherever the margin is
    clear (|u| or the window gap > margin * max|u|), then run the oracle's backward under the GPU's decisions
    (as _adopt_mono_decisions does for MonotonicAlignment, tests/test_gpu_parity.py).  Returns the number of
    adopted flips per layer."""
    flips = []
    for l, (tc, tp) in enumerate(zip(convs, pools)):
        h, u, idx, Lr = ccache[l]
        scale = np.abs(u).max()
        gmask = _np(tc.output) > 0  # the fused ReLU's output: positive exactly where the GPU passed u
        omask = u > 0
        clear = np.abs(u) > margin * scale
        assert np.array_equal(gmask[clear], omask[clear]), f"layer {l}: ReLU decisions differ off the near-tie band"
        gidx = tp.indices.cpu().numpy().astype(idx.dtype)
        r = np.maximum(u, 0.0)[:, :2 * idx.shape[1]].reshape(idx.shape[0], idx.shape[1], 2, -1)
        gap = np.abs(r[:, :, 0] - r[:, :, 1])
        clear_p = gap > margin * scale
        assert np.array_equal(gidx[clear_p], idx[clear_p]), f"layer {l}: max-pooling decisions differ off the band"
        flips.append(int((gmask != omask).sum() + (gidx != idx).sum()))
        # run the backward under the GPU's decisions: relu_bwd reads only the sign of u
        ccache[l] = (h, np.where(gmask, 1.0, -1.0), gidx, Lr)
    return flips


@pytest.mark.gpu
def test_conv_bilstm_encoder_matches_oracle(fe):
    """timit/timit.lua:108-125 at its sizes (D=123, 256 conv maps, LSTM 128 per direction).  Weights from a seeded
    generator; the oracle gets the fp32-rounded x / dy the GPU sees; ReLU / max-pooling near ties are adopted from
    the GPU (_adopt_conv_decisions) -- the bar stays 1e-4 on every tensor."""
    import s2s_amd
    rng = np.random.default_rng(11)
    B, L, D = 4, 64, 123
    enc = s2s_amd.ConvBiLSTMEncoder(D, generator=torch.Generator().manual_seed(11)).cuda()
    P = {}
    convs = [m for m in enc.convlayer.modules if isinstance(m, fe.TemporalConvolution)]
    pools = [m for m in enc.convlayer.modules if isinstance(m, fe.TemporalMaxPooling)]
    for l, m in enumerate(convs):
        P[f"conv{l}.W"], P[f"conv{l}.b"] = _np(m.weight), _np(m.bias)
    cells = enc.rnn.cells
    for pre, c in zip(("f.", "b."), cells):
        for k, v in c.named().items():
            P[pre + k] = _np(v)
    x = rng.standard_normal((B, L, D)).astype(np.float32).astype(np.float64)
    y = enc.forward(cu(x))
    yr, cache = fo.conv_bilstm_fwd(x, P)
    assert_rel(_np(y), yr, "y")
    dy = rng.standard_normal(yr.shape).astype(np.float32).astype(np.float64)
    enc.zeroGradParameters()
    enc.backward(cu(x), cu(dy), 1.0)
    _adopt_conv_decisions(convs, pools, cache[1])
    G = {k: np.zeros_like(v) for k, v in P.items()}
    fo.conv_bilstm_bwd(P, cache, dy, G)
    torch.cuda.synchronize()
    pairs = []
    for l, m in enumerate(convs):
        pairs += [(f"dconv{l}.W", m.gradWeight, G[f"conv{l}.W"]), (f"dconv{l}.b", m.gradBias, G[f"conv{l}.b"])]
    for pre, c in zip(("f.", "b."), cells):
        pairs += [(f"d{pre}{k}", g, G[pre + k]) for k, g in c.named(grads=True).items()]
    _assert_grads(pairs)


@pytest.mark.gpu
def test_vgg_encoder_matches_oracle(fe):
    """librispeech/model_vgg.lua:23-51 with 40 mel bands (the 2048-wide 1x1 convs narrowed to 256)."""
    import s2s_amd
    rng = np.random.default_rng(12)
    B, L, Fq = 2, 40, 40
    enc = s2s_amd.VGGEncoder(Fq, outputFrameSize=128, hidden=256, generator=torch.Generator().manual_seed(12)).cuda()
    mods = enc.seq.modules
    convs = [m for m in mods if isinstance(m, fe.SpatialConvolutionMM)]
    lins = [m for m in mods if isinstance(m, fe.TemporalConvolution)]
    P = {}
    for l, m in enumerate(convs):
        P[f"vgg{l}.W"], P[f"vgg{l}.b"] = _np(m.weight), _np(m.bias)
    for l, m in enumerate(lins):
        P[f"lin{l}.W"], P[f"lin{l}.b"] = _np(m.weight), _np(m.bias)
    x = rng.standard_normal((B, 3, L, Fq))
    y = enc.forward(cu(x))
    yr, cache = fo.vgg_fwd(x, P)
    assert y.shape == (B, (L - 8) // 2, 128)
    assert_rel(_np(y), yr, "y")
    dy = rng.standard_normal(yr.shape)
    enc.zeroGradParameters()
    enc.backward(cu(x), cu(dy), 1.0)
    G = {k: np.zeros_like(v) for k, v in P.items()}
    fo.vgg_bwd(P, cache, dy, G)
    torch.cuda.synchronize()
    pairs = []
    for l, m in enumerate(convs):
        pairs += [(f"dvgg{l}.W", m.gradWeight, G[f"vgg{l}.W"]), (f"dvgg{l}.b", m.gradBias, G[f"vgg{l}.b"])]
    for l, m in enumerate(lins):
        pairs += [(f"dlin{l}.W", m.gradWeight, G[f"lin{l}.W"]), (f"dlin{l}.b", m.gradBias, G[f"lin{l}.b"])]
    # default init: the conv weight gradients are sums that cancel to ~1e-3 of their terms, beyond what fp32
    # arithmetic of the reference algorithm itself reaches -- the bar per tensor is max(1e-4, 16 x the fp32
    # restatement's own error on these inputs) (tests/test_gpu_fullsize.py explains the floor)
    P32 = {k: v.astype(np.float32) for k, v in P.items()}
    _, cache32 = fo.vgg_fwd(x.astype(np.float32), P32)
    G32 = {k: np.zeros_like(v) for k, v in P32.items()}
    fo.vgg_bwd(P32, cache32, dy.astype(np.float32), G32)
    floor = {n: rel_err(G32[n[1:]], r) for n, _, r in pairs}
    errs = {n: rel_err(_np(g), r) for n, g, r in pairs}
    # (the escape is bounded: a floor above 1e-3 would mean the case itself is unjudgeable)
    uncapped = {n: f"{floor[n]:.1e}" for n in floor if not floor[n] <= 1e-3}
    assert not uncapped, uncapped
    bad = {n: f"{errs[n]:.2e} (fp32 floor {floor[n]:.2e})" for n in errs if not errs[n] <= max(RTOL, FLOOR_FACTOR * floor[n])}
    assert not bad, bad


# --------------------------------------------------------------------------- external decoder_mlp (VGG model)

def _mlp_layers(rng, dims, O):
    """librispeech/model_vgg.lua:71-77: Maxout(D, M, 7) -> Linear(M, M) -> Maxout(M, M, 7) -> Linear(M, O)."""
    D, M = dims
    L = []
    for kind, i, o in (("maxout", D, M), ("linear", M, M), ("maxout", M, M), ("linear", M, O)):
        if kind == "maxout":
            L.append(("maxout", rng.standard_normal((o * 7, i)) / np.sqrt(i), rng.standard_normal(o * 7) * 0.1, 7))
        else:
            L.append(("linear", rng.standard_normal((o, i)) / np.sqrt(i), rng.standard_normal(o) * 0.1))
    L.append(("logsoftmax",))
    return L


def test_oracle_vgg_step_under_its_own_decisions_is_unchanged():
    """The decision-adoption hooks of the VGG oracle (vgg_fwd / mlp_fwd decide / maxout_idx, used by the bf16
    config-5 test): adopting the oracle's own ReLU / max-pooling / Maxout decisions reproduces the plain step
    bit for bit, and raw reports the pre-decision values those decisions came from."""
    import vgg_case as vc
    P, layers, cfg = fo.vgg_random_case(F=24, hidden=64, out=32, S=16, Sc=24, O=9, M=8, seed=3, dtype=np.float64)
    rng = np.random.default_rng(3)
    x = rng.standard_normal((2, 3, 20, 24))
    labels = rng.integers(0, 9, (2, 5)).astype(np.int32)
    raw = {}
    nll, logp, G, mg = fo.vgg_model_step(x, labels, P, layers, cfg, raw=raw)
    decide = {"conv": [u > 0 for u in raw["conv"]], "lin": [u > 0 for u in raw["lin"]], "pool": dict(raw["pool"])}
    mx = [np.argmax(g, axis=2) for g in raw["mlp"]]
    assert len(raw["conv"]) == 4 and len(raw["lin"]) == 4 and sorted(raw["pool"]) == [1, 3] and len(mx) == 2
    raw2 = {}
    nll2, logp2, G2, mg2 = fo.vgg_model_step(x, labels, P, layers, cfg, decide, mx, raw2)
    assert np.array_equal(logp, logp2) and all(np.array_equal(G[k], G2[k]) for k in G)
    assert vc.decision_margins(decide, mx, raw2) == {k: (0, 0.0, 0.0, 0.0) for k in
                                                     ("conv0", "conv1", "conv2", "conv3", "lin0", "lin1", "lin2",
                                                      "lin3", "pool1", "pool3", "maxout0", "maxout1")}
    # one adopted flip (the smallest |u| of the last 1x1 layer) changes the step and is reported with its margin
    u = raw["lin"][3]
    k = np.unravel_index(np.argmin(np.abs(u)), u.shape)
    decide["lin"][3] = decide["lin"][3].copy()
    decide["lin"][3][k] = not decide["lin"][3][k]
    raw3 = {}
    _, logp3, _, _ = fo.vgg_model_step(x, labels, P, layers, cfg, decide, mx, raw3)
    m = vc.decision_margins(decide, mx, raw3)
    assert m["lin3"][0] == 1 and abs(m["lin3"][1] - 1.0 / u.size) < 1e-15
    assert abs(m["lin3"][2] - abs(u[k]) / np.abs(u).max()) < 1e-12
    # its local scale is the unit row (b, l) of the 1x1 layer's output
    assert abs(m["lin3"][3] - abs(u[k]) / np.abs(u[k[:-1]]).max()) < 1e-12 and m["lin3"][3] >= m["lin3"][2]
    assert not np.array_equal(logp, logp3)


def test_oracle_mlp_stack_matches_torch():
    rng = np.random.default_rng(21)
    layers = _mlp_layers(rng, (12, 5), 9)
    v = rng.standard_normal((6, 12))
    y, cache = fo.mlp_fwd(v, layers)
    dy = rng.standard_normal(y.shape)
    grads = [(np.zeros_like(L[1]), np.zeros_like(L[2])) if L[0] != "logsoftmax" else None for L in layers]
    dv = fo.mlp_bwd(layers, cache, dy, grads)
    vt = t64(v, True)
    ts = [(t64(L[1], True), t64(L[2], True)) if L[0] != "logsoftmax" else None for L in layers]
    h = vt
    for L, tw in zip(layers, ts):
        if L[0] == "maxout":
            u = h @ tw[0].T + tw[1]
            h = F.max_pool1d(u[:, None, :], L[3], L[3])[:, 0, :]
        elif L[0] == "linear":
            h = h @ tw[0].T + tw[1]
        else:
            h = torch.log_softmax(h, 1)
    h.backward(t64(dy))
    assert_rel(y, h.detach().numpy(), "y", 1e-12)
    assert_rel(dv, vt.grad.numpy(), "dv", 1e-12)
    for g, tw in zip(grads, ts):
        if g is not None:
            assert_rel(g[0], tw[0].grad.numpy(), "dW", 1e-12)
            assert_rel(g[1], tw[1].grad.numpy(), "db", 1e-12)


def test_oracle_external_mlp_equals_fused_chorowski_mlp():
    """attention_bwd with the decoder_mlp's input gradient injected (dmlp_in) == the fused Maxout ->
    Linear -> LogSoftMax path, when the external stack is that same MLP."""
    from oracle import s2s_oracle as orc
    rng = np.random.default_rng(22)
    cfg = orc.ModelConfig(inputFrameSize=8, hiddenFrameSize=16, outputFrameSize=8, scoreDepth=12, stateDepth=10,
                          outputDepth=7, mlpDepth=4, maxoutWindow=3, numLayers=1)
    P = orc.init_params(cfg, seed=3)
    B, L, T = 2, 9, 4
    h = rng.standard_normal((B, L, 16))
    labels = rng.integers(0, 7, (B, T))
    logp, cache = orc.attention_fwd(h, labels, P, cfg)
    dlogp = rng.standard_normal(logp.shape)
    G1 = orc.zeros_like_params(P)
    dh1 = orc.attention_bwd(P, cfg, cache, dlogp, G1)
    layers = [("maxout", P["Wm"], P["bm"], 3), ("linear", P["Wo"], P["bo"]), ("logsoftmax",)]
    v = cache["v"].reshape(B * T, -1)
    y, mc = fo.mlp_fwd(v, layers)
    assert_rel(y.reshape(B, T, -1), logp, "logp", 1e-12)
    grads = [(np.zeros_like(P["Wm"]), np.zeros_like(P["bm"])), (np.zeros_like(P["Wo"]), np.zeros_like(P["bo"])), None]
    dv = fo.mlp_bwd(layers, mc, dlogp.reshape(B * T, -1), grads)
    G2 = orc.zeros_like_params(P)
    dh2 = orc.attention_bwd(P, cfg, cache, None, G2, dmlp_in=dv.reshape(B, T, -1))
    assert_rel(dh2, dh1, "dh", 1e-12)
    for k in G1:
        if k not in ("Wm", "bm", "Wo", "bo"):
            assert_rel(G2[k], G1[k], k, 1e-12)
    assert_rel(grads[0][0], G1["Wm"], "Wm", 1e-12)
    assert_rel(grads[1][0], G1["Wo"], "Wo", 1e-12)


@pytest.mark.gpu
@pytest.mark.parametrize("B,L,T,A,Sc,S,O,M,K", [(8, 30, 6, 128, 128, 64, 29, 8, 7), (3, 17, 5, 64, 48, 32, 11, 4, 3)])
def test_external_mlp_attention_equals_fused(fe, B, L, T, A, Sc, S, O, M, K):
    """Attention with the decoder_mlp run outside (external_mlp) as Maxout -> Linear -> LogSoftMax modules
    equals the fused MaxoutMLP decoder on the same weights (XCD-local and per-step decoders)."""
    import s2s_amd
    torch.manual_seed(5)
    rng = np.random.default_rng(6)
    fused = s2s_amd.Attention(s2s_amd.GRU(S, S), s2s_amd.MaxoutMLP(S + A, M, K, O), Sc, 10, 0, S, A, O, True,
                              0.0).cuda()
    mlp = fe.Sequential(fe.Maxout(S + A, M, K), fe.Linear(M, O), fe.LogSoftMax())
    ext = s2s_amd.Attention(s2s_amd.GRU(S, S), mlp, Sc, 10, 0, S, A, O, True, 0.0).cuda()
    fw, _ = fused.parameters()
    ew, _ = ext.parameters()
    for a, b in zip(ew, fw):  # own (10) + recurrent (3), then Wm, bm, Wo, bo in the same order
        a.copy_(b)
    h = cu(rng.standard_normal((B, L, A)) * 0.5)
    lab = cu(rng.integers(0, O, (B, T)), torch.int32)
    dlogp = cu(rng.standard_normal((B, T, O)))
    outs = []
    for att in (fused, ext):
        logp = att.forward([h, lab]).clone()
        att.zeroGradParameters()
        dh = att.backward([h, None], dlogp, 0.5)[0].clone()
        outs.append([logp, dh] + [g.clone() for g in att.parameters()[1]])
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(outs[0], outs[1])):
        assert_rel(_np(b), _np(a), f"tensor {i}", 2e-5)


@pytest.mark.gpu
def test_vgg_attention_model_step_matches_oracle(fe):
    """librispeech/model_vgg.lua end to end (VGG encoder, GRU attention decoder, two-Maxout MLP) + the loss seed,
    reduced widths (1x1 layers 128, A = 128, S = 64, Sc = 128: the XCD-local decoder)."""
    import s2s_amd
    from oracle import s2s_oracle as orc
    torch.manual_seed(9)
    rng = np.random.default_rng(9)
    B, L, Fq, T, O, M = 2, 40, 40, 6, 29, 8
    model = s2s_amd.VGGAttentionModel(Fq, outputFrameSize=128, hidden=128, scoreDepth=128, stateDepth=64,
                                      outputDepth=O, mlpDepth=M).cuda()
    enc_mods = model.encoder.seq.modules
    # conditioning: at the default init the encoder output is bias-dominated (frames differ by ~1 % of
    # |h|, |h| ~ 0.1), so every score-path gradient (dwe, dWs, dV) is a sum whose terms cancel to
    # ~1e-3 of their size -- fp32-ill-conditioned for any implementation.  Zero biases and a larger
    # last layer give O(1) annotations that differ across frames.
    with torch.no_grad():
        for m in enc_mods:
            if getattr(m, "bias", None) is not None:
                m.bias.zero_()
        [m for m in enc_mods if isinstance(m, fe.TemporalConvolution)][-1].weight.mul_(20.0)
    P = {}
    for l, m in enumerate([m for m in enc_mods if isinstance(m, fe.SpatialConvolutionMM)]):
        P[f"vgg{l}.W"], P[f"vgg{l}.b"] = _np(m.weight), _np(m.bias)
    for l, m in enumerate([m for m in enc_mods if isinstance(m, fe.TemporalConvolution)]):
        P[f"lin{l}.W"], P[f"lin{l}.b"] = _np(m.weight), _np(m.bias)
    dec = model.decoder
    names = ("V", "Ws", "bs", "we", "Wy", "by", "Wc", "bc", "Wd", "bd", "dec.Wz", "dec.Wr", "dec.Wh")
    for n, t in zip(names, dec._tensors(False)[:13]):
        P[n] = _np(t)
    layers = []
    for m in dec.decoder_mlp.modules:
        if isinstance(m, fe.Maxout):
            layers.append(("maxout", _np(m.linear.weight), _np(m.linear.bias), m.window))
        elif isinstance(m, fe.Linear):
            layers.append(("linear", _np(m.weight), _np(m.bias)))
        else:
            layers.append(("logsoftmax",))
    cfg = orc.ModelConfig(inputFrameSize=8, hiddenFrameSize=16, outputFrameSize=64, scoreDepth=128, stateDepth=64,
                          outputDepth=O, mlpDepth=M, maxoutWindow=7, numLayers=1)
    x = rng.standard_normal((B, 3, L, Fq)) * 10
    labels = np.append(rng.integers(0, O - 1, (B, T - 1)), np.full((B, 1), O - 1), axis=1).astype(np.int32)
    model.zeroGradParameters()
    nll, logp = model.step(cu(x), cu(labels, torch.int32))
    torch.cuda.synchronize()
    nll_r, logp_r, G, mg = fo.vgg_model_step(x, labels, P, layers, cfg)
    assert_rel(_np(logp), logp_r, "logp")
    assert_rel(_np(nll), nll_r, "nll")
    pairs = []
    for l, m in enumerate([m for m in enc_mods if isinstance(m, fe.SpatialConvolutionMM)]):
        pairs += [(f"dvgg{l}.W", m.gradWeight, G[f"vgg{l}.W"]), (f"dvgg{l}.b", m.gradBias, G[f"vgg{l}.b"])]
    for l, m in enumerate([m for m in enc_mods if isinstance(m, fe.TemporalConvolution)]):
        pairs += [(f"dlin{l}.W", m.gradWeight, G[f"lin{l}.W"]), (f"dlin{l}.b", m.gradBias, G[f"lin{l}.b"])]
    for n, g in zip(names, dec._tensors(True)[:13]):
        pairs.append(("d" + n, g, G[n]))
    mods = [m for m in dec.decoder_mlp.modules if not isinstance(m, fe.LogSoftMax)]
    for i, (m, g) in enumerate(zip(mods, [g for g in mg if g is not None])):
        lin = m.linear if isinstance(m, fe.Maxout) else m
        pairs += [(f"dmlp{i}.W", lin.gradWeight, g[0]), (f"dmlp{i}.b", lin.gradBias, g[1])]
    _assert_grads(pairs)


@pytest.mark.gpu
@pytest.mark.parametrize("prec", ["fp32", "bf16-all"])
def test_vgg_graph_step_equals_eager(fe, prec):
    """VGGAttentionModel.graph_step (the config-5 bench's captured step) is bitwise the eager
    zeroGradParameters() + step(), also after the inputs are refilled in place (new data, one capture)."""
    import s2s_amd
    rng = np.random.default_rng(4)
    B, L, Fq, T, O = 2, 40, 40, 6, 29

    def make():
        return s2s_amd.VGGAttentionModel(Fq, outputFrameSize=128, hidden=128, scoreDepth=128, stateDepth=64,
                                         outputDepth=O, mlpDepth=8, generator=torch.Generator().manual_seed(3),
                                         precision=prec).cuda()

    eager, graphed = make(), make()
    x = cu(rng.standard_normal((B, 3, L, Fq)) * 10)
    labels = cu(np.append(rng.integers(0, O - 1, (B, T - 1)), np.full((B, 1), O - 1), axis=1), torch.int32)
    xg, lg = x.clone(), labels.clone()
    for it in range(3):
        if it == 2:  # new data in the captured buffers
            x.copy_(cu(rng.standard_normal((B, 3, L, Fq)) * 10))
            xg.copy_(x)
        eager.zeroGradParameters()
        nll_e, logp_e = eager.step(x, labels)
        nll_g, logp_g = graphed.graph_step(xg, lg)
        torch.cuda.synchronize()
        assert torch.equal(logp_e, logp_g) and torch.equal(nll_e, nll_g), it
        for i, (ge, gg) in enumerate(zip(eager.parameters()[1], graphed.parameters()[1])):
            assert torch.equal(ge, gg), (it, i)
    assert len(graphed._graphs) == 1


@pytest.mark.gpu
def test_vgg_graph_step_keeps_big_gemm_path(fe):
    """At full width (1x1 layers 2048) the VGG model's big products run on the big-tile bf16 GEMM (gemm_bf16.hip),
    whose staging buffer is per stream and cannot be allocated inside a capture: graph_step's eager warm-up runs on
    the capture stream, so the captured step takes the same kernels as the eager one (same number of big-GEMM
    calls) and the replay is bitwise the eager step."""
    import ctypes
    import s2s_amd
    from s2s_amd import _lib
    calls = _lib.lib.s2s_debug_gemm_big_calls
    calls.restype = ctypes.c_long
    rng = np.random.default_rng(14)
    B, L, Fq, T, O = 2, 256, 40, 20, 29

    def make():
        return s2s_amd.VGGAttentionModel(Fq, outputFrameSize=512, hidden=2048, outputDepth=O,
                                         generator=torch.Generator().manual_seed(4), precision="bf16-all").cuda()

    eager, graphed = make(), make()
    x = cu(rng.standard_normal((B, 3, L, Fq)))
    labels = cu(np.append(rng.integers(0, O - 1, (B, T - 1)), np.full((B, 1), O - 1), axis=1), torch.int32)
    n0 = calls()
    eager.zeroGradParameters()
    nll_e, logp_e = eager.step(x, labels)
    torch.cuda.synchronize()
    per_step = calls() - n0
    assert per_step > 0
    n1 = calls()
    nll_g, logp_g = graphed.graph_step(x.clone(), labels.clone())  # eager warm-up + capture (+ replay)
    torch.cuda.synchronize()
    assert calls() - n1 == 2 * per_step, (calls() - n1, per_step)
    assert torch.equal(logp_e, logp_g) and torch.equal(nll_e, nll_g)
    for i, (ge, gg) in enumerate(zip(eager.parameters()[1], graphed.parameters()[1])):
        assert torch.equal(ge, gg), i


@pytest.mark.gpu
def test_conv_bilstm_graph_step_equals_eager(fe):
    """ConvBiLSTMAttentionModel.graph_step (timit/timit.lua:106-145: LSTM decoder, hybrid attention, per-step
    decoder kernels) is bitwise the eager zeroGradParameters() + step(), also with new data in the captured
    buffers."""
    import s2s_amd
    rng = np.random.default_rng(8)
    B, L, D, T, O = 3, 64, 20, 7, 11

    def make():
        return s2s_amd.ConvBiLSTMAttentionModel(D, numPhonemes=O, hiddenFrameSize=32, outputFrameSize=16, stateDepth=48,
                                                scoreDepth=30, penalty=0.1, generator=torch.Generator().manual_seed(2)).cuda()

    eager, graphed = make(), make()
    x = cu(rng.standard_normal((B, L, D)))
    labels = cu(rng.integers(0, O, (B, T)), torch.int32)
    xg, lg = x.clone(), labels.clone()
    for it in range(3):
        if it == 2:
            x.copy_(cu(rng.standard_normal((B, L, D))))
            xg.copy_(x)
        eager.zeroGradParameters()
        nll_e, logp_e = eager.step(x, labels)
        nll_g, logp_g = graphed.graph_step(xg, lg)
        torch.cuda.synchronize()
        assert torch.equal(logp_e, logp_g) and torch.equal(nll_e, nll_g), it
        for i, (ge, gg) in enumerate(zip(eager.parameters()[1], graphed.parameters()[1])):
            assert torch.equal(ge, gg), (it, i)


@pytest.mark.gpu
@pytest.mark.parametrize("model,graph", [("convlstm", False), ("convlstm", True), ("vgg", True)])
def test_param_grads_beside_the_backward_are_bitwise_serial(fe, model, graph):
    """overlap_param_grads (s2s_ctx_set_wgrad_overlap: the Attention, LSTM and TemporalConvolution parameter
    gradients on the context's side stream beside the next module's backward -- the model steps' default) gives
    bitwise the serial step's outputs and gradients, eager and captured: timit.lua's conv + BiLSTM model at its
    widths (the XCD-local LSTM decoder) and a small VGG model (GRU decoder, external MLP)."""
    import s2s_amd
    rng = np.random.default_rng(21)
    if model == "convlstm":
        B, T, O = 8, 12, 62
        shape = (B, 160, 123)

        def make(ov):
            m = s2s_amd.ConvBiLSTMAttentionModel(generator=torch.Generator().manual_seed(5), penalty=0.1).cuda()
            m.overlap = ov
            return m
    else:
        B, T, O = 2, 6, 29
        shape = (B, 3, 40, 40)

        def make(ov):
            m = s2s_amd.VGGAttentionModel(40, outputFrameSize=128, hidden=128, scoreDepth=128, stateDepth=64,
                                          outputDepth=O, mlpDepth=8, generator=torch.Generator().manual_seed(3)).cuda()
            m.overlap = ov
            return m
    ser, ovl = make(False), make(True)
    x = cu(rng.standard_normal(shape))
    labels = cu(rng.integers(0, O, (B, T)), torch.int32)
    for it in range(3):
        ser.zeroGradParameters()
        nll_s, logp_s = ser.step(x, labels)
        if graph:
            nll_o, logp_o = ovl.graph_step(x, labels)
        else:
            ovl.zeroGradParameters()
            nll_o, logp_o = ovl.step(x, labels)
        torch.cuda.synchronize()
        assert torch.equal(logp_s, logp_o) and torch.equal(nll_s, nll_o), it
        for i, (a, b) in enumerate(zip(ser.parameters()[1], ovl.parameters()[1])):
            assert torch.equal(a, b), (it, i)


@pytest.mark.gpu
def test_lstm_fwd_bwd_one_graph_replays(fe):
    """BiRNN(LSTM) forward + backward captured in ONE graph equals the eager pair on every replay (the backward's
    carries used to be cleared by hipMemsetAsync, whose graph node left the previous replay's values in place from
    the second replay on; the library clears with fill kernels now)."""
    import s2s_amd
    rng = np.random.default_rng(11)
    B, L, D, H = 3, 6, 32, 16
    x = cu(rng.standard_normal((B, L, D)))
    gy = cu(rng.standard_normal((B, L, 2 * H)))

    def make():
        return s2s_amd.BiRNN(s2s_amd.LSTM(D, H, False, torch.Generator().manual_seed(1)),
                             s2s_amd.LSTM(D, H, False, torch.Generator().manual_seed(2))).cuda()

    def fn(m):
        m.zeroGradParameters()
        y = m.forward(x)
        return y, m.backward(x, gy, 0.5)

    eager, graphed = make(), make()
    fn(graphed)
    torch.cuda.synchronize()
    graph, side = torch.cuda.CUDAGraph(), torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.graph(graph, stream=side, capture_error_mode="thread_local"):
        yg, dxg = fn(graphed)
    torch.cuda.current_stream().wait_stream(side)
    for it in range(3):
        ye, dxe = fn(eager)
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(ye, yg) and torch.equal(dxe, dxg), it
        for i, (ge, gg) in enumerate(zip(eager.parameters()[1], graphed.parameters()[1])):
            assert torch.equal(ge, gg), (it, i)


# --------------------------------------------------------------------------- LSTM decoder (conv + BiLSTM model)

def _lstm_dec_case(rng, S, A, Sc, O, hybrid, mlp_kind):
    """Decoder parameters of the timit/timit.lua:126-145 model family: LSTM(S, S) decoder_recurrent,
    hybrid location-aware attention, and either the fused Maxout MLP or an external ReLU MLP."""
    from oracle import s2s_oracle as orc
    kW, nF = hybrid
    cfg = orc.ModelConfig(inputFrameSize=8, hiddenFrameSize=16, outputFrameSize=A // 2, scoreDepth=Sc, stateDepth=S,
                          outputDepth=O, mlpDepth=4, maxoutWindow=3, numLayers=1, hybridAttendFilterSize=kW,
                          hybridAttendFeatureMaps=nF, decoderLSTM=True)
    P = {"V": rng.standard_normal((Sc, A)) * 0.2, "Ws": rng.standard_normal((Sc, S)) * 0.2,
         "bs": rng.standard_normal(Sc) * 0.1, "we": rng.standard_normal((1, Sc)) * 0.3,
         "Wy": rng.standard_normal((S, O)) * 0.3, "by": rng.standard_normal(S) * 0.1,
         "Wc": rng.standard_normal((S, A)) * 0.2, "bc": rng.standard_normal(S) * 0.1,
         "Wd": rng.standard_normal((S, 2 * S)) * 0.2, "bd": rng.standard_normal(S) * 0.1,
         "Wm": rng.standard_normal((4 * 3, S + A)) * 0.2, "bm": rng.standard_normal(12) * 0.1,
         "Wo": rng.standard_normal((O, 4)) * 0.3, "bo": rng.standard_normal(O) * 0.1}
    if nF:
        P.update({"hybW": rng.standard_normal((nF, kW)) * 0.3, "hybb": rng.standard_normal(nF) * 0.1,
                  "hybU": rng.standard_normal((Sc, nF)) * 0.3})
    for q in "ifgo":
        P[f"dec.W{q}x"] = rng.standard_normal((S, S)) * 0.2
        P[f"dec.b{q}x"] = rng.standard_normal(S) * 0.1
        P[f"dec.W{q}h"] = rng.standard_normal((S, S)) * 0.2
        P[f"dec.b{q}h"] = rng.standard_normal(S) * 0.1
    return cfg, P


def test_oracle_lstm_decoder_finite_differences():
    from oracle import s2s_oracle as orc
    rng = np.random.default_rng(31)
    cfg, P = _lstm_dec_case(rng, 6, 8, 5, 7, (5, 3), "maxout")
    B, L, T = 2, 9, 4
    h = rng.standard_normal((B, L, 8))
    labels = rng.integers(0, 7, (B, T))
    logp, cache = orc.attention_fwd(h, labels, P, cfg)
    dl = rng.standard_normal(logp.shape)
    G = {k: np.zeros_like(v) for k, v in P.items()}
    dh = orc.attention_bwd(P, cfg, cache, dl, G)
    eps = 1e-6
    for key in ("dec.Wix", "dec.bfh", "dec.Wgx", "dec.Woh", "Wd", "hybW", "Ws"):
        for _ in range(2):
            i = tuple(rng.integers(0, n) for n in P[key].shape)
            old = P[key][i]
            P[key][i] = old + eps
            fp = (orc.attention_fwd(h, labels, P, cfg)[0] * dl).sum()
            P[key][i] = old - eps
            fm = (orc.attention_fwd(h, labels, P, cfg)[0] * dl).sum()
            P[key][i] = old
            assert abs((fp - fm) / (2 * eps) - G[key][i]) <= 1e-6 * max(1.0, abs(G[key][i])), key
    i = (1, 3, 2)
    old = h[i]
    h[i] = old + eps
    fp = (orc.attention_fwd(h, labels, P, cfg)[0] * dl).sum()
    h[i] = old - eps
    fm = (orc.attention_fwd(h, labels, P, cfg)[0] * dl).sum()
    h[i] = old
    assert abs((fp - fm) / (2 * eps) - dh[i]) <= 1e-6


def _load_lstm_attention(s2s, fe, P, cfg, mlp):
    S, A, Sc, O = cfg.stateDepth, cfg.annotationDepth, cfg.scoreDepth, cfg.outputDepth
    cell = s2s.LSTM(S, S, peepholes=False)
    att = s2s.Attention(cell, mlp, Sc, cfg.hybridAttendFilterSize, cfg.hybridAttendFeatureMaps, S, A, O, True,
                        cfg.penalty)
    with torch.no_grad():
        for n in ("V", "Ws", "bs", "we", "Wy", "by", "Wc", "bc", "Wd", "bd") + (("hybW", "hybb", "hybU")
                                                                                if cfg.hybridAttendFeatureMaps else ()):
            att.own[n].copy_(torch.tensor(P[n]))
        for n, t in cell.named().items():
            t.copy_(torch.tensor(P["dec." + n]))
        if isinstance(mlp, s2s.MaxoutMLP):
            for t, n in zip(mlp.weight, ("Wm", "bm", "Wo", "bo")):
                t.copy_(torch.tensor(P[n]))
    return att.cuda(), cell


@pytest.mark.gpu
@pytest.mark.parametrize("B,L,T,S,A,Sc,O,hyb", [(4, 30, 6, 32, 64, 48, 11, (5, 16)), (3, 20, 5, 64, 32, 16, 62, (0, 0))])
def test_lstm_decoder_matches_oracle(fe, B, L, T, S, A, Sc, O, hyb):
    """decoder_recurrent = LSTM(S, S) (timit/timit.lua:137) with the fused Maxout MLP, hybrid attention on/off."""
    import s2s_amd
    from oracle import s2s_oracle as orc
    rng = np.random.default_rng(B * 100 + L)
    cfg, P = _lstm_dec_case(rng, S, A, Sc, O, hyb, "maxout")
    att, cell = _load_lstm_attention(s2s_amd, fe, P, cfg, s2s_amd.MaxoutMLP(S + A, 4, 3, O))
    h = rng.standard_normal((B, L, A)) * 0.5
    labels = rng.integers(0, O, (B, T)).astype(np.int32)
    logp = att.forward([cu(h), cu(labels, torch.int32)])
    lref, cache = orc.attention_fwd(h, labels, P, cfg)
    assert_rel(_np(logp), lref, "logp")
    dl = rng.standard_normal(lref.shape)
    att.zeroGradParameters()
    dh = att.backward([cu(h), None], cu(dl), 0.5)[0]
    G = {k: np.zeros_like(v) for k, v in P.items()}
    dhr = orc.attention_bwd(P, cfg, cache, dl, G, 0.5)
    torch.cuda.synchronize()
    pairs = [("dh", dh, dhr)]
    for n in ("V", "Ws", "bs", "we", "Wy", "by", "Wc", "bc", "Wd", "bd") + (("hybW", "hybb", "hybU") if hyb[1] else ()):
        pairs.append(("d" + n, att.own_grad[n], G[n]))
    for n, g in cell.named(grads=True).items():
        pairs.append(("d" + n, g, G["dec." + n]))
    for t, n in zip(att.decoder_mlp.gradWeight, ("Wm", "bm", "Wo", "bo")):
        pairs.append(("d" + n, t, G[n]))
    _assert_grads(pairs)


@pytest.mark.gpu
def test_conv_bilstm_model_decoder_external_relu_mlp(fe):
    """The timit/timit.lua:126-145 decoder as built there: LSTM(S, S) recurrence, hybrid attention (kW = 5,
    nF = 16), decoder_mlp = Linear(S+A, 2*O) -> ReLU -> Linear(2*O, O) -> LogSoftMax (external_mlp)."""
    import s2s_amd
    from oracle import s2s_oracle as orc
    rng = np.random.default_rng(41)
    B, L, T, S, A, Sc, O = 3, 14, 6, 32, 64, 48, 11
    cfg, P = _lstm_dec_case(rng, S, A, Sc, O, (5, 16), "relu")
    mlp = fe.Sequential(fe.Linear(S + A, 2 * O), fe.ReLU(), fe.Linear(2 * O, O), fe.LogSoftMax())
    att, cell = _load_lstm_attention(s2s_amd, fe, P, cfg, mlp)
    lins = [m for m in mlp.modules if isinstance(m, fe.Linear)]
    layers = [("linear", _np(lins[0].weight), _np(lins[0].bias)), ("relu",),
              ("linear", _np(lins[1].weight), _np(lins[1].bias)), ("logsoftmax",)]
    h = rng.standard_normal((B, L, A)) * 0.5
    labels = rng.integers(0, O, (B, T)).astype(np.int32)
    logp = att.forward([cu(h), cu(labels, torch.int32)])
    _, cache = orc.attention_fwd(h, labels, P, cfg)
    lref, mc = fo.mlp_fwd(cache["v"].reshape(B * T, -1), layers)
    assert_rel(_np(logp), lref.reshape(B, T, O), "logp")
    dl = rng.standard_normal((B, T, O))
    att.zeroGradParameters()
    dh = att.backward([cu(h), None], cu(dl), 1.0)[0]
    mg = [(np.zeros_like(Lr[1]), np.zeros_like(Lr[2])) if Lr[0] == "linear" else None for Lr in layers]
    dv = fo.mlp_bwd(layers, mc, dl.reshape(B * T, O), mg)
    G = {k: np.zeros_like(v) for k, v in P.items()}
    dhr = orc.attention_bwd(P, cfg, cache, None, G, dmlp_in=dv.reshape(B, T, -1))
    torch.cuda.synchronize()
    pairs = [("dh", dh, dhr)]
    for n in ("V", "Ws", "bs", "we", "Wy", "by", "Wc", "bc", "Wd", "bd", "hybW", "hybb", "hybU"):
        pairs.append(("d" + n, att.own_grad[n], G[n]))
    for n, g in cell.named(grads=True).items():
        pairs.append(("d" + n, g, G["dec." + n]))
    pairs += [("dmlp0.W", lins[0].gradWeight, mg[0][0]), ("dmlp0.b", lins[0].gradBias, mg[0][1]),
              ("dmlp2.W", lins[1].gradWeight, mg[2][0]), ("dmlp2.b", lins[1].gradBias, mg[2][1])]
    _assert_grads(pairs)


@pytest.mark.gpu
def test_conv_bilstm_attention_model_step_matches_oracle(fe):
    """timit/timit.lua:106-145 end to end (conv + BiLSTM encoder, LSTM decoder with hybrid attention, ReLU
    decoder_mlp, loss seed) at reduced widths; scoreDepth 20 (not a multiple of 16, like the reference's
    150) runs on zero-padded score channels."""
    import s2s_amd
    from oracle import s2s_oracle as orc
    torch.manual_seed(13)
    rng = np.random.default_rng(13)
    B, L, D, T, O = 3, 60, 20, 5, 11
    model = s2s_amd.ConvBiLSTMAttentionModel(D, numPhonemes=O, hiddenFrameSize=32, outputFrameSize=16, stateDepth=32,
                                             scoreDepth=20).cuda()
    enc, dec = model.encoder, model.decoder
    P = {}
    convs = [m for m in enc.convlayer.modules if isinstance(m, fe.TemporalConvolution)]
    for l, m in enumerate(convs):
        P[f"conv{l}.W"], P[f"conv{l}.b"] = _np(m.weight), _np(m.bias)
    for pre, c in zip(("f.", "b."), enc.rnn.cells):
        for k, v in c.named().items():
            P[pre + k] = _np(v)
    Pd = {n: _np(t) for n, t in dec.own.items()}
    for n, t in dec.decoder_recurrent.named().items():
        Pd["dec." + n] = _np(t)
    S, A, Sc = 32, 32, 20
    for name, shp in (("Wm", (3, S + A)), ("bm", (3,)), ("Wo", (O, 1)), ("bo", (O,))):
        Pd[name] = np.zeros(shp)
    cfg = orc.ModelConfig(inputFrameSize=8, hiddenFrameSize=16, outputFrameSize=A // 2, scoreDepth=Sc, stateDepth=S,
                          outputDepth=O, mlpDepth=1, maxoutWindow=3, numLayers=1, hybridAttendFilterSize=5,
                          hybridAttendFeatureMaps=16, decoderLSTM=True)
    lins = [m for m in dec.decoder_mlp.modules if isinstance(m, fe.Linear)]
    layers = [("linear", _np(lins[0].weight), _np(lins[0].bias)), ("relu",),
              ("linear", _np(lins[1].weight), _np(lins[1].bias)), ("logsoftmax",)]
    pools = [m for m in enc.convlayer.modules if isinstance(m, fe.TemporalMaxPooling)]
    x = rng.standard_normal((B, L, D)).astype(np.float32).astype(np.float64)
    labels = rng.integers(0, O, (B, T)).astype(np.int32)
    model.zeroGradParameters()
    nll, logp = model.step(cu(x), cu(labels, torch.int32))
    torch.cuda.synchronize()
    # oracle: encoder, decoder with the external MLP, loss seed, backward (timit/timit.lua:262-295)
    h, ecache = fo.conv_bilstm_fwd(x, P)
    _, acache = orc.attention_fwd(h, labels, Pd, cfg)
    lref, mc = fo.mlp_fwd(acache["v"].reshape(B * T, -1), layers)
    lref = lref.reshape(B, T, O)
    onehot = np.zeros_like(lref)
    np.put_along_axis(onehot, labels[..., None].astype(np.int64), 1.0, axis=2)
    assert_rel(_np(logp), lref, "logp")
    assert_rel(_np(nll), -(onehot * lref).sum((1, 2)), "nll")
    sc = 1.0 / B
    mg = [(np.zeros_like(Lr[1]), np.zeros_like(Lr[2])) if Lr[0] == "linear" else None for Lr in layers]
    dv = fo.mlp_bwd(layers, mc, -onehot.reshape(B * T, O), mg, sc)
    Gd = {k: np.zeros_like(v) for k, v in Pd.items()}
    dh = orc.attention_bwd(Pd, cfg, acache, None, Gd, sc, dmlp_in=dv.reshape(B, T, -1))
    Ge = {k: np.zeros_like(v) for k, v in P.items()}
    _adopt_conv_decisions(convs, pools, ecache[1])
    fo.conv_bilstm_bwd(P, ecache, dh, Ge, sc)
    pairs = []
    for l, m in enumerate(convs):
        pairs += [(f"dconv{l}.W", m.gradWeight, Ge[f"conv{l}.W"]), (f"dconv{l}.b", m.gradBias, Ge[f"conv{l}.b"])]
    for pre, c in zip(("f.", "b."), enc.rnn.cells):
        pairs += [(f"d{pre}{k}", g, Ge[pre + k]) for k, g in c.named(grads=True).items()]
    for n, g in dec.own_grad.items():
        pairs.append(("d" + n, g, Gd[n]))
    for n, g in dec.decoder_recurrent.named(grads=True).items():
        pairs.append(("ddec." + n, g, Gd["dec." + n]))
    pairs += [("dmlp0.W", lins[0].gradWeight, mg[0][0]), ("dmlp2.W", lins[1].gradWeight, mg[2][0]),
              ("dmlp2.b", lins[1].gradBias, mg[2][1])]
    _assert_grads(pairs)


# --------------------------------------------------------------------------- beam search, every decoder variant

def _check_beam(att, h, P, cfg, eos, K, maxlen, mlp=None):
    """decoder:BeamSearch on the device vs the oracle's per-utterance search (Attention.lua:332-438).  A
    hypothesis may flip only at an fp32-vs-fp64 near tie, so a differing prediction must score (teacher-forced,
    oracle) within 1e-4 of the oracle's best; the reported score equals the oracle's rescoring of the GPU's
    own prediction."""
    from oracle import s2s_oracle as orc
    B = h.shape[0]
    toks, lens, scores = att.BeamSearch(cu(h), eos, K, maxlen)
    toks, lens, scores = toks.cpu().numpy(), lens.cpu().numpy(), scores.cpu().numpy()

    def rescore(b, seq):
        st, Vh, tot, y = orc.decoder_zero_state(h.shape[1], cfg.stateDepth), h[b] @ P["V"].T, 0.0, -1
        for tok in seq:
            lp, st = orc.decoder_step(h[b], Vh, st, y, P, cfg, mlp)
            tot, y = tot + lp[tok], tok
        return tot

    agree = 0
    for b in range(B):
        seq = [int(t) for t in toks[b, :lens[b]]]
        assert all(t == -1 for t in toks[b, lens[b]:])
        assert seq[-1] == eos or len(seq) == maxlen + 1
        ref_seq, ref_score = orc.beam_search(h[b], P, cfg, eos, K, maxlen, mlp=mlp)
        mine = rescore(b, seq)
        assert abs(mine - scores[b]) <= 1e-4 * max(1.0, abs(mine)), (b, mine, scores[b])
        if seq == list(ref_seq):
            agree += 1
        else:
            assert mine >= ref_score - 1e-4 * max(1.0, abs(ref_score)), (b, seq, ref_seq, mine, ref_score)
    assert agree >= B - 1
    return toks, lens


@pytest.mark.gpu
@pytest.mark.parametrize("hyb,K,maxlen", [((5, 16), 4, 10), ((0, 0), 3, 8), ((5, 16), 1, 6)])
def test_beam_search_lstm_decoder_matches_oracle(fe, hyb, K, maxlen):
    """BeamSearch with the timit/timit.lua:137 LSTM decoder_recurrent (the cell carried per hypothesis) and
    hybrid location-aware attention (alpha_{t-1} carried), fused Maxout MLP."""
    import s2s_amd
    rng = np.random.default_rng(K * 10 + maxlen)
    B, L, S, A, Sc, O, eos = 5, 24, 32, 64, 48, 11, 2
    cfg, P = _lstm_dec_case(rng, S, A, Sc, O, hyb, "maxout")
    att, _ = _load_lstm_attention(s2s_amd, fe, P, cfg, s2s_amd.MaxoutMLP(S + A, 4, 3, O))
    h = rng.standard_normal((B, L, A)) * 1.5
    toks, lens = _check_beam(att, h, P, cfg, eos, K, maxlen)
    one = att.BeamSearch(cu(h[1]), eos, K, maxlen).cpu().numpy()
    assert list(one) == list(toks[1, :lens[1]])


@pytest.mark.gpu
def test_beam_search_gru_hybrid_matches_oracle(fe):
    """BeamSearch with the Chorowski GRU decoder and hybrid attention (kW = 5, nF = 8)."""
    import s2s_amd
    from oracle import s2s_oracle as orc
    torch.manual_seed(3)
    rng = np.random.default_rng(17)
    B, L, S, A, Sc, O, M, Kw, eos = 4, 26, 32, 64, 64, 13, 4, 3, 3
    cfg = orc.ModelConfig(inputFrameSize=8, hiddenFrameSize=16, outputFrameSize=A // 2, scoreDepth=Sc, stateDepth=S,
                          outputDepth=O, mlpDepth=M, maxoutWindow=Kw, numLayers=1, hybridAttendFilterSize=5,
                          hybridAttendFeatureMaps=8)
    att = s2s_amd.Attention(s2s_amd.GRU(S, S), s2s_amd.MaxoutMLP(S + A, M, Kw, O), Sc, 5, 8, S, A, O, True,
                            0.0).cuda()
    with torch.no_grad():
        att.own["hybU"].mul_(4.0)  # location features visibly steer the scores
    P = {n: _np(t) for n, t in att.own.items()}
    P.update({f"dec.W{g}": _np(t) for g, t in zip("zrh", att.decoder_recurrent.weight)})
    P.update({n: _np(t) for n, t in zip(("Wm", "bm", "Wo", "bo"), att.decoder_mlp.weight)})
    h = rng.standard_normal((B, L, A)) * 1.5
    _check_beam(att, h, P, cfg, eos, 4, 9)


@pytest.mark.gpu
def test_beam_search_external_mlp_matches_oracle(fe):
    """BeamSearch of the timit/timit.lua:126-145 decoder as built there: LSTM recurrence, hybrid attention, and the
    external decoder_mlp Linear -> ReLU -> Linear -> LogSoftMax run between the search's step and advance calls."""
    import s2s_amd
    rng = np.random.default_rng(43)
    B, L, S, A, Sc, O, eos = 4, 20, 32, 64, 48, 11, 2
    cfg, P = _lstm_dec_case(rng, S, A, Sc, O, (5, 16), "relu")
    mlp = fe.Sequential(fe.Linear(S + A, 2 * O), fe.ReLU(), fe.Linear(2 * O, O), fe.LogSoftMax())
    att, _ = _load_lstm_attention(s2s_amd, fe, P, cfg, mlp)
    lins = [m for m in mlp.modules if isinstance(m, fe.Linear)]
    layers = [("linear", _np(lins[0].weight), _np(lins[0].bias)), ("relu",),
              ("linear", _np(lins[1].weight), _np(lins[1].bias)), ("logsoftmax",)]
    ext = lambda v: fo.mlp_fwd(v[None], layers)[0][0]  # noqa: E731
    h = rng.standard_normal((B, L, A)) * 1.5
    _check_beam(att, h, P, cfg, eos, 3, 8, mlp=ext)


@pytest.mark.gpu
@pytest.mark.parametrize("K", [2, 3, 4])
def test_beam_search_keeps_K_hypotheses_from_the_first_step(fe, K):
    """Attention.lua:369-387: the first step (one zero-state row) seeds all K hypotheses, eos among them
    finishing at once.  Swept over maxseqlength so an eos ranked k-th at step 0 and ties in later
    selections both come up (this case's utterance 1 finishes on eos at step 0 for K = 4)."""
    import s2s_amd
    from oracle import s2s_oracle as orc
    torch.manual_seed(3)
    rng = np.random.default_rng(17)
    B, L, S, A, Sc, O, M, Kw, eos = 4, 26, 32, 64, 64, 13, 4, 3, 3
    cfg = orc.ModelConfig(inputFrameSize=8, hiddenFrameSize=16, outputFrameSize=A // 2, scoreDepth=Sc, stateDepth=S,
                          outputDepth=O, mlpDepth=M, maxoutWindow=Kw, numLayers=1, hybridAttendFilterSize=5,
                          hybridAttendFeatureMaps=8)
    att = s2s_amd.Attention(s2s_amd.GRU(S, S), s2s_amd.MaxoutMLP(S + A, M, Kw, O), Sc, 5, 8, S, A, O, True,
                            0.0).cuda()
    with torch.no_grad():
        att.own["hybU"].mul_(4.0)
    P = {n: _np(t) for n, t in att.own.items()}
    P.update({f"dec.W{g}": _np(t) for g, t in zip("zrh", att.decoder_recurrent.weight)})
    P.update({n: _np(t) for n, t in zip(("Wm", "bm", "Wo", "bo"), att.decoder_mlp.weight)})
    h = rng.standard_normal((B, L, A)) * 1.5
    for maxlen in (1, 2, 3, 5, 8):
        _check_beam(att, h, P, cfg, eos, K, maxlen)


@pytest.mark.gpu
def test_host_parameters_are_refused_not_launched(fe):
    """A module whose parameters are still host tensors (no .cuda()) must raise before any launch: the kernels
    take raw device pointers and a host pointer would fault on the GPU."""
    import s2s_amd
    conv = fe.SpatialConvolutionMM(1, 4, 5, 1)
    with pytest.raises(s2s_amd.nn.S2SArgumentError, match="cuda"):
        conv.forward(torch.ones(1, 10, 5, device="cuda"))
    rnn = s2s_amd.RNN(s2s_amd.GRU(8, 16))
    with pytest.raises(s2s_amd.nn.S2SArgumentError, match="cuda"):
        rnn.forward(torch.ones(2, 5, 8, device="cuda"))


def _timit_lstm_dec_case(rng, S, A, Sc, O, kW, nF):
    """timit/timit.lua:127-155's decoder parameters at the reference's default init scale (U(+-1/sqrt(fan_in)) ->
    standard deviation 1/sqrt(3 fan_in)), in the oracle's dict layout."""
    from oracle import s2s_oracle as orc
    cfg = orc.ModelConfig(inputFrameSize=8, hiddenFrameSize=16, outputFrameSize=A // 2, scoreDepth=Sc, stateDepth=S,
                          outputDepth=O, mlpDepth=4, maxoutWindow=3, numLayers=1, hybridAttendFilterSize=kW,
                          hybridAttendFeatureMaps=nF, decoderLSTM=True)

    def u(shape, fan):
        return rng.uniform(-1.0, 1.0, shape) / np.sqrt(fan)
    P = {"V": u((Sc, A), A), "Ws": u((Sc, S), S), "bs": u(Sc, S), "we": u((1, Sc), Sc), "Wy": u((S, O), O),
         "by": u(S, O), "Wc": u((S, A), A), "bc": u(S, A), "Wd": u((S, 2 * S), 2 * S), "bd": u(S, 2 * S),
         "Wm": u((12, S + A), S + A), "bm": u(12, S + A), "Wo": u((O, 4), 4), "bo": u(O, 4),
         "hybW": u((nF, kW), kW), "hybb": u(nF, kW), "hybU": u((Sc, nF), nF)}
    for q in "ifgo":
        P[f"dec.W{q}x"], P[f"dec.b{q}x"] = u((S, S), S), u(S, S)
        P[f"dec.W{q}h"], P[f"dec.b{q}h"] = u((S, S), S), u(S, S)
    return cfg, P


@pytest.mark.gpu
@pytest.mark.parametrize("B,L,T,pen", [(32, 62, 12, 0.0), (25, 62, 10, 0.3)])
def test_timit_lstm_hybrid_decoder_xcd_matches_oracle(fe, B, L, T, pen):
    """The timit/timit.lua:127-155 decoder at the reference's own shape -- LSTM(400, 400) decoder_recurrent, scoreDepth
    150 (run on 160 zero-padded channels), hybrid attention kW = 5 / 16 maps, annotations 2 x 128, external ReLU
    decoder_mlp, 62 phonemes, the 62 annotation frames of a 512-frame utterance -- runs on the XCD-local LSTM kernels
    (dec_xcd_lstm.inc; the live kernel profile names them: B = 32 is 8 chains of 4 utterances, B = 25 leaves a last
    chain of one), and every output and gradient matches the float64 oracle at the 1e-4 bar (MonotonicAlignment
    decisions adopted as in tests/test_gpu_parity.py) and the per-step launches (s2s_debug_dec_mode(1)) to 1e-4, the
    oracle bar itself: the folded c -> d -> gates products and the chunked sums reassociate, and the score layer's
    cancelling sums (dbs, dWs, the hybrid fold's dhybb / dhybU) differ by up to 8.8e-5 with the penalty on; every other
    tensor agrees to ~1e-6."""
    import ctypes
    import s2s_amd
    from oracle import s2s_oracle as orc
    from s2s_amd import _lib
    from s2s_amd import profile as prof
    S, A, Sc, O, kW, nF = 400, 256, 150, 62, 5, 16
    rng = np.random.default_rng(B * 10 + T)
    cfg, P = _timit_lstm_dec_case(rng, S, A, Sc, O, kW, nF)
    cfg.penalty = pen
    mlp = fe.Sequential(fe.Linear(S + A, 2 * O), fe.ReLU(), fe.Linear(2 * O, O), fe.LogSoftMax())
    att, cell = _load_lstm_attention(s2s_amd, fe, P, cfg, mlp)
    lins = [m for m in mlp.modules if isinstance(m, fe.Linear)]
    layers = [("linear", _np(lins[0].weight), _np(lins[0].bias)), ("relu",),
              ("linear", _np(lins[1].weight), _np(lins[1].bias)), ("logsoftmax",)]
    h = rng.standard_normal((B, L, A)) * 0.5
    labels = rng.integers(0, O, (B, T)).astype(np.int32)
    dl = rng.standard_normal((B, T, O))
    mode = _lib.lib.s2s_debug_dec_mode
    mode.argtypes = [ctypes.c_int]

    def run():
        logp = att.forward([cu(h), cu(labels, torch.int32)]).clone()
        ind = att.mono_ind().clone() if pen > 0 else None
        att.zeroGradParameters()
        dh = att.backward([cu(h), None], cu(dl), 1.0)[0].clone()
        torch.cuda.synchronize()
        grads = [t.clone() for t in list(att.own_grad.values()) + list(cell.named(grads=True).values())]
        return logp, dh, grads, ind

    _lib.check(_lib.lib.s2s_prof_enable(1))
    try:
        prof.collect()
        logp, dh, grads, ind = run()
        ran = prof.collect()
    finally:
        _lib.lib.s2s_prof_enable(0)
    assert "dec_fwd_xcd_lstm" in ran and "dec_bwd_xcd_lstm" in ran, sorted(ran)
    _, cache = orc.attention_fwd(h, labels, P, cfg)
    if pen > 0:  # adopt the GPU's MonotonicAlignment decisions where the statistic is within fp32 noise of 0
        gi = _np(ind)
        a = cache["alpha"]
        prev = np.concatenate([np.zeros_like(a[:, :1]), a[:, :-1]], 1)
        stat = ((L - np.arange(L))[None, None, :] * (a - prev)).sum(-1)
        clear = np.abs(stat) > 1e-4
        assert np.array_equal(gi[clear], cache["mono_ind"][clear]), "MonotonicAlignment decisions differ"
        cache["mono_ind"] = gi
    lref, mc = fo.mlp_fwd(cache["v"].reshape(B * T, -1), layers)
    assert_rel(_np(logp), lref.reshape(B, T, O), "logp")
    mg = [(np.zeros_like(Lr[1]), np.zeros_like(Lr[2])) if Lr[0] == "linear" else None for Lr in layers]
    dv = fo.mlp_bwd(layers, mc, dl.reshape(B * T, O), mg)
    G = {k: np.zeros_like(v) for k, v in P.items()}
    dhr = orc.attention_bwd(P, cfg, cache, None, G, dmlp_in=dv.reshape(B, T, -1))
    names = list(att.own_grad.keys()) + ["dec." + n for n in cell.named(grads=True)]
    pairs = [("dh", dh, dhr)] + [("d" + n, g, G[n]) for n, g in zip(names, grads) if n in G]
    _assert_grads(pairs)
    # the per-step launches on the same inputs
    mode(1)
    try:
        logp_s, dh_s, grads_s, _ = run()
    finally:
        mode(-1)
    diffs = {"logp": rel_err(_np(logp), _np(logp_s)), "dh": rel_err(_np(dh), _np(dh_s))}
    diffs.update({"d" + n: rel_err(_np(g), _np(gs)) for n, g, gs in zip(names, grads, grads_s)})
    print("XCD-local vs per-step launches, max rel diff:", {k: f"{v:.1e}" for k, v in diffs.items()})
    bad = {k: f"{v:.2e}" for k, v in diffs.items() if not v <= 1e-4}
    assert not bad, bad
