"""GPU parity: libs2s_hip.so (through the C ABI / the host mirror) against the CPU oracle.

Tolerance (fp32 vs the oracle's float64): for every output / gradient tensor,
max|gpu - ref| <= RTOL * max|ref| with RTOL = 1e-4 (BASELINE.json north star: "outputs
within 1e-4 rel of the Torch7 CPU reference").
"""
import numpy as np
import pytest
import torch

from oracle import s2s_oracle as orc

pytestmark = pytest.mark.gpu
RTOL = 1e-4


def rel_err(g, r):
    g = np.asarray(g, dtype=np.float64)
    r = np.asarray(r, dtype=np.float64)
    assert g.shape == r.shape, (g.shape, r.shape)
    denom = max(np.abs(r).max(), 1e-30)
    return float(np.abs(g - r).max() / denom)


def assert_rel(g, r, name, rtol=RTOL, atol_zero=1e-7):
    assert np.isfinite(g).all(), f"{name}: non-finite values"
    if np.abs(np.asarray(r, dtype=np.float64)).max() == 0.0:
        # an exactly-zero reference (e.g. every attention gradient of a one-frame utterance: softmax over
        # one frame is constant) has no relative scale: fp32 rounding residue must stay absolutely tiny
        a = float(np.abs(np.asarray(g, dtype=np.float64)).max())
        assert a <= atol_zero, f"{name}: reference is exactly 0, max |gpu| {a:.3e} > {atol_zero:.0e}"
        return
    e = rel_err(g, r)
    assert e <= rtol, f"{name}: max rel err {e:.3e} > {rtol:.0e}"


@pytest.fixture(scope="module")
def s2s():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import s2s_amd
    return s2s_amd


def cu(a, dtype=torch.float32):
    return torch.tensor(np.ascontiguousarray(a), dtype=dtype, device="cuda")


# --------------------------------------------------------------------------- GRU layer

@pytest.mark.parametrize("B,L,D,H", [(3, 7, 20, 32), (5, 16, 123, 64), (17, 9, 64, 16)])
@pytest.mark.parametrize("bidir", [False, True])
def test_gru_layer_matches_oracle(s2s, B, L, D, H, bidir):
    rng = np.random.default_rng(B * 100 + L)
    x = rng.standard_normal((B, L, D))
    cells = [s2s.GRU(D, H) for _ in range(2 if bidir else 1)]
    Ws = [[w.double().numpy() for w in c.weight] for c in cells]
    if bidir:
        mod = s2s.BiRNN(cells[0], cells[1])
    else:
        mod = s2s.RNN(cells[0], reverse=(L % 2 == 1))
    mod.cuda()
    xs = cu(x)
    y = mod.forward(xs).cpu().numpy()
    dy = rng.standard_normal(y.shape)
    mod.zeroGradParameters()
    dx = mod.backward(xs, cu(dy), 0.5).cpu().numpy()
    torch.cuda.synchronize()
    revs = [False, True] if bidir else [mod.reverse]
    dx_ref = np.zeros_like(x)
    for i, (W, rev) in enumerate(zip(Ws, revs)):
        yr, sv = orc.gru_seq_fwd(x, W[0], W[1], W[2], rev)
        assert_rel(y[:, :, i * H:(i + 1) * H], yr, f"y[{i}]")
        G = {k: np.zeros_like(v) for k, v in zip(("Wz", "Wr", "Wh"), W)}
        dxr, _ = orc.gru_seq_bwd(x, W[0], W[1], W[2], sv, dy[:, :, i * H:(i + 1) * H], G, rev, 0.5)
        dx_ref += dxr
        for k, g in zip(("Wz", "Wr", "Wh"), cells[i].gradWeight):
            assert_rel(g.cpu().numpy(), G[k], f"d{k}[{i}]")
    assert_rel(dx, dx_ref, "dx")


def test_gru_single_utterance_2d(s2s):
    """2-D input = the reference's SGD mode (RNN.lua:122-124)."""
    rng = np.random.default_rng(0)
    cell = s2s.GRU(12, 16)
    mod = s2s.RNN(cell, reverse=True).cuda()
    x = rng.standard_normal((6, 12))
    y = mod.forward(cu(x)).cpu().numpy()
    W = [w.cpu().double().numpy() for w in cell.weight]
    yr, _ = orc.gru_seq_fwd(x[None], *W, True)
    assert y.shape == (6, 16)
    assert_rel(y, yr[0], "y")


# --------------------------------------------------------------------------- LSTM layer (§8 A7)

@pytest.mark.parametrize("B,L,D,H", [(3, 7, 20, 32), (17, 9, 64, 16), (5, 12, 40, 48)])
@pytest.mark.parametrize("bidir", [False, True])
@pytest.mark.parametrize("peep", [False, True])
def test_lstm_layer_matches_oracle(s2s, B, L, D, H, bidir, peep):
    """nn.RNN(nn.LSTM(D, H, peepholes)) fwd + BPTT through s2s_lstm_{fwd,bwd} vs the oracle
    (LSTM.lua:16-58, 118-136): y, dx and every weight / bias gradient (accumulated, scale 0.5)."""
    rng = np.random.default_rng(B * 1000 + L * 10 + H)
    x = rng.standard_normal((B, L, D))
    cells = [s2s.LSTM(D, H, peepholes=peep) for _ in range(2 if bidir else 1)]
    Ps = [{k: v.double().numpy() for k, v in c.named().items()} for c in cells]
    mod = s2s.BiRNN(cells[0], cells[1]) if bidir else s2s.RNN(cells[0], reverse=(L % 2 == 1))
    mod.cuda()
    xs = cu(x)
    y = mod.forward(xs).cpu().numpy()
    dy = rng.standard_normal(y.shape)
    mod.zeroGradParameters()
    for c in cells:  # gradients accumulate onto what is already there
        for g in c.gradWeight:
            g.fill_(0.25)
    dx = mod.backward(xs, cu(dy), 0.5).cpu().numpy()
    torch.cuda.synchronize()
    revs = [False, True] if bidir else [mod.reverse]
    dx_ref = np.zeros_like(x)
    for i, (P, rev) in enumerate(zip(Ps, revs)):
        yr, sv = orc.lstm_seq_fwd(x, P, rev, peep)
        assert_rel(y[:, :, i * H:(i + 1) * H], yr, f"y[{i}]")
        G = {k: np.full_like(v, 0.25) for k, v in P.items()}
        dx_ref += orc.lstm_seq_bwd(x, P, sv, dy[:, :, i * H:(i + 1) * H], G, rev, peep, 0.5)
        for k, g in cells[i].named(grads=True).items():
            assert_rel(g.cpu().numpy(), G[k], f"d{k}[{i}]")
    assert_rel(dx, dx_ref, "dx")


@pytest.mark.parametrize("local", [1, 0])
@pytest.mark.parametrize("B,L,D,H", [(32, 14, 256, 128), (5, 9, 40, 64), (20, 31, 64, 128)])
def test_persistent_lstm_matches_oracle_and_per_step(s2s, monkeypatch, local, B, L, D, H):
    """The persistent BiLSTM layer (lstm_persist.hip: the whole sweep of both directions in one launch, one
    hand-off seam per step; XCD-local sentinel slots when local=1, tagged granules when 0) -- at the conv + BiLSTM
    encoder's shape (timit/timit.lua:108-125: 256 conv maps in, 128 units per direction, 14 frames after the conv
    stack) and two ragged ones -- against the oracle (1e-4) and bit for bit against the per-step launches
    (S2S_LSTM_MODE=step: the same chunk order and partial sums), over repeated launches."""
    import ctypes
    from s2s_amd import _lib
    knob = _lib.lib.s2s_debug_lstm_local
    knob.argtypes = [ctypes.c_int]
    rng = np.random.default_rng(B * 100 + L)
    x = rng.standard_normal((B, L, D))
    cells = [s2s.LSTM(D, H, peepholes=False) for _ in range(2)]
    Ps = [{k: v.double().numpy() for k, v in c.named().items()} for c in cells]
    dyn = rng.standard_normal((B, L, 2 * H))
    from s2s_amd import profile as prof
    outs, ran = {}, {}
    knob(local)
    try:
        for mode in ("step", "persistent"):
            monkeypatch.setenv("S2S_LSTM_MODE", mode)
            mod = s2s.BiRNN(cells[0], cells[1]).cuda()
            res = []
            _lib.check(_lib.lib.s2s_prof_enable(1))
            prof.collect()
            for rep in range(2):
                y = mod.forward(cu(x)).clone()
                mod.zeroGradParameters()
                dx = mod.backward(cu(x), cu(dyn), 0.5).clone()
                res.append((y, dx, [g.clone() for c in cells for g in c.named(grads=True).values()]))
            torch.cuda.synchronize()
            ran[mode] = prof.collect()
            _lib.lib.s2s_prof_enable(0)
            outs[mode] = res
    finally:
        _lib.lib.s2s_prof_enable(0)
        knob(1)
    assert "lstm_fwd_persist" in ran["persistent"] and "lstm_bwd_persist" in ran["persistent"], sorted(ran["persistent"])
    assert "lstm_fwd_steps" in ran["step"] and "lstm_fwd_persist" not in ran["step"], sorted(ran["step"])
    for rep in range(2):
        a, b = outs["step"][rep], outs["persistent"][rep]
        assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1]), rep
        for i, (ga, gb) in enumerate(zip(a[2], b[2])):
            assert torch.equal(ga, gb), (rep, i)
    y, dx, grads = outs["persistent"][0]
    y, dx = y.cpu().numpy(), dx.cpu().numpy()
    dx_ref = np.zeros_like(x)
    gi = 0
    for i, (P, rev) in enumerate(zip(Ps, (False, True))):
        yr, sv = orc.lstm_seq_fwd(x, P, rev, False)
        assert_rel(y[:, :, i * H:(i + 1) * H], yr, f"y[{i}]")
        G = {k: np.zeros_like(v) for k, v in P.items()}
        dx_ref += orc.lstm_seq_bwd(x, P, sv, dyn[:, :, i * H:(i + 1) * H], G, rev, False, 0.5)
        for k in cells[i].named(grads=True):
            assert_rel(grads[gi].cpu().numpy(), G[k], f"d{k}[{i}]")
            gi += 1
    assert_rel(dx, dx_ref, "dx")


# --------------------------------------------------------------------------- attention decoder

ATT_CASES = [
    # B, L, T, A, Sc, S, O, M, K, penalty
    (3, 20, 5, 32, 48, 32, 7, 4, 3, 0.0),
    (4, 33, 6, 64, 64, 48, 29, 8, 7, 0.0),
    (2, 16, 4, 32, 32, 16, 5, 3, 2, 0.25),
    (19, 8, 3, 16, 16, 16, 62, 5, 7, 0.0),
    # shapes served by the persistent decoder kernels (S=64, A=128, Sc=128), ragged B and L
    (5, 37, 6, 128, 128, 64, 29, 4, 7, 0.3),
    (18, 16, 4, 128, 128, 64, 62, 8, 7, 0.0),
]


@pytest.mark.parametrize("B,L,T,A,Sc,S,O,M,K,pen", ATT_CASES)
def test_attention_decoder_matches_oracle(s2s, B, L, T, A, Sc, S, O, M, K, pen):
    _check_attention(s2s, B, L, T, A, Sc, S, O, M, K, pen)


# shapes served by the XCD-local decoder kernels (dec_xcd.inc): chains of U utterances on one XCD;
# U = 8 (4 chunks of 32 frames), ragged last chain, U = 4 (7 chunks), penalty on
XCD_CASES = [
    (32, 128, 12, 512, 512, 256, 62, 8, 7, 0.0),
    (21, 50, 9, 128, 128, 64, 29, 4, 7, 0.2),
    (5, 200, 7, 128, 128, 64, 29, 4, 7, 0.0),
    (3, 20, 5, 128, 128, 64, 11, 4, 3, 0.0),
    # edge shapes: one utterance of one frame and one label; one label per utterance, ragged chain
    (1, 1, 1, 128, 128, 64, 11, 4, 3, 0.0),
    (9, 3, 1, 512, 512, 256, 62, 8, 7, 0.0),
]


@pytest.mark.parametrize("local", [1, 0])
@pytest.mark.parametrize("B,L,T,A,Sc,S,O,M,K,pen", XCD_CASES)
def test_xcd_decoder_matches_oracle(s2s, B, L, T, A, Sc, S, O, M, K, pen, local):
    """XCD-local decoder (folded Wx' = W_d Wd_c Wc, L2-resident granule hand-offs when local=1 and
    the census finds each chain on one XCD; write-through sc1 hand-offs when local=0)."""
    import ctypes
    from s2s_amd import _lib
    fn = _lib.lib.s2s_debug_dec_local
    fn.argtypes = [ctypes.c_int]
    fn(local)
    try:
        _check_attention(s2s, B, L, T, A, Sc, S, O, M, K, pen)
    finally:
        fn(1)


# chunks too long for LDS residency (> 32 frames): h / Vh rows streamed from global memory each step
XCD_STREAM_CASES = [
    (32, 400, 6, 512, 512, 256, 29, 8, 7, 0.0),
    (21, 500, 5, 128, 128, 64, 29, 4, 7, 0.2),
]


@pytest.mark.parametrize("B,L,T,A,Sc,S,O,M,K,pen", XCD_STREAM_CASES)
def test_xcd_decoder_streamed_chunks_match_oracle(s2s, B, L, T, A, Sc, S, O, M, K, pen):
    """LibriSpeech-length utterances (config 4: L = 400) on the XCD-local decoder with streamed chunks."""
    _check_attention(s2s, B, L, T, A, Sc, S, O, M, K, pen)


@pytest.mark.parametrize("B,L,T,A,Sc,S,O", [(32, 128, 12, 512, 512, 256, 62), (21, 50, 9, 128, 128, 64, 29)])
def test_xcd_decoder_streamed_bitwise_equals_resident(s2s, monkeypatch, B, L, T, A, Sc, S, O):
    """The streamed-chunk kernels do the resident kernels' arithmetic in the same order: bitwise equal."""
    rng = np.random.default_rng(4)
    att = s2s.Attention(s2s.GRU(S, S), s2s.MaxoutMLP(S + A, 8, 7, O), Sc, 10, 0, S, A, O, True, 0.2).cuda()
    h = cu(rng.standard_normal((B, L, A)) * 0.5)
    labels = cu(rng.integers(0, O, (B, T)), torch.int32)
    dlogp = cu(rng.standard_normal((B, T, O)))
    outs = {}
    for stream in ("2", "0", "1"):  # resident (default at these shapes), no residency, Vh-only
        monkeypatch.setenv("S2S_DEC_STREAM", stream)
        logp = att.forward([h, labels]).clone()
        att.zeroGradParameters()
        dh = att.backward([h, None], dlogp)[0].clone()
        outs[stream] = [logp, dh] + [g.clone() for g in att.parameters()[1]]
    torch.cuda.synchronize()
    for mode in ("0", "1"):
        for i, (a, b) in enumerate(zip(outs["2"], outs[mode])):
            assert torch.equal(a, b), f"mode {mode} tensor {i} differs: max |d| = {(a - b).abs().max().item():.3e}"


def _check_attention(s2s, B, L, T, A, Sc, S, O, M, K, pen, kW=10, nF=0):
    rng = np.random.default_rng(L * 7 + T)
    torch.manual_seed(L * 7 + T)  # module init draws from torch's generator
    cfg = orc.ModelConfig(inputFrameSize=8, hiddenFrameSize=16, outputFrameSize=A // 2, scoreDepth=Sc, stateDepth=S,
                          outputDepth=O, mlpDepth=M, maxoutWindow=K, penalty=pen, numLayers=1,
                          hybridAttendFilterSize=kW if nF else 0, hybridAttendFeatureMaps=nF)
    dec_gru = s2s.GRU(S, S)
    mlp = s2s.MaxoutMLP(S + A, M, K, O)
    att = s2s.Attention(dec_gru, mlp, Sc, kW, nF, S, A, O, True, pen).cuda()
    P = {n: t.cpu().double().numpy() for n, t in zip(
        ("V", "Ws", "bs", "we", "Wy", "by", "Wc", "bc", "Wd", "bd", "dec.Wz", "dec.Wr", "dec.Wh", "Wm", "bm", "Wo",
         "bo", "hybW", "hybb", "hybU"), att.parameters()[0])}
    h = rng.standard_normal((B, L, A)) * 0.5
    labels = rng.integers(0, O, (B, T)).astype(np.int32)
    hs = cu(h)
    logp = att.forward([hs, cu(labels, torch.int32)]).cpu().numpy()
    lref, cache = orc.attention_fwd(h, labels, P, cfg)
    assert_rel(logp, lref, "logp")
    assert_rel(att.alpha().cpu().numpy(), cache["alpha"], "alpha")
    if pen > 0:
        _adopt_mono_decisions(att, cache, L)
    dlogp = rng.standard_normal(logp.shape)
    att.zeroGradParameters()
    dh = att.backward([hs, None], cu(dlogp), 0.5)[0].cpu().numpy()
    G = orc.zeros_like_params(P)
    dhr = orc.attention_bwd(P, cfg, cache, dlogp, G, 0.5)
    assert_rel(dh, dhr, "dh")
    for name, g in zip(P.keys(), att.parameters()[1]):
        assert_rel(g.cpu().numpy(), G[name], "d" + name)


@pytest.mark.parametrize("B,L,T,A,Sc,S,O,M,K,pen,kW,nF", [
    (3, 37, 7, 32, 48, 32, 11, 4, 3, 0.0, 5, 6),      # the reference's fallback filter (timit.lua:129-130), ragged chunk
    (2, 20, 6, 32, 32, 16, 9, 3, 2, 0.3, 4, 3),       # even filter (pads kW/2 left, kW/2-1 right), penalty on
    (4, 128, 12, 512, 512, 256, 62, 8, 7, 0.0, 5, 16),  # Chorowski sizes with hybrid features on
])
def test_hybrid_attention_matches_oracle(s2s, B, L, T, A, Sc, S, O, M, K, pen, kW, nF):
    """Hybrid location-aware attention (Attention.lua:75-98): UF = TCZB(nF, Sc, 1)(
    TemporalConvolution(1, nF, kW)(pad(alpha_{t-1}))) added to the scores; the backward carries
    d alpha_{t-1} into the previous step's softmax.  Per-step kernels vs the oracle (itself pinned by
    torch autograd and finite differences), forward, dh and every gradient incl. the conv's."""
    _check_attention(s2s, B, L, T, A, Sc, S, O, M, K, pen, kW, nF)


def _adopt_mono_decisions(att, cache, L, margin=1e-4):
    """MonotonicAlignment's gradient depends on the discrete decisions 1[penalty_t > 0]
    (MonotonicAlignment.lua:27-39, 44-77).  Their statistic sum_l (L-l)(alpha_t - alpha_{t-1}) sits
    within fp32 noise of 0 whenever attention barely moves between steps (typical of random weights),
    where any fp32 implementation -- the reference's CudaTensor path too -- may decide differently from
    the float64 oracle.  Require the GPU's decisions to agree wherever the statistic is clear of 0,
    then run the oracle's backward under the GPU's decisions."""
    gi = att.mono_ind().cpu().numpy().astype(np.float64)
    a = cache["alpha"]
    prev = np.concatenate([np.zeros_like(a[:, :1]), a[:, :-1]], 1)
    stat = ((L - np.arange(L))[None, None, :] * (a - prev)).sum(-1)
    clear = np.abs(stat) > margin
    assert np.array_equal(gi[clear], cache["mono_ind"][clear]), "MonotonicAlignment decisions differ"
    cache["mono_ind"] = gi


@pytest.mark.parametrize("injected", [True, False])
def test_attention_dropout_matches_oracle(s2s, injected):
    """Decoder MLP with nn.Dropout(p) in front (timit/model_chorowski_baseline_dropout.lua:56):
    injected masks, or masks drawn in-kernel (Bernoulli(1-p)/(1-p) statistics checked, then the
    oracle run with the mask the GPU used)."""
    B, L, T, A, Sc, S, O, M, K, p = 32, 128, 12, 512, 512, 256, 62, 8, 7, 0.5
    rng = np.random.default_rng(17)
    torch.manual_seed(17)
    cfg = orc.ModelConfig(inputFrameSize=8, hiddenFrameSize=16, outputFrameSize=A // 2, scoreDepth=Sc, stateDepth=S,
                          outputDepth=O, mlpDepth=M, maxoutWindow=K, numLayers=1)
    att = s2s.Attention(s2s.GRU(S, S), s2s.MaxoutMLP(S + A, M, K, O, dropout=p), Sc, 10, 0, S, A, O, True,
                        0.0).cuda()
    P = {n: t.cpu().double().numpy() for n, t in zip(
        ("V", "Ws", "bs", "we", "Wy", "by", "Wc", "bc", "Wd", "bd", "dec.Wz", "dec.Wr", "dec.Wh", "Wm", "bm", "Wo",
         "bo"), att.parameters()[0])}
    h = rng.standard_normal((B, L, A)) * 0.5
    labels = rng.integers(0, O, (B, T)).astype(np.int32)
    if injected:
        mask = (rng.random((B, T, S + A)) >= p) / (1.0 - p)
        att.dropout_mask = cu(mask)
    logp = att.forward([cu(h), cu(labels, torch.int32)]).cpu().numpy()
    used = att.dropout_mask_used().cpu().double().numpy()
    if injected:
        assert np.array_equal(used, mask.astype(np.float32).astype(np.float64))
    else:
        vals = np.unique(used)
        assert set(vals.tolist()) <= {0.0, float(np.float32(1.0 / (1.0 - p)))}, vals[:5]
        assert abs((used == 0).mean() - p) < 0.01
        mask = used
    lref, cache = orc.attention_fwd(h, labels, P, cfg, mask)
    assert_rel(logp, lref, "logp")
    dlogp = rng.standard_normal(logp.shape)
    att.zeroGradParameters()
    dh = att.backward([cu(h), None], cu(dlogp), 1.0)[0].cpu().numpy()
    G = orc.zeros_like_params(P)
    dhr = orc.attention_bwd(P, cfg, cache, dlogp, G, 1.0, mask)
    assert_rel(dh, dhr, "dh")
    for name, g in zip(P.keys(), att.parameters()[1]):
        assert_rel(g.cpu().numpy(), G[name], "d" + name)
    # evaluate(): nn.Dropout is the identity
    att.evaluate()
    logp_eval = att.forward([cu(h), cu(labels, torch.int32)]).cpu().numpy()
    lref0, _ = orc.attention_fwd(h, labels, P, cfg)
    assert_rel(logp_eval, lref0, "logp (evaluate)")


def test_model_step_dropout_config3(s2s):
    """BASELINE config 3 class: model_chorowski_baseline_dropout.lua (p = 0.5), B = 64, injected
    masks (L, T reduced so the float64 oracle stays in seconds)."""
    kw = dict(dropout=0.5)
    B, L, T = 64, 48, 16
    cfg_o = orc.ModelConfig()
    model = s2s.ChorowskiBaseline(s2s.ModelConfig(**kw))
    P = orc.unflatten(model.params.cpu().double().numpy(), cfg_o)
    x, labels = orc.synthetic_batch(cfg_o, B, L, T, seed=3, pad=10, eos=23)
    rng = np.random.default_rng(4)
    mask = (rng.random((B, T, cfg_o.stateDepth + 2 * cfg_o.outputFrameSize)) >= 0.5) / 0.5
    nll, logp = model.step(cu(x), cu(labels, torch.int32), dropout_mask=cu(mask))
    torch.cuda.synchronize()
    nll_ref, G, lref, enc = orc.training_step(x, labels, P, cfg_o, dropout_mask=mask)
    assert_rel(logp.cpu().numpy(), lref, "logp")
    Gg = orc.unflatten(model.grads.cpu().double().numpy(), cfg_o)
    for k in G:
        assert_rel(Gg[k], G[k], "grad " + k)


def test_model_step_dropout_back_to_back_steps(s2s):
    """Config 3 trains with a fresh in-kernel dropout seed every step (timit.lua's nn.Dropout draws
    new masks per forward).  A graph-mode context replays one graph and reads each step's seed from a
    device word (a per-step re-capture crashed the runtime intermittently): many steps back to back
    without a host sync complete, a repeated seed reproduces its step bitwise and a new seed changes
    the masks."""
    B, L, T = 16, 32, 8
    cfg_o = orc.ModelConfig()
    model = s2s.ChorowskiBaseline(s2s.ModelConfig(dropout=0.5), graph=True, overlap=True)
    x, labels = orc.synthetic_batch(cfg_o, B, L, T, seed=5, pad=4, eos=23)
    xg, lg = cu(x), cu(labels, torch.int32)
    stream = torch.cuda.Stream()
    with torch.cuda.stream(stream):
        for _ in range(12):
            model.step(xg, lg, stream=stream)
        _, a = model.step(xg, lg, stream=stream, dropout_seed=7)
        a = a.clone()
        _, b = model.step(xg, lg, stream=stream, dropout_seed=7)
        b = b.clone()
        _, c = model.step(xg, lg, stream=stream, dropout_seed=8)
    stream.synchronize()
    assert torch.isfinite(a).all()
    assert torch.equal(a, b)
    assert not torch.equal(a, c)


def test_labelmask_input_equals_int_labels(s2s):
    rng = np.random.default_rng(5)
    B, L, T, A, Sc, S, O = 2, 12, 4, 32, 32, 16, 9
    att = s2s.Attention(s2s.GRU(S, S), s2s.MaxoutMLP(S + A, 4, 3, O), Sc, 10, 0, S, A, O, True, 0.0).cuda()
    h = cu(rng.standard_normal((B, L, A)))
    labels = rng.integers(0, O, (B, T))
    mask = np.zeros((B, T, O), np.float32)
    np.put_along_axis(mask, labels[..., None], 1.0, 2)
    a = att.forward([h, cu(labels, torch.int32)]).clone()
    b = att.forward([h, cu(mask)])
    assert torch.equal(a, b)


# --------------------------------------------------------------------------- whole training step

def _model_case(s2s, cfg_kw, B, L, T, seed=1234, graph=False, overlap=False):
    cfg_o = orc.ModelConfig(**cfg_kw)
    model = s2s.ChorowskiBaseline(s2s.ModelConfig(**cfg_kw), graph=graph, overlap=overlap)
    P = orc.unflatten(model.params.cpu().double().numpy(), cfg_o)
    x, labels = orc.synthetic_batch(cfg_o, B, L, T, seed=seed, pad=min(10, L // 4), eos=min(23, cfg_o.outputDepth - 1))
    return cfg_o, model, P, x, labels


def _check_step(model, cfg_o, P, x, labels, stream=None, nll=None, logp=None):
    """One step (or the given step outputs nll / logp) against the float64 oracle."""
    if logp is None:
        nll, logp = model.step(cu(x), cu(labels, torch.int32), stream=stream)
    torch.cuda.synchronize()
    nll_ref, G, lref, enc = orc.training_step(x, labels, P, cfg_o)
    assert_rel(logp.cpu().numpy(), lref, "logp")
    assert_rel(model.encoder_output().cpu().numpy(), enc, "encoder.output")
    assert abs(float(nll.mean()) - nll_ref) <= RTOL * abs(nll_ref)
    Gg = orc.unflatten(model.grads.cpu().double().numpy(), cfg_o)
    for k in G:
        assert_rel(Gg[k], G[k], "grad " + k)


def test_model_step_small(s2s):
    kw = dict(inputFrameSize=20, hiddenFrameSize=32, outputFrameSize=32, scoreDepth=48, stateDepth=32,
              outputDepth=11, mlpDepth=6, maxoutWindow=3, numLayers=2)
    cfg_o, model, P, x, labels = _model_case(s2s, kw, 5, 24, 7)
    _check_step(model, cfg_o, P, x, labels)


@pytest.mark.parametrize("B,L,T", [(1, 4, 1), (1, 1, 3), (2, 3, 2), (33, 6, 2)])
def test_model_step_degenerate_shapes(s2s, B, L, T):
    """Edge shapes of the reference's per-utterance trainer: one utterance (its SGD mode), a single
    frame, a single output label, and a ragged last chain (B = 33)."""
    kw = dict(inputFrameSize=20, hiddenFrameSize=32, outputFrameSize=32, scoreDepth=48, stateDepth=32,
              outputDepth=11, mlpDepth=6, maxoutWindow=3, numLayers=2)
    cfg_o = orc.ModelConfig(**kw)
    model = s2s.ChorowskiBaseline(s2s.ModelConfig(**kw))
    P = orc.unflatten(model.params.cpu().double().numpy(), cfg_o)
    rng = np.random.default_rng(B * 100 + L * 10 + T)
    x = rng.standard_normal((B, L, 20))
    labels = rng.integers(0, 11, (B, T)).astype(np.int32)
    _check_step(model, cfg_o, P, x, labels)


def test_model_step_chorowski_config2(s2s):
    """BASELINE config 2 at full size: B=32, L=128, T=40, F=123, 3x BiGRU(256), Sc=512, O=62."""
    cfg_o, model, P, x, labels = _model_case(s2s, {}, 32, 128, 40)
    _check_step(model, cfg_o, P, x, labels)


def test_model_step_config2_dims_b45_graph(s2s):
    """Config-2 model at B=45 under graph replay with the side stream, as the bench runs it: three 16-row
    tiles (the last ragged), 6 of the 8 chain slots used, so the persistent launches' spare slots are 2
    chains wide -- one-step x-projection / dy / dh slices with 45 of 64 producer rows valid, the split-K
    start with 32 producers, the sync-region hand-over -- against the float64 oracle."""
    cfg_o, model, P, x, labels = _model_case(s2s, {}, 45, 64, 20, seed=5, graph=True, overlap=True)
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    xs, ls = cu(x), cu(labels, torch.int32)
    with torch.cuda.stream(st):
        for _ in range(2):  # capture, then a replay
            nll, logp = model.step(xs, ls, stream=st)
    st.synchronize()
    _check_step(model, cfg_o, P, x, labels, nll=nll, logp=logp)


def test_model_step_librispeech_shape(s2s):
    """config 4 shape class (F=80, O=29 chars), reduced L/T so the oracle stays in seconds."""
    kw = dict(inputFrameSize=80, outputDepth=29)
    cfg_o, model, P, x, labels = _model_case(s2s, kw, 4, 100, 30, seed=7)
    _check_step(model, cfg_o, P, x, labels)


def test_model_step_graph_replay_bitwise(s2s):
    kw = dict(inputFrameSize=20, hiddenFrameSize=32, outputFrameSize=32, scoreDepth=48, stateDepth=32,
              outputDepth=11, mlpDepth=6, maxoutWindow=3, numLayers=2)
    cfg_o, model, P, x, labels = _model_case(s2s, kw, 4, 20, 6, graph=True)
    st = torch.cuda.Stream()
    xs, ls = cu(x), cu(labels, torch.int32)
    with torch.cuda.stream(st):
        outs = []
        for _ in range(3):
            nll, logp = model.step(xs, ls, stream=st)
            outs.append((nll.clone(), logp.clone(), model.grads.clone()))
    st.synchronize()
    for o in outs[1:]:
        for a, b in zip(outs[0], o):
            assert torch.equal(a, b)
    eager = s2s.ChorowskiBaseline(s2s.ModelConfig(**kw))
    eager.params.copy_(model.params)
    nll2, logp2 = eager.step(xs, ls)
    torch.cuda.synchronize()
    assert torch.equal(logp2, outs[0][1]) and torch.equal(eager.grads, outs[0][2])


@pytest.mark.parametrize("graph", [False, True])
def test_model_step_overlap_bitwise(s2s, graph):
    """S2S_CTX_OVERLAP (weight-gradient GEMMs on a side stream, persistent GRU workgroups on
    exclusive CUs) must give the same bits as the single-stream step, at config-2 size."""
    cfg = s2s.ModelConfig()
    ref = s2s.ChorowskiBaseline(cfg)
    ovl = s2s.ChorowskiBaseline(cfg, graph=graph, overlap=True)
    ovl.params.copy_(ref.params)
    g = torch.Generator().manual_seed(5)
    x = torch.randn(32, 128, cfg.inputFrameSize, generator=g).cuda()
    lab = torch.randint(0, cfg.outputDepth, (32, 40), generator=g).to(torch.int32).cuda()
    nll_r, logp_r = ref.step(x, lab)
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        for _ in range(3):
            nll_o, logp_o = ovl.step(x, lab, stream=st)
    st.synchronize()
    torch.cuda.synchronize()
    assert torch.equal(logp_o, logp_r) and torch.equal(nll_o, nll_r)
    assert torch.equal(ovl.grads, ref.grads)


@pytest.mark.parametrize("graph", [False, True])
def test_bucket_events_mark_final_gradients(s2s, graph):
    """S2S_BUCKET_EVENTS: a stream that waits on bucket i's event sees that bucket's
    final gradients -- eager and under hipGraph replay (external event nodes).  A copy taken on a
    second stream right after each wait must equal the gradient after the whole step; a wait that
    did not hold would copy zeroed or half-accumulated values (the step zeroes grads first)."""
    cfg = s2s.ModelConfig()
    model = s2s.ChorowskiBaseline(cfg, graph=graph, overlap=True)
    buckets = model.grad_buckets()
    assert len(buckets) == cfg.numLayers + 1
    st, comm = torch.cuda.Stream(), torch.cuda.Stream()
    snaps = [torch.empty(n, device="cuda") for _, n in buckets]
    g = torch.Generator().manual_seed(11)
    for rep in range(3):
        x = torch.randn(32, 128, cfg.inputFrameSize, generator=g).cuda()
        lab = torch.randint(0, cfg.outputDepth, (32, 40), generator=g).to(torch.int32).cuda()
        st.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(st):
            model.step(x, lab, stream=st, bucket_events=True)
            for i, (off, n) in enumerate(buckets):
                model.wait_bucket(i, comm)
                with torch.cuda.stream(comm):
                    snaps[i].copy_(model.grads[off:off + n])
        torch.cuda.synchronize()
        for i, (off, n) in enumerate(buckets):
            assert torch.equal(snaps[i], model.grads[off:off + n]), (rep, i)
        assert model.grads.abs().sum() > 0


@pytest.mark.parametrize("B", [32, 45])
def test_fused_dy_dealing_does_not_change_the_step(s2s, B):
    """The BPTT launch's spare-slot producers compute its dy (the layer above's dX) unit by unit
    in a fixed k order, so how the units are dealt to the producers -- XCD-grouped by direction (the default,
    s2s_debug_gru_xp_group(1)) or round-robin (0) -- must not change a bit of the step; and the whole step matches the
    dX computed by a GEMM in front of the BPTT (s2s_debug_gru_fused_dy(0)) to fp32 summation noise."""
    import ctypes
    from s2s_amd import _lib
    fg, fd = _lib.lib.s2s_debug_gru_xp_group, _lib.lib.s2s_debug_gru_fused_dy
    fg.argtypes = fd.argtypes = [ctypes.c_int]
    cfg = s2s.ModelConfig()
    model = s2s.ChorowskiBaseline(cfg, graph=False)
    g = torch.Generator().manual_seed(B)
    x = torch.randn(B, 96, cfg.inputFrameSize, generator=g).cuda()
    lab = torch.randint(0, cfg.outputDepth, (B, 20), generator=g).to(torch.int32).cuda()
    outs = {}
    try:
        for arm, (grp, fused) in {"grouped": (1, 1), "round-robin": (0, 1), "gemm": (0, 0)}.items():
            fg(grp)
            fd(fused)
            nll, logp = model.step(x, lab)
            torch.cuda.synchronize()
            outs[arm] = (logp.clone(), model.grads.clone())
    finally:
        fg(1)
        fd(1)
    assert torch.equal(outs["grouped"][0], outs["round-robin"][0])
    assert torch.equal(outs["grouped"][1], outs["round-robin"][1])
    ga, gb = outs["grouped"][1], outs["gemm"][1]
    assert (ga - gb).abs().max().item() <= 1e-5 * gb.abs().max().item()


@pytest.mark.parametrize("B", [32, 45])
def test_mlp_head_summing_slabs_is_bitwise_the_reduce(s2s, B):
    """The merged MLP head of the XCD-local decoder sums the MLP GEMM's split-K slabs itself (GemmDeferReduce,
    s2s_debug_head_sums_slabs(1)) in the reduce kernel's slice order and expression, so logp, nll and every gradient
    are bitwise those of the separate splitk_reduce launch (0)."""
    import ctypes
    from s2s_amd import _lib
    fn = _lib.lib.s2s_debug_head_sums_slabs
    fn.argtypes = [ctypes.c_int]
    cfg = s2s.ModelConfig()
    model = s2s.ChorowskiBaseline(cfg, graph=False)
    g = torch.Generator().manual_seed(7 + B)
    x = torch.randn(B, 96, cfg.inputFrameSize, generator=g).cuda()
    lab = torch.randint(0, cfg.outputDepth, (B, 40), generator=g).to(torch.int32).cuda()
    outs = {}
    try:
        for arm, on in (("reduce", 0), ("head", 1)):
            fn(on)
            nll, logp = model.step(x, lab)
            torch.cuda.synchronize()
            outs[arm] = (nll.clone(), logp.clone(), model.grads.clone())
    finally:
        fn(1)
    for a, b in zip(outs["reduce"], outs["head"]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B", [32, 45])
def test_mlp_head_backward_in_the_forward_head_launch_is_bitwise_separate(s2s, B):
    """The model step writes the loss seed before the encoder, so the decoder forward's merged head launch also runs the
    MLP head's backward row by row (AttnDims::dlogp_early; no dec_mlp_head_bwd launch between the decoder launches).
    With the merged launch off (s2s_debug_merge_alpha_head(0): alpha / VBAR, the head and the head backward as separate
    launches) the same per-row sums run in the same order: logp, nll and every gradient are bitwise equal."""
    import ctypes
    from s2s_amd import _lib
    fn = _lib.lib.s2s_debug_merge_alpha_head
    fn.argtypes = [ctypes.c_int]
    cfg = s2s.ModelConfig()
    model = s2s.ChorowskiBaseline(cfg, graph=False)
    g = torch.Generator().manual_seed(17 + B)
    x = torch.randn(B, 96, cfg.inputFrameSize, generator=g).cuda()
    lab = torch.randint(0, cfg.outputDepth, (B, 40), generator=g).to(torch.int32).cuda()
    outs = {}
    try:
        for arm, on in (("separate", 0), ("fused", 1)):
            fn(on)
            nll, logp = model.step(x, lab)
            torch.cuda.synchronize()
            outs[arm] = (nll.clone(), logp.clone(), model.grads.clone())
    finally:
        fn(1)
    for a, b in zip(outs["separate"], outs["fused"]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("B", [32, 20, 9])
def test_decoder_four_row_products_match_the_sixteen_row_form(s2s, B):
    """Chains of at most 4 utterances (B <= 32) run the XCD-local decoder's skinny products on
    v_mfma_f32_4x4x1_16b_f32 (s2s_debug_dec_r4(1): handoff.h mfma4_aw_acc + mfma4_fold) instead of the 16 x 16 x 4
    form with 12 padding rows (0): the same products with the four k-quads added in another order, so logp, nll and
    every gradient agree to fp32 summation noise, and two steps of the 4 x 4 form are bitwise equal."""
    import ctypes
    from s2s_amd import _lib
    fn = _lib.lib.s2s_debug_dec_r4
    fn.argtypes = [ctypes.c_int]
    cfg = s2s.ModelConfig()
    model = s2s.ChorowskiBaseline(cfg, graph=False)
    g = torch.Generator().manual_seed(11 + B)
    x = torch.randn(B, 96, cfg.inputFrameSize, generator=g).cuda()
    lab = torch.randint(0, cfg.outputDepth, (B, 40), generator=g).to(torch.int32).cuda()
    outs = {}
    try:
        for arm, on in (("r16", 0), ("r4", 1), ("r4b", 1)):
            fn(on)
            nll, logp = model.step(x, lab)
            torch.cuda.synchronize()
            outs[arm] = (nll.clone(), logp.clone(), model.grads.clone())
    finally:
        fn(1)
    for a, b in zip(outs["r4"], outs["r4b"]):
        assert torch.equal(a, b)
    for a, b in zip(outs["r4"], outs["r16"]):
        assert torch.isfinite(a).all()
        assert (a - b).abs().max().item() <= 2e-5 * max(b.abs().max().item(), 1e-30)


@pytest.mark.parametrize("B", [32, 20])
def test_dvh_product_form_matches_the_per_term_form(s2s, B):
    """dec_xcd_dvh sums its tanh terms as r = 1 / (2^(K Vh) 2^(K ws) + 1) when every |K ws|, |K Vh| of the workgroup is
    <= 63 (one v_exp per four terms), else as r = 1 / (2^(K (ws + Vh)) + 1); s2s_debug_dvh_wide(1) forces the latter
    everywhere.  The two forms round differently, so the step's gradients agree to fp32 noise, not bitwise."""
    import ctypes
    from s2s_amd import _lib
    fn = _lib.lib.s2s_debug_dvh_wide
    fn.argtypes = [ctypes.c_int]
    cfg = s2s.ModelConfig()
    model = s2s.ChorowskiBaseline(cfg, graph=False)
    g = torch.Generator().manual_seed(23 + B)
    x = torch.randn(B, 96, cfg.inputFrameSize, generator=g).cuda()
    lab = torch.randint(0, cfg.outputDepth, (B, 40), generator=g).to(torch.int32).cuda()
    outs = {}
    try:
        for arm, on in (("product", 0), ("per_term", 1)):
            fn(on)
            nll, logp = model.step(x, lab)
            torch.cuda.synchronize()
            outs[arm] = (logp.clone(), model.grads.clone())
    finally:
        fn(0)
    assert torch.equal(outs["product"][0], outs["per_term"][0])  # the forward does not use dvh
    ga, gb = outs["product"][1], outs["per_term"][1]
    assert torch.isfinite(ga).all()
    assert (ga - gb).abs().max().item() <= 1e-5 * gb.abs().max().item()


@pytest.mark.parametrize("B,L,T,vscale", [(32, 96, 40, 1.0), (25, 400, 60, 1.0), (32, 96, 24, 5000.0)])
def test_decoder_attention_product_form_matches_the_per_term_form(s2s, B, L, T, vscale):
    """The XCD-local decoder's attention terms (dec_xcd.inc stage_vh): r = 1 / (2^(K Vh) 2^(K ws) + 1) with 2^(K Vh)
    staged once per launch (the product form, default) against r = 1 / (2^(K (ws + Vh)) + 1) per term
    (s2s_debug_dec_pf(0)), in F2's scores and B4's dws sums: the same values rounded differently, so logp and every
    gradient agree to fp32 noise (1e-5 of the tensor's max).  L = 400 runs the streamed level (Vh resident, h from
    L2).  vscale = 5000: V scaled so |K Vh| exceeds the product form's range (kPfMax) in every chunk -- the kernels
    then take the per-term form themselves and the two runs are bitwise equal."""
    import ctypes
    from s2s_amd import _lib
    from oracle import s2s_oracle as orc
    fn = _lib.lib.s2s_debug_dec_pf
    fn.argtypes = [ctypes.c_int]
    cfg = s2s.ModelConfig()
    ocfg = orc.ModelConfig()
    model = s2s.ChorowskiBaseline(cfg, graph=False)
    if vscale != 1.0:
        P = orc.unflatten(model.params.cpu().double().numpy(), ocfg)
        P["V"] = P["V"] * vscale
        model.params.copy_(torch.tensor(orc.flatten(P, ocfg), dtype=torch.float32))
    g = torch.Generator().manual_seed(7 + B + L)
    x = torch.randn(B, L, cfg.inputFrameSize, generator=g).cuda()
    lab = torch.randint(0, cfg.outputDepth, (B, T), generator=g).to(torch.int32).cuda()
    outs = {}
    try:
        for arm, on in (("product", 1), ("per_term", 0)):
            fn(on)
            model.step(x, lab)
            _, logp = model.step(x, lab)
            torch.cuda.synchronize()
            outs[arm] = (logp.clone(), model.grads.clone())
    finally:
        fn(1)
    (la, ga), (lb, gb) = outs["product"], outs["per_term"]
    assert torch.isfinite(ga).all() and torch.isfinite(la).all()
    if vscale != 1.0:
        assert torch.equal(la, lb) and torch.equal(ga, gb)
        return
    assert (la - lb).abs().max().item() <= 1e-5 * lb.abs().max().item()
    assert (ga - gb).abs().max().item() <= 1e-5 * gb.abs().max().item()


@pytest.mark.parametrize("B,ragged", [(8, False), (32, False), (32, True), (45, False), (64, False)])
def test_bptt_inlaunch_wgrad_matches_the_gemm(s2s, B, ragged):
    """The first encoder layer's weight gradients computed inside its BPTT launch by workers beside the chains
    (s2s_debug_bptt_wgrad(1), gru_persist.hip bptt_wgrad: each utterance tile's partials written through and the
    last arriving tile, by a ticket, adding them in tile order) against the weight-gradient GEMM behind the launch (0): the same
    products in another summation order, so layer 1's six dW tensors agree to fp32 summation noise (1e-5 of each
    tensor's max) and every other gradient is bitwise unchanged; two in-launch steps are bitwise equal."""
    import ctypes
    from s2s_amd import _lib
    fn = _lib.lib.s2s_debug_bptt_wgrad
    fn.argtypes = [ctypes.c_int]
    cfg = s2s.ModelConfig()
    model = s2s.ChorowskiBaseline(cfg, graph=False)
    g = torch.Generator().manual_seed(B)
    L, T = 96, 20
    x = torch.randn(B, L, cfg.inputFrameSize, generator=g).cuda()
    lab = torch.randint(0, cfg.outputDepth, (B, T), generator=g).to(torch.int32).cuda()
    kw = {}
    if ragged:
        fl = torch.randint(L // 3, L + 1, (B,), generator=g).tolist()
        fl[0] = L
        kw = dict(frame_lengths=fl, label_lengths=[T] * B)
    outs = {}
    try:
        for arm, on in (("gemm", 0), ("inlaunch", 1), ("again", 1)):
            fn(on)
            model.step(x, lab, **kw)
            torch.cuda.synchronize()
            outs[arm] = model.grads.clone()
    finally:
        fn(0)
    H, D = cfg.hiddenFrameSize, cfg.inputFrameSize
    n0 = 6 * H * (H + D)  # layer 1's six (H, H + D) gate weights lead the flat gradient vector
    assert torch.equal(outs["inlaunch"], outs["again"])
    assert torch.equal(outs["inlaunch"][n0:], outs["gemm"][n0:])
    for i in range(6):
        a = outs["inlaunch"][i * H * (H + D):(i + 1) * H * (H + D)]
        b = outs["gemm"][i * H * (H + D):(i + 1) * H * (H + D)]
        assert b.abs().max().item() > 0
        assert (a - b).abs().max().item() <= 1e-5 * b.abs().max().item(), (i, (a - b).abs().max().item())


@pytest.mark.parametrize("local,ring", [(1, 1), (1, 0), (0, 1)])
@pytest.mark.parametrize("B,H", [(32, 256), (45, 128)])
def test_persistent_gru_bitwise_equals_per_step_launches(s2s, monkeypatch, local, ring, B, H):
    """The persistent layer kernel (in-launch granule hand-offs; XCD-local L2-resident chains when
    local=1 and the census finds them on one XCD, write-through sc1 when local=0) must reproduce
    the per-step launch path bit for bit -- same arithmetic, same summation order -- over
    repeated launches.  ring: the local chains' sentinel slots as the 4-slot ring re-armed in the loop
    (1, the default) or one slot per step re-armed at launch start (0)."""
    import ctypes
    from s2s_amd import _lib
    fn = _lib.lib.s2s_debug_gru_local
    fn.argtypes = [ctypes.c_int]
    fr = _lib.lib.s2s_debug_gru_ring
    fr.argtypes = [ctypes.c_int]
    rng = np.random.default_rng(11)
    L, D = 40, 48
    x = cu(rng.standard_normal((B, L, D)))
    f, b = s2s.GRU(D, H), s2s.GRU(D, H)
    outs = {}
    fn(local)
    fr(ring)
    for mode in ("step", "persistent"):
        monkeypatch.setenv("S2S_GRU_MODE", mode)
        mod = s2s.BiRNN(f, b).cuda()
        res = []
        for rep in range(3):
            y = mod.forward(x).clone()
            mod.zeroGradParameters()
            dy = torch.ones_like(y) * 0.01 + y * 0.5
            dx = mod.backward(x, dy).clone()
            res.append((y, dx, [g.clone() for g in f.gradWeight + b.gradWeight]))
        torch.cuda.synchronize()
        outs[mode] = res
    fn(1)
    fr(1)
    for rep in range(3):
        ys, dxs, gs = outs["step"][rep]
        yp, dxp, gp = outs["persistent"][rep]
        assert torch.equal(ys, yp), f"y differs (rep {rep})"
        assert torch.equal(dxs, dxp), f"dx differs (rep {rep})"
        for i, (a, c) in enumerate(zip(gs, gp)):
            assert torch.equal(a, c), f"grad {i} differs (rep {rep})"


@pytest.mark.parametrize("B,L,T,A,Sc,S,O", [(32, 40, 12, 512, 512, 256, 62), (21, 50, 9, 128, 128, 64, 29)])
def test_persistent_decoder_bitwise_equals_per_step_launches(s2s, monkeypatch, B, L, T, A, Sc, S, O):
    """The persistent decoder kernels (granule hand-offs, 128 workgroups per 16-row tile) must
    reproduce the per-step launch path bit for bit, forward and backward, over repeated launches -- except dh:
    the per-step path forms dh = sum_t alpha_t^T dc_t + dVh V by GEMMs after its loop (a per-frame
    read-modify-write in every step cost more than the GEMM), the persistent kernel accumulates it step by step,
    so the two sum the same products in different orders (held to 1e-6 of max |dh|)."""
    rng = np.random.default_rng(3)
    att = s2s.Attention(s2s.GRU(S, S), s2s.MaxoutMLP(S + A, 8, 7, O), Sc, 10, 0, S, A, O, True, 0.2).cuda()
    h = cu(rng.standard_normal((B, L, A)) * 0.5)
    labels = cu(rng.integers(0, O, (B, T)), torch.int32)
    dlogp = cu(rng.standard_normal((B, T, O)))
    outs = {}
    for mode in ("step", "persist"):
        monkeypatch.setenv("S2S_DEC_MODE", mode)
        res = []
        for _ in range(2):
            logp = att.forward([h, labels]).clone()
            alpha = att.alpha().clone()
            att.zeroGradParameters()
            dh = att.backward([h, None], dlogp)[0].clone()
            res.append([logp, alpha, dh] + [g.clone() for g in att.parameters()[1]])
        torch.cuda.synchronize()
        outs[mode] = res
    names = ["logp", "alpha", "dh"] + ["d" + n for n in s2s.Attention.PARAM_NAMES]
    for rep in range(2):
        for name, a, b in zip(names, outs["step"][rep], outs["persist"][rep]):
            if name == "dh":
                assert (a - b).abs().max().item() <= 1e-6 * a.abs().max().item(), f"dh (rep {rep})"
                continue
            assert torch.equal(a, b), f"{name} differs (rep {rep}): max |d| = {(a - b).abs().max().item():.3e}"


@pytest.mark.parametrize("maxnorm,wd,colnorm,eta", [(1e20, 0.0, False, 0.0), (0.5, 0.0, True, 0.0),
                                                    (1e20, 1e-3, True, 0.0), (0.5, 1e-3, True, 1e-3)])
def test_optimizer_step_matches_oracle(s2s, maxnorm, wd, colnorm, eta):
    """Device optimizer step (s2s_optim_adadelta_step) vs the oracle's restatement of
    timit.lua:292-347: global-norm clip, L2, gradient noise (eta 1e-3, gamma .55: timit.lua:185-189's
    default table), optim.adadelta (rho .95, eps 1e-8, exp_logmel7_chorowski_normNLL_colnorm.lua:32-33),
    column-norm constraint -- three steps on the Chorowski flat layout, fp32 on the GPU vs float64."""
    cfg = s2s.ModelConfig()
    mats = s2s.optim.weight_matrices(cfg)
    n = sum(int(np.prod(s)) for _, s in s2s.param_shapes(cfg))
    rng = np.random.default_rng(21)
    x = (rng.standard_normal(n) * 0.08).astype(np.float32)   # many rows above norm 1
    xg = cu(x)
    gg = torch.empty_like(xg)
    opt = s2s.optim.Adadelta(params=xg, grads=gg, mats=mats, rho=0.95, eps=1e-8, maxnorm=maxnorm, weightDecay=wd,
                             colnormconstr=colnorm, gradnoise_eta=eta, gradnoise_seed=99)
    xr, st = x.astype(np.float64), {}
    for it in range(3):
        g = (rng.standard_normal(n) * 1e-3).astype(np.float32)
        gg.copy_(cu(g))
        opt.step()
        gr = g.astype(np.float64)
        gn = orc.optimizer_step(xr, gr, st, 0.95, 1e-8, maxnorm, wd, 1.0 if colnorm else 0.0, mats,
                                gradnoise_eta=eta, gradnoise_seed=99)
        torch.cuda.synchronize()
        assert abs(opt.gradnorm.item() - gn) <= 1e-5 * gn
        assert_rel(gg.cpu().numpy(), gr, f"g[{it}]", 1e-5)
        assert_rel(xg.cpu().numpy(), xr, f"x[{it}]", 1e-5)
    if colnorm:
        xs = xg.cpu().numpy()
        for off, r, c in mats:
            assert np.linalg.norm(xs[off:off + r * c].reshape(r, c), axis=1).max() <= 1.0 + 1e-5


def test_optimizer_noise_counter_resumes(s2s):
    """A resumed trainer restores gradnoise = {eta, gamma, t} (timit/timit.lua:92) and continues the schedule
    (t += 1, :312): s2s_optim_set_noise_step(t) on a fresh state draws the next step's noise with t + 1, the
    oracle's state["gradnoise_t"] = t."""
    cfg = s2s.ModelConfig()
    n = sum(int(np.prod(s)) for _, s in s2s.param_shapes(cfg))
    rng = np.random.default_rng(5)
    x = (rng.standard_normal(n) * 0.08).astype(np.float32)
    xg = cu(x)
    gg = torch.empty_like(xg)
    opt = s2s.optim.Adadelta(params=xg, grads=gg, rho=0.95, eps=1e-8, gradnoise_eta=1e-3, gradnoise_seed=7)
    opt.set_noise_step(41)
    xr, st = x.astype(np.float64), {"gradnoise_t": 41}
    for it in range(2):
        g = (rng.standard_normal(n) * 1e-3).astype(np.float32)
        gg.copy_(cu(g))
        opt.step()
        gr = g.astype(np.float64)
        orc.optimizer_step(xr, gr, st, 0.95, 1e-8, gradnoise_eta=1e-3, gradnoise_seed=7)
        torch.cuda.synchronize()
        assert_rel(gg.cpu().numpy(), gr, f"g[{it}]", 1e-5)
        assert_rel(xg.cpu().numpy(), xr, f"x[{it}]", 1e-5)
    assert st["gradnoise_t"] == 43


@pytest.mark.parametrize("K,maxlen", [(1, 8), (5, 12)])
def test_beam_search_matches_oracle(s2s, K, maxlen):
    """decoder:BeamSearch (Attention.lua:332-438) on the device for a batch of
    utterances vs the oracle's per-utterance restatement.  Every prediction must equal the oracle's,
    except at an fp32-vs-fp64 near tie of the final hypotheses: a differing prediction must score
    (teacher-forced, oracle) within 1e-4 of the oracle's best in both directions; the reported score
    must equal the oracle's rescoring of the GPU's own prediction."""
    B, L, A, Sc, S, O, M, Kw, eos = 6, 30, 64, 64, 32, 11, 4, 3, 2
    rng = np.random.default_rng(K * 100 + maxlen)
    torch.manual_seed(K)
    cfg = orc.ModelConfig(inputFrameSize=8, hiddenFrameSize=16, outputFrameSize=A // 2, scoreDepth=Sc, stateDepth=S,
                          outputDepth=O, mlpDepth=M, maxoutWindow=Kw, numLayers=1)
    att = s2s.Attention(s2s.GRU(S, S), s2s.MaxoutMLP(S + A, M, Kw, O), Sc, 10, 0, S, A, O, True, 0.0).cuda()
    P = {n: t.cpu().double().numpy() for n, t in zip(
        ("V", "Ws", "bs", "we", "Wy", "by", "Wc", "bc", "Wd", "bd", "dec.Wz", "dec.Wr", "dec.Wh", "Wm", "bm", "Wo",
         "bo"), att.parameters()[0])}
    h = rng.standard_normal((B, L, A)) * 1.5
    toks, lens, scores = att.BeamSearch(cu(h), eos, K, maxlen)
    toks, lens, scores = toks.cpu().numpy(), lens.cpu().numpy(), scores.cpu().numpy()
    agree = 0
    for b in range(B):
        seq = list(toks[b, :lens[b]])
        assert all(t == -1 for t in toks[b, lens[b]:])
        assert seq[-1] == eos or len(seq) == maxlen + 1
        ref_seq, ref_score = orc.beam_search(h[b], P, cfg, eos, K, maxlen)
        lp, _ = orc.attention_fwd(h[b][None], np.array([seq]), P, cfg)
        mine = float(lp[0, np.arange(len(seq)), seq].sum())
        assert abs(mine - scores[b]) <= 1e-4 * max(1.0, abs(mine)), (b, mine, scores[b])
        if seq == list(ref_seq):
            agree += 1
        else:  # only a genuine near tie of the two final hypotheses may flip
            assert abs(mine - ref_score) <= 1e-4 * max(1.0, abs(ref_score)), (b, seq, ref_seq, mine, ref_score)
    print(f"beam search: {agree} / {B} predictions identical to the oracle's")
    one = att.BeamSearch(cu(h[0]), eos, K, maxlen).cpu().numpy()
    assert list(one) == list(toks[0, :lens[0]])


def test_edit_distance_matches_oracle(s2s):
    """WagnerFischer (utils.lua:3-27) on the device vs the oracle, ragged lengths incl. empty."""
    rng = np.random.default_rng(5)
    n, la, lb = 40, 25, 31
    a = rng.integers(0, 5, (n, la)).astype(np.int32)
    b = rng.integers(0, 5, (n, lb)).astype(np.int32)
    alen = rng.integers(0, la + 1, n).astype(np.int32)
    blen = rng.integers(0, lb + 1, n).astype(np.int32)
    got = s2s.nn.edit_distance(cu(a, torch.int32), cu(alen, torch.int32), cu(b, torch.int32),
                               cu(blen, torch.int32)).cpu().numpy()
    want = [orc.wagner_fischer(list(a[i, :alen[i]]), list(b[i, :blen[i]])) for i in range(n)]
    assert list(got) == want
