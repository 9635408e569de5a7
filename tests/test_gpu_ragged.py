"""GPU: variable-length minibatches (VERDICT r1 "next" 6).

The reference forwards every utterance alone at its own length ("data is variable length",
timit/timit.lua:239-240) and sums the per-utterance gradients before / B (:292-295).  The batched kernels
take padded (B, L_max) / (B, T_max) batches with per-utterance frame / label lengths; every test here
compares them with the oracle run per utterance on the UNPADDED slices (oracle.training_step_ragged and
per-utterance oracle layer calls): max|gpu - ref| <= 1e-4 max|ref| per tensor, and exact zeros on the
padding (encoder outputs, alpha, dx, logp-gradient-free steps).
"""
import numpy as np
import pytest
import torch

from oracle import s2s_oracle as orc

pytestmark = pytest.mark.gpu
RTOL = 1e-4


@pytest.fixture(scope="module")
def s2s():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import s2s_amd
    return s2s_amd


def cu(a, dtype=torch.float32):
    return torch.tensor(np.ascontiguousarray(a), dtype=dtype, device="cuda")


def rel(a, r):
    a = np.asarray(a, np.float64)
    r = np.asarray(r, np.float64)
    return float(np.abs(a - r).max() / max(np.abs(r).max(), 1e-30))


def check(errs):
    bad = {k: f"{v:.2e}" for k, v in errs.items() if not v <= RTOL}
    assert not bad, bad


@pytest.mark.parametrize("mode", ["persistent", "step"])
@pytest.mark.parametrize("B,L,D,H", [(5, 23, 40, 64), (19, 16, 123, 32)])
def test_bigru_lengths_match_per_utterance(s2s, monkeypatch, mode, B, L, D, H):
    """nn.RNN(GRU) forward + reverse directions on a padded batch: each utterance's outputs, dx and the
    summed weight gradients equal the oracle run on the utterance alone; zeros on padding frames."""
    if mode == "step":
        monkeypatch.setenv("S2S_GRU_MODE", "step")
    rng = np.random.default_rng(B * 31 + L)
    lens = rng.integers(1, L + 1, B)
    lens[0] = L
    x = rng.standard_normal((B, L, D))
    cells = [s2s.GRU(D, H) for _ in range(2)]
    Ws = [[w.double().numpy() for w in c.weight] for c in cells]
    mod = s2s.BiRNN(cells[0], cells[1]).cuda()
    mod.lengths = lens
    xs = cu(x)
    y = mod.forward(xs).cpu().numpy()
    dy = rng.standard_normal(y.shape)
    mod.zeroGradParameters()
    dx = mod.backward(xs, cu(dy), 0.5).cpu().numpy()
    torch.cuda.synchronize()
    errs = {}
    for i, (W, rev) in enumerate(zip(Ws, [False, True])):
        G = {k: np.zeros_like(v) for k, v in zip(("Wz", "Wr", "Wh"), W)}
        yr = np.zeros((B, L, H))
        dxr = np.zeros_like(x)
        for b in range(B):
            xb = x[b:b + 1, :lens[b]]
            yb, sv = orc.gru_seq_fwd(xb, W[0], W[1], W[2], rev)
            yr[b, :lens[b]] = yb[0]
            dxb, _ = orc.gru_seq_bwd(xb, W[0], W[1], W[2], sv, dy[b:b + 1, :lens[b], i * H:(i + 1) * H], G, rev, 0.5)
            dxr[b, :lens[b]] = dxb[0]
        errs[f"y[{i}]"] = rel(y[:, :, i * H:(i + 1) * H], yr)
        for k, g in zip(("Wz", "Wr", "Wh"), cells[i].gradWeight):
            errs[f"d{k}[{i}]"] = rel(g.cpu().numpy(), G[k])
        if i == 0:
            dx_ref = dxr
        else:
            dx_ref = dx_ref + dxr
    errs["dx"] = rel(dx, dx_ref)
    check(errs)
    pad = np.arange(L)[None, :] >= lens[:, None]
    assert (y[pad] == 0).all() and (dx[pad] == 0).all()


@pytest.mark.parametrize("mode,peep", [("persistent", False), ("step", False), ("step", True)])
@pytest.mark.parametrize("B,L,D,H", [(32, 14, 256, 128), (7, 19, 40, 64)])
def test_bilstm_lengths_match_per_utterance(s2s, monkeypatch, mode, peep, B, L, D, H):
    """nn.RNN(LSTM) forward + reverse directions on a padded batch (the conv + BiLSTM encoder's
    recurrence, timit/timit.lua:108-125, at its shape B = 32, 256 maps, 128 units, 14 frames, and a ragged one):
    each utterance's outputs, dx and the summed weight gradients equal the oracle run on the utterance alone
    (h = c = 0 on padding frames, the reverse direction starting from zero state at the utterance's own last
    frame); zeros on padding frames.  The persistent kernels (lstm_persist.hip) and the per-step launches (with
    and without peepholes) both take the lengths."""
    monkeypatch.setenv("S2S_LSTM_MODE", mode)
    rng = np.random.default_rng(B * 37 + L)
    lens = rng.integers(1, L + 1, B)
    lens[0] = L
    lens[-1] = 1
    x = rng.standard_normal((B, L, D))
    cells = [s2s.LSTM(D, H, peepholes=peep) for _ in range(2)]
    Ps = [{k: v.double().numpy() for k, v in c.named().items()} for c in cells]
    mod = s2s.BiRNN(cells[0], cells[1]).cuda()
    mod.lengths = lens
    xs = cu(x)
    y = mod.forward(xs).cpu().numpy()
    dy = rng.standard_normal(y.shape)
    mod.zeroGradParameters()
    dx = mod.backward(xs, cu(dy), 0.5).cpu().numpy()
    torch.cuda.synchronize()
    errs = {}
    dx_ref = np.zeros_like(x)
    for i, (P, rev) in enumerate(zip(Ps, [False, True])):
        G = {k: np.zeros_like(v) for k, v in P.items()}
        yr = np.zeros((B, L, H))
        for b in range(B):
            xb = x[b:b + 1, :lens[b]]
            yb, sv = orc.lstm_seq_fwd(xb, P, rev, peep)
            yr[b, :lens[b]] = yb[0]
            dxb = orc.lstm_seq_bwd(xb, P, sv, dy[b:b + 1, :lens[b], i * H:(i + 1) * H], G, rev, peep, 0.5)
            dx_ref[b, :lens[b]] += dxb[0]
        errs[f"y[{i}]"] = rel(y[:, :, i * H:(i + 1) * H], yr)
        for k, g in cells[i].named(grads=True).items():
            errs[f"d{k}[{i}]"] = rel(g.cpu().numpy(), G[k])
    errs["dx"] = rel(dx, dx_ref)
    check(errs)
    pad = np.arange(L)[None, :] >= lens[:, None]
    assert (y[pad] == 0).all() and (dx[pad] == 0).all()


def test_bilstm_full_lengths_bitwise_equal_unmasked(s2s):
    """lengths all = L is the unmasked path bit for bit (the persistent BiLSTM at the encoder's shape)."""
    rng = np.random.default_rng(4)
    B, L, D, H = 32, 14, 256, 128
    x = cu(rng.standard_normal((B, L, D)))
    dyv = cu(rng.standard_normal((B, L, 2 * H)))
    cells = [s2s.LSTM(D, H) for _ in range(2)]
    res = []
    for lengths in (None, [L] * B):
        mod = s2s.BiRNN(cells[0], cells[1]).cuda()
        mod.lengths = lengths
        y = mod.forward(x).clone()
        mod.zeroGradParameters()
        dx = mod.backward(x, dyv, 1.0).clone()
        res.append((y, dx, [g.clone() for c in cells for g in c.named(grads=True).values()]))
    torch.cuda.synchronize()
    (y0, dx0, g0), (y1, dx1, g1) = res
    assert torch.equal(y0, y1) and torch.equal(dx0, dx1)
    assert all(torch.equal(a, b) for a, b in zip(g0, g1))


# (B, L, T, A, Sc, S, O, M, K, penalty): XCD-local decoder shapes (Chorowski sizes; S=64 ones with the
# penalty on, ragged last chain), and a per-step-kernel shape
RAGGED_ATT = [
    (10, 128, 12, 512, 512, 256, 62, 8, 7, 0.0),
    (9, 50, 9, 128, 128, 64, 29, 4, 7, 0.2),
    (5, 37, 6, 64, 64, 48, 29, 8, 7, 0.25),
]


@pytest.mark.parametrize("B,L,T,A,Sc,S,O,M,K,pen", RAGGED_ATT)
def test_attention_lengths_match_per_utterance(s2s, B, L, T, A, Sc, S, O, M, K, pen):
    """nn.Attention on padded annotations and labels with frame / label lengths: softmax over each
    utterance's own L_b frames (alpha = 0 past them), MonotonicAlignment with its own L_b and no penalty
    gradient at steps >= T_b.  Reference: the oracle decoder on each unpadded utterance."""
    rng = np.random.default_rng(L * 11 + T)
    torch.manual_seed(L * 11 + T)
    cfg = orc.ModelConfig(inputFrameSize=8, hiddenFrameSize=16, outputFrameSize=A // 2, scoreDepth=Sc, stateDepth=S,
                          outputDepth=O, mlpDepth=M, maxoutWindow=K, penalty=pen, numLayers=1)
    att = s2s.Attention(s2s.GRU(S, S), s2s.MaxoutMLP(S + A, M, K, O), Sc, 10, 0, S, A, O, True, pen).cuda()
    P = {n: t.cpu().double().numpy() for n, t in zip(
        ("V", "Ws", "bs", "we", "Wy", "by", "Wc", "bc", "Wd", "bd", "dec.Wz", "dec.Wr", "dec.Wh", "Wm", "bm", "Wo",
         "bo"), att.parameters()[0])}
    flen = rng.integers(1, L + 1, B)
    tlen = rng.integers(1, T + 1, B)
    flen[0], tlen[-1] = L, T
    h = rng.standard_normal((B, L, A)) * 0.5  # padding frames hold finite garbage: masked, never read
    labels = rng.integers(0, O, (B, T)).astype(np.int32)
    att.frame_lengths, att.label_lengths = flen, tlen
    hs = cu(h)
    logp = att.forward([hs, cu(labels, torch.int32)]).cpu().numpy()
    alpha = att.alpha().cpu().numpy()
    gind = att.mono_ind().cpu().numpy().astype(np.float64)
    dlogp = rng.standard_normal(logp.shape)
    dlogp[np.arange(T)[None, :] >= tlen[:, None]] = 0.0  # nll_seed's dlogp on padding steps
    att.zeroGradParameters()
    dh = att.backward([hs, None], cu(dlogp), 0.5)[0].cpu().numpy()
    torch.cuda.synchronize()
    G = orc.zeros_like_params(P)
    dhr = np.zeros_like(h)
    errs = {}
    lerr, aerr = 0.0, 0.0
    lmax = max(np.abs(logp).max(), 1e-30)
    for b in range(B):
        Lb, Tb = flen[b], tlen[b]
        lref, cache = orc.attention_fwd(h[b:b + 1, :Lb], labels[b:b + 1, :Tb], P, cfg)
        lerr = max(lerr, np.abs(logp[b, :Tb] - lref[0]).max() / lmax)
        aerr = max(aerr, np.abs(alpha[b, :Tb, :Lb] - cache["alpha"][0]).max())
        if pen > 0:  # the GPU's MonotonicAlignment decisions where the statistic is clear of 0
            a = cache["alpha"]
            prev = np.concatenate([np.zeros_like(a[:, :1]), a[:, :-1]], 1)
            stat = ((Lb - np.arange(Lb))[None, None, :] * (a - prev)).sum(-1)
            clear = np.abs(stat) > 1e-4
            assert np.array_equal(gind[b:b + 1, :Tb][clear], cache["mono_ind"][clear]), b
            cache["mono_ind"] = gind[b:b + 1, :Tb]
        dhr[b:b + 1, :Lb] = orc.attention_bwd(P, cfg, cache, dlogp[b:b + 1, :Tb], G, 0.5)
    errs["logp"] = lerr
    errs["alpha (abs)"] = aerr
    errs["dh"] = rel(dh, dhr)
    for name, g in zip(P.keys(), att.parameters()[1]):
        errs["d" + name] = rel(g.cpu().numpy(), G[name])
    check(errs)
    assert (alpha[np.broadcast_to(np.arange(L)[None, None, :] >= flen[:, None, None], alpha.shape)] == 0).all()
    assert (gind[np.arange(T)[None, :] >= tlen[:, None]] == 0).all()
    assert (dh[np.arange(L)[None, :] >= flen[:, None]] == 0).all()


def _ragged_batch(cfg, B, L, T, seed):
    rng = np.random.default_rng(seed)
    flen = rng.integers(max(1, L // 5), L + 1, B)
    tlen = rng.integers(max(1, T // 5), T + 1, B)
    flen[rng.integers(0, B)] = L
    tlen[rng.integers(0, B)] = T
    x, labels = orc.synthetic_batch(cfg, B, L, T, seed=seed, pad=0, eos=23)  # padding frames: finite garbage
    for b in range(B):
        labels[b, tlen[b] - 1] = 23   # EOS ends every utterance
        labels[b, tlen[b]:] = 0       # padding labels: any valid class
    return x, labels, flen, tlen


def _check_ragged_step(model, cfg_o, x, labels, flen, tlen, nll, logp):
    P = orc.unflatten(model.params.cpu().double().numpy(), cfg_o)
    nll_r, G, logps, encs = orc.training_step_ragged(x, labels, flen, tlen, P, cfg_o)
    lp = logp.cpu().numpy()
    enc = model.encoder_output().cpu().numpy()
    lmax = max(np.abs(lref).max() for lref in logps)
    emax = max(np.abs(e).max() for e in encs)
    errs = {"logp": max(np.abs(lp[b, :tlen[b]] - logps[b]).max() for b in range(len(flen))) / lmax,
            "encoder.output": max(np.abs(enc[b, :flen[b]] - encs[b]).max() for b in range(len(flen))) / emax,
            "nll": rel(nll.cpu().numpy(), nll_r)}
    Gg = orc.unflatten(model.grads.cpu().double().numpy(), cfg_o)
    errs.update({"grad " + k: rel(Gg[k], G[k]) for k in G})
    check(errs)
    assert (enc[np.arange(x.shape[1])[None, :] >= flen[:, None]] == 0).all()


def test_model_step_mixed_lengths_config2_dims(s2s):
    """The whole Chorowski step (config-2 model, XCD-local decoder) on a mixed-length batch of 12, graph
    replay + side stream as the bench runs it; then the SAME captured graph replayed with new lengths and
    inputs written into the same buffers (lengths are read on the device): still the per-utterance result."""
    cfg_o = orc.ModelConfig()
    model = s2s.ChorowskiBaseline(s2s.ModelConfig(), graph=True, overlap=True)
    B, L, T = 12, 96, 30
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    xs = torch.empty((B, L, cfg_o.inputFrameSize), device="cuda")
    ls = torch.empty((B, T), device="cuda", dtype=torch.int32)
    for rep, seed in enumerate((3, 4)):
        x, labels, flen, tlen = _ragged_batch(cfg_o, B, L, T, seed)
        xs.copy_(cu(x))
        ls.copy_(cu(labels, torch.int32))
        with torch.cuda.stream(st):
            nll, logp = model.step(xs, ls, stream=st, frame_lengths=flen, label_lengths=tlen)
        st.synchronize()
        _check_ragged_step(model, cfg_o, x, labels, flen, tlen, nll, logp)
    assert model.ctx.graph_stats()[:2] == (1, 2)


def test_model_step_mixed_lengths_small_dims(s2s):
    """Small model (per-step decoder kernels, per-step and persistent GRU both at these sizes) with B = 7
    utterances of mixed lengths, eager."""
    kw = dict(inputFrameSize=20, hiddenFrameSize=32, outputFrameSize=32, scoreDepth=48, stateDepth=32,
              outputDepth=29, mlpDepth=6, maxoutWindow=3, numLayers=2)
    cfg_o = orc.ModelConfig(**kw)
    model = s2s.ChorowskiBaseline(s2s.ModelConfig(**kw))
    x, labels, flen, tlen = _ragged_batch(cfg_o, 7, 40, 9, 8)
    nll, logp = model.step(cu(x), cu(labels, torch.int32), frame_lengths=flen, label_lengths=tlen)
    torch.cuda.synchronize()
    _check_ragged_step(model, cfg_o, x, labels, flen, tlen, nll, logp)


def test_full_lengths_equal_no_lengths_bitwise(s2s):
    """Lengths all equal to L / T are the unmasked step bit for bit (masking is exact, not approximate)."""
    cfg = s2s.ModelConfig()
    a = s2s.ChorowskiBaseline(cfg)
    b = s2s.ChorowskiBaseline(cfg)
    b.params.copy_(a.params)
    g = torch.Generator().manual_seed(2)
    x = torch.randn(8, 64, cfg.inputFrameSize, generator=g).cuda()
    lab = torch.randint(0, cfg.outputDepth, (8, 20), generator=g).to(torch.int32).cuda()
    n1, l1 = a.step(x, lab)
    n1, l1 = n1.clone(), l1.clone()
    n2, l2 = b.step(x, lab, frame_lengths=[64] * 8, label_lengths=[20] * 8)
    torch.cuda.synchronize()
    assert torch.equal(l1, l2) and torch.equal(n1, n2) and torch.equal(a.grads, b.grads)
