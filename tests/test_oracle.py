"""Pins the CPU oracle (oracle/s2s_oracle.py) before anything is checked against it.

* the reference notebooks' known answers;
* an independent PyTorch autograd formulation (tests/torch_ref.py) in float64;
* central finite differences in float64;
* batched == per-utterance loop (the reference's own batch semantics, timit/timit.lua:240-295);
* the committed golden fixtures under tests/golden/.
"""
import os

import numpy as np
import pytest
import torch

from oracle import s2s_oracle as orc
import torch_ref

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def tiny_cfg(**kw):
    base = dict(inputFrameSize=5, hiddenFrameSize=4, outputFrameSize=3, scoreDepth=6, stateDepth=4,
                outputDepth=7, mlpDepth=3, maxoutWindow=2, penalty=0.0, numLayers=2)
    base.update(kw)
    return orc.ModelConfig(**base)


# --------------------------------------------------------------------------- known answers

def test_temporal_conv_iota_known_answer():
    """Attention.ipynb cells 4-6: TemporalConvolution(5,4,1), weights 1..20 row-major,
    bias 0, input ones(10,5) -> every row = [15, 40, 65, 90]; batched (8,10,5) keeps shape."""
    W = np.arange(1, 21, dtype=np.float64).reshape(4, 5)
    y = orc.temporal_conv(W, np.zeros(4), np.ones((10, 5)), 1)
    assert y.shape == (10, 4)
    np.testing.assert_array_equal(y, np.tile([15, 40, 65, 90], (10, 1)))
    assert orc.temporal_conv(W, None, np.ones((8, 10, 5)), 1).shape == (8, 10, 4)


@pytest.mark.parametrize("kW,L", [(3, 10), (3, 11), (4, 10), (4, 11)])
def test_hybrid_padding_shapes_known_answer(kW, L):
    """Attention.ipynb cells 8-15 / Attention.lua:76-90: odd kW pads (kW-1)/2 both sides,
    even kW pads kW/2 left and kW/2-1 right; the conv then returns L frames."""
    if kW % 2 == 1:
        pl = pr = (kW - 1) // 2
    else:
        pl, pr = kW // 2, kW // 2 - 1
    a = np.ones((L, 1))
    padded = np.concatenate([np.zeros((pl, 1)), a, np.zeros((pr, 1))])
    y = orc.temporal_conv(np.ones((5, kW)), np.zeros(5), padded, kW)
    assert y.shape == (L, 5)


def test_nll_equals_classnll_identity():
    """AttentionSmallModel.ipynb:304-351: -sum(labelmask * logprobs) == sum ClassNLLCriterion
    (and /B in batch mode).  Pins the loss definition at timit/timit.lua:262-272."""
    rng = np.random.default_rng(0)
    logp = orc.log_softmax(rng.standard_normal((4, 9, 7)), -1)
    labels = rng.integers(0, 7, (4, 9))
    onehot = np.zeros_like(logp)
    np.put_along_axis(onehot, labels[..., None], 1.0, 2)
    lm = -(onehot * logp).sum()
    classnll = -np.take_along_axis(logp, labels[..., None], 2).sum()
    assert abs(lm - classnll) < 1e-12


def test_maxout_first_max_wins():
    """nn.TemporalMaxPooling (3p) strict '>' scan: ties go to the first element."""
    cfg = tiny_cfg()
    u = np.array([[1.0, 1.0, 0.5, 0.5, -2.0, 3.0]])
    am = np.argmax(u.reshape(1, 3, 2), axis=2)
    np.testing.assert_array_equal(am, [[0, 0, 1]])


# --------------------------------------------------------------------------- autograd + FD

def _torch_params(P):
    return {k: torch.tensor(v, requires_grad=True) for k, v in P.items()}


def _torch_loss(x, labels, TP, cfg, B):
    logp, pens = torch_ref.model_forward(torch.tensor(x), labels, TP, cfg)
    onehot = torch.nn.functional.one_hot(torch.as_tensor(labels).long(), cfg.outputDepth).double()
    loss = -(onehot * logp).sum()
    for diff, a, aprev in pens:
        ind = (cfg.penalty * torch.clamp(diff.detach(), min=0) > 0).double()
        loss = loss + (cfg.penalty * ind * diff).sum()
    return loss / (B if B > 1 else 1), logp


@pytest.mark.parametrize("penalty,kW,nF", [(0.0, 0, 0), (0.3, 0, 0), (0.0, 3, 2), (0.3, 4, 3)])
def test_oracle_matches_torch_autograd(penalty, kW, nF):
    """kW/nF > 0: hybrid location-aware attention (Attention.lua:75-98), odd and even filters;
    torch's conv1d + autograd is an independent statement of the conv, its padding and the
    d alpha_{t-1} path through the carried hidden state."""
    cfg = tiny_cfg(penalty=penalty, hybridAttendFilterSize=kW, hybridAttendFeatureMaps=nF)
    B, L, T = 3, 6, 5
    P = orc.init_params(cfg, seed=7)
    x, labels = orc.synthetic_batch(cfg, B, L, T, seed=3, pad=1, eos=2)
    nll, G, logp, _ = orc.training_step(x, labels, P, cfg, normalizeNLL=False)
    TP = _torch_params(P)
    loss, tlogp = _torch_loss(x, labels, TP, cfg, B)
    loss.backward()
    np.testing.assert_allclose(logp, tlogp.detach().numpy(), rtol=1e-12, atol=1e-12)
    for k in P:
        np.testing.assert_allclose(G[k], TP[k].grad.numpy(), rtol=1e-9, atol=1e-11, err_msg=k)


@pytest.mark.parametrize("kW,nF", [(0, 0), (5, 2)])
def test_oracle_finite_differences(kW, nF):
    cfg = tiny_cfg(hybridAttendFilterSize=kW, hybridAttendFeatureMaps=nF)
    B, L, T = 2, 5, 4
    P = orc.init_params(cfg, seed=11)
    x, labels = orc.synthetic_batch(cfg, B, L, T, seed=5, pad=1, eos=1)
    _, G, _, _ = orc.training_step(x, labels, P, cfg, normalizeNLL=False)
    rng = np.random.default_rng(2)

    def loss_of(P2):
        logp, _ = orc.attention_fwd(orc.encoder_fwd(x, P2, cfg.numLayers)[0], labels, P2, cfg)
        oh = np.zeros_like(logp)
        np.put_along_axis(oh, labels[..., None], 1.0, 2)
        return -(oh * logp).sum() / B

    eps = 1e-6
    for k in P:
        flat = P[k].reshape(-1)
        for idx in rng.choice(flat.size, size=min(4, flat.size), replace=False):
            old = flat[idx]
            flat[idx] = old + eps
            lp = loss_of(P)
            flat[idx] = old - eps
            lm = loss_of(P)
            flat[idx] = old
            fd = (lp - lm) / (2 * eps)
            an = G[k].reshape(-1)[idx]
            assert abs(fd - an) <= 1e-6 + 1e-5 * abs(fd), (k, idx, fd, an)


def test_batched_equals_per_utterance_loop():
    """timit/timit.lua:240-295 runs utterances one at a time and divides by B."""
    cfg = tiny_cfg()
    B, L, T = 3, 6, 4
    P = orc.init_params(cfg, seed=1)
    x, labels = orc.synthetic_batch(cfg, B, L, T, seed=9, pad=1, eos=0)
    nll, G, logp, _ = orc.training_step(x, labels, P, cfg)
    acc = orc.zeros_like_params(P)
    nlls = []
    for b in range(B):
        n1, g1, lp1, _ = orc.training_step(x[b:b + 1], labels[b:b + 1], P, cfg)
        nlls.append(n1)
        np.testing.assert_allclose(lp1[0], logp[b], rtol=1e-12, atol=1e-13)
        for k in acc:
            acc[k] += g1[k]
    assert abs(np.mean(nlls) - nll) < 1e-12
    for k in acc:
        np.testing.assert_allclose(acc[k] / B, G[k], rtol=1e-10, atol=1e-13, err_msg=k)


def test_lstm_matches_torch_autograd():
    rng = np.random.default_rng(4)
    B, L, D, H = 2, 5, 3, 4
    for peep in (False, True):
        P = {}
        for g in "ifgo":
            P[f"W{g}x"] = rng.uniform(-.5, .5, (H, D)); P[f"b{g}x"] = rng.uniform(-.5, .5, H)
            P[f"W{g}h"] = rng.uniform(-.5, .5, (H, H)); P[f"b{g}h"] = rng.uniform(-.5, .5, H)
            if peep and g != "g":
                P[f"W{g}c"] = rng.uniform(-.5, .5, (H, H)); P[f"b{g}c"] = rng.uniform(-.5, .5, H)
        x = rng.standard_normal((B, L, D))
        dy = rng.standard_normal((B, L, H))
        for rev in (False, True):
            y, sv = orc.lstm_seq_fwd(x, P, rev, peep)
            G = {k: np.zeros_like(v) for k, v in P.items()}
            dx = orc.lstm_seq_bwd(x, P, sv, dy, G, rev, peep)
            TP = {k: torch.tensor(v, requires_grad=True) for k, v in P.items()}
            tx = torch.tensor(x, requires_grad=True)
            ty = torch_ref.lstm_rnn(tx, TP, rev, peep)
            (ty * torch.tensor(dy)).sum().backward()
            np.testing.assert_allclose(y, ty.detach().numpy(), rtol=1e-12, atol=1e-13)
            np.testing.assert_allclose(dx, tx.grad.numpy(), rtol=1e-10, atol=1e-12)
            for k in P:
                np.testing.assert_allclose(G[k], TP[k].grad.numpy(), rtol=1e-10, atol=1e-12, err_msg=k)


# --------------------------------------------------------------------------- golden fixtures

def test_oracle_reproduces_golden_fixtures():
    path = os.path.join(GOLDEN, "tiny_step.npz")
    if not os.path.exists(path):
        pytest.skip("golden fixture not generated")
    g = np.load(path)
    cfg = orc.ModelConfig(**{k: (float(g["cfg_" + k]) if k == "penalty" else int(g["cfg_" + k]))
                             for k in ("inputFrameSize", "hiddenFrameSize", "outputFrameSize", "scoreDepth",
                                       "stateDepth", "outputDepth", "mlpDepth", "maxoutWindow", "penalty",
                                       "numLayers")})
    P = orc.unflatten(g["params"], cfg)
    nll, G, logp, enc = orc.training_step(g["x"], g["labels"], P, cfg)
    np.testing.assert_allclose(logp, g["logp"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(enc, g["enc"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(orc.flatten(G, cfg), g["grads"], rtol=1e-10, atol=1e-12)
    assert abs(nll - float(g["nll"])) < 1e-12


def test_oracle_reproduces_chorowski_fixture():
    g = np.load(os.path.join(GOLDEN, "chorowski_L32_T10.npz"))
    cfg = orc.ModelConfig()
    P = orc.init_params(cfg, seed=int(g["seed"]))
    x, labels = orc.synthetic_batch(cfg, 2, 32, 10, seed=int(g["seed"]), pad=10, eos=23)
    np.testing.assert_array_equal(labels, g["labels"])
    nll, G, logp, enc = orc.training_step(x, labels, P, cfg)
    np.testing.assert_allclose(logp, g["logp"], rtol=1e-12, atol=1e-12)
    np.testing.assert_allclose(enc, g["enc"], rtol=1e-12, atol=1e-12)
    flatG = orc.flatten(G, cfg)
    np.testing.assert_allclose(flatG[g["grad_idx"]], g["grad_vals"], rtol=1e-9, atol=1e-14)
    assert flatG.size == 4356735 - 512 - 1  # SURVEY §8d count includes the zero TCZB biases (V: 512, we: 1)


def test_column_norm_constraint_semantics():
    """TrainUtils.lua:52-104: rows (W:norm(2,2)) with norm + 1e-8 >= maxval are scaled to maxval
    (up to the 1e-8), the others untouched; applied after the update (timit.lua:344-346)."""
    rng = np.random.default_rng(4)
    W = rng.standard_normal((6, 9))
    W[:3] *= 0.05                       # rows well inside the unit ball
    out = orc.column_norm_constraint(W, 1.0)
    np.testing.assert_array_equal(out[:3], W[:3])
    np.testing.assert_allclose(np.linalg.norm(out[3:], axis=1), 1.0, rtol=1e-7)
    out2 = orc.column_norm_constraint(W, 0.5)
    assert np.all(np.linalg.norm(out2, axis=1) <= 0.5 + 1e-7)


def test_optimizer_step_matches_adadelta_definition():
    """optim.adadelta (3p) with the trainer's clip and L2 (timit.lua:292-308), two steps by hand."""
    rng = np.random.default_rng(8)
    x0 = rng.standard_normal(50)
    g0 = rng.standard_normal(50)
    x, g, st = x0.copy(), g0.copy(), {}
    gn = orc.optimizer_step(x, g, st, rho=0.9, eps=1e-6, maxnorm=2.0, weightDecay=0.01)
    assert abs(gn - np.linalg.norm(g0)) < 1e-12
    gc = g0 * (2.0 / np.linalg.norm(g0)) + 0.01 * x0
    v = 0.1 * gc * gc
    d = np.sqrt(1e-6) / np.sqrt(v + 1e-6) * gc
    np.testing.assert_allclose(x, x0 - d, rtol=1e-13)
    np.testing.assert_allclose(st["accDelta"], 0.1 * d * d, rtol=1e-13)


def test_wagner_fischer_known_answers():
    """utils.lua:3-27 on textbook pairs (kitten/sitting = 3, flaw/lawn = 2) and the empty cases."""
    enc = lambda w: [ord(c) for c in w]
    assert orc.wagner_fischer(enc("kitten"), enc("sitting")) == 3
    assert orc.wagner_fischer(enc("flaw"), enc("lawn")) == 2
    assert orc.wagner_fischer([], [1, 2, 3]) == 3
    assert orc.wagner_fischer([4, 5], []) == 2
    assert orc.wagner_fischer([1, 2, 3], [1, 2, 3]) == 0


@pytest.mark.parametrize("variant", ["gru", "hybrid", "lstm", "hybrid_lstm"])
def test_beam_search_step_matches_teacher_forced_forward(variant):
    """decoder_step restates the training forward's step: the beam search's score of its best
    hypothesis equals the teacher-forced log-likelihood of that sequence (attention_fwd with the
    hypothesis as labels), and K = 1 is greedy decoding -- for the content / hybrid attention and the
    GRU / LSTM decoder_recurrent (the carried hidden {alpha, s, mem})."""
    kw = dict(hybridAttendFeatureMaps=3, hybridAttendFilterSize=5) if "hybrid" in variant else {}
    cfg = tiny_cfg(decoderLSTM="lstm" in variant, **kw)
    P = orc.init_params(cfg, seed=13)
    if cfg.decoderLSTM:  # LSTM(S, S) gates (LSTM.lua:25-29); init_params draws the GRU's
        prng, S = np.random.default_rng(5), cfg.stateDepth
        for q in "ifgo":
            P.update({f"dec.W{q}x": prng.standard_normal((S, S)) * 0.4, f"dec.b{q}x": prng.standard_normal(S) * 0.1,
                      f"dec.W{q}h": prng.standard_normal((S, S)) * 0.4, f"dec.b{q}h": prng.standard_normal(S) * 0.1})
    rng = np.random.default_rng(3)
    h = rng.standard_normal((9, cfg.annotationDepth))
    for K in (1, 3):
        seq, score = orc.beam_search(h, P, cfg, eos=2, K=K, maxseqlength=6)
        logp, _ = orc.attention_fwd(h[None], np.array([seq]), P, cfg)
        assert abs(logp[0, np.arange(len(seq)), seq].sum() - score) < 1e-10
        assert seq[-1] == 2 or len(seq) == 7
    greedy, y, st = [], -1, orc.decoder_zero_state(9, cfg.stateDepth)
    Vh = h @ P["V"].T
    for _ in range(7):
        lp, st = orc.decoder_step(h, Vh, st, y, P, cfg)
        y = int(np.argmax(lp))
        greedy.append(y)
        if y == 2:
            break
    assert orc.beam_search(h, P, cfg, eos=2, K=1, maxseqlength=6)[0] == greedy


def test_beam_search_external_mlp_equals_fused():
    """An external decoder_mlp (the Maxout -> Linear -> LogSoftMax stack as a callable) searches exactly
    like the fused MaxoutMLP."""
    from oracle import frontend_oracle as fo
    cfg = tiny_cfg()
    P = orc.init_params(cfg, seed=17)
    h = np.random.default_rng(4).standard_normal((9, cfg.annotationDepth))
    layers = [("maxout", P["Wm"], P["bm"], cfg.maxoutWindow), ("linear", P["Wo"], P["bo"]), ("logsoftmax",)]
    mlp = lambda v: fo.mlp_fwd(v[None], layers)[0][0]  # noqa: E731
    for K in (1, 4):
        a = orc.beam_search(h, P, cfg, eos=2, K=K, maxseqlength=6)
        b = orc.beam_search(h, P, cfg, eos=2, K=K, maxseqlength=6, mlp=mlp)
        assert a[0] == b[0] and abs(a[1] - b[1]) < 1e-12


def test_gradient_noise_draws_and_schedule():
    """timit.lua:310-315: t counts optimizer steps from 1, sigma = (eta / (1 + t)^gamma)^0.5, and the
    counter-based draws are standard normal, deterministic in (seed, t) and fresh per step."""
    z = orc.gradient_noise(200000, 7, 1)
    assert abs(z.mean()) < 0.01 and abs(z.std() - 1) < 0.01
    assert np.array_equal(z, orc.gradient_noise(200000, 7, 1))
    assert np.corrcoef(z, orc.gradient_noise(200000, 7, 2))[0, 1] < 0.01
    assert np.corrcoef(z, orc.gradient_noise(200000, 8, 1))[0, 1] < 0.01
    n = 1000
    x, st = np.zeros(n), {}
    for t in (1, 2):
        g = np.zeros(n)
        orc.optimizer_step(x, g, st, gradnoise_eta=1e-3, gradnoise_gamma=0.55, gradnoise_seed=3)
        np.testing.assert_allclose(g, orc.gradient_noise(n, 3, t) * (1e-3 / (1 + t) ** 0.55) ** 0.5, rtol=1e-12)
    assert st["gradnoise_t"] == 2


def test_forced_maxout_decisions():
    """training_step(maxout_idx=...) runs the step under given Maxout winners: its own argmax reproduces the
    free run exactly, and a different winner changes m (and logp) accordingly."""
    cfg = orc.ModelConfig(inputFrameSize=6, hiddenFrameSize=4, outputFrameSize=4, scoreDepth=5, stateDepth=4,
                          outputDepth=5, mlpDepth=3, maxoutWindow=3, numLayers=1)
    P = orc.init_params(cfg, seed=3)
    x, labels = orc.synthetic_batch(cfg, 2, 7, 4, seed=1, pad=1, eos=2)
    enc, _ = orc.encoder_fwd(x, P, cfg.numLayers)
    lp, cache = orc.attention_fwd(enc, labels, P, cfg)
    am = cache["argmax"]
    nll, G, lp2, _ = orc.training_step(x, labels, P, cfg, maxout_idx=am)
    nll0, G0, lp0, _ = orc.training_step(x, labels, P, cfg)
    assert np.array_equal(lp2, lp0) and nll == nll0
    assert all(np.array_equal(G[k], G0[k]) for k in G)
    other = (am + 1) % cfg.maxoutWindow
    _, c2 = orc.attention_fwd(enc, labels, P, cfg, maxout_idx=other)
    u = c2["u"].reshape(2, 4, cfg.mlpDepth, cfg.maxoutWindow)
    np.testing.assert_array_equal(c2["m"], np.take_along_axis(u, other[..., None], 3)[..., 0])
