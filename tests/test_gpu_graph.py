"""GPU: the captured-step cache of a graph-mode context (s2s_ctx_set_graph_cache / s2s_ctx_graph_stats),
dropout under replay, and the decoder's trainer-visible surface after a model step (decoder:alpha(),
Ws(), penalty(), Vh.output -- Attention.lua:241-249, timit/timit.lua:519-521).

Every graph-mode result is compared BITWISE with an eager context on the same inputs: a replay of a
stale or wrongly-keyed graph (old pointers, old shape, a seed baked in at capture) would differ.
"""
import numpy as np
import pytest
import torch

from oracle import s2s_oracle as orc

pytestmark = pytest.mark.gpu

KW = dict(inputFrameSize=20, hiddenFrameSize=32, outputFrameSize=32, scoreDepth=48, stateDepth=32,
          outputDepth=11, mlpDepth=6, maxoutWindow=3, numLayers=2)


@pytest.fixture(scope="module")
def s2s():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import s2s_amd
    return s2s_amd


def _inputs(B, L, T, seed, F=20, O=11):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(B, L, F, generator=g).cuda()
    lab = torch.randint(0, O, (B, T), generator=g).to(torch.int32).cuda()
    return x, lab


@pytest.mark.parametrize("capacity", [8, 1])
def test_graph_cache_alternating_keys_bitwise(s2s, capacity):
    """Two shapes x two input buffers each, visited round robin for 12 steps.  capacity 8: one capture
    per key, then replays; capacity 1: every step evicts (drains, destroys) and re-captures -- the
    path that crashed in round 1 when the previous replay was destroyed while still running."""
    cfg = s2s.ModelConfig(**KW)
    gm = s2s.ChorowskiBaseline(cfg, graph=True, overlap=True)
    gm.ctx.set_graph_cache(capacity)
    ref = s2s.ChorowskiBaseline(cfg)
    ref.params.copy_(gm.params)
    keys = [_inputs(4, 20, 6, 1), _inputs(4, 20, 6, 2), _inputs(3, 16, 5, 3), _inputs(3, 16, 5, 4)]
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    outs = []
    with torch.cuda.stream(st):
        for i in range(12):
            x, lab = keys[i % 4]
            nll, logp = gm.step(x, lab, stream=st)
            outs.append((nll.clone(), logp.clone(), gm.grads.clone()))
    st.synchronize()
    for i, (nll, logp, grads) in enumerate(outs):
        x, lab = keys[i % 4]
        n2, l2 = ref.step(x, lab)
        torch.cuda.synchronize()
        assert torch.equal(l2, logp) and torch.equal(n2, nll), i
        assert torch.equal(ref.grads, grads), i
    captures, replays, cached = gm.ctx.graph_stats()
    assert replays == 12
    assert captures == (4 if capacity == 8 else 12)
    assert cached == min(capacity, 4)


def test_graph_injected_dropout_masks_one_capture(s2s):
    """Injected nn.Dropout masks change every step but the graph must not: the mask is copied into a
    model-owned buffer whose pointer is part of the key, the seed (unused) is not."""
    cfg = s2s.ModelConfig(**KW, dropout=0.5)
    gm = s2s.ChorowskiBaseline(cfg, graph=True, overlap=True)
    ref = s2s.ChorowskiBaseline(cfg)
    ref.params.copy_(gm.params)
    x, lab = _inputs(4, 20, 6, 9)
    width = cfg.stateDepth + cfg.annotationDepth
    g = torch.Generator().manual_seed(3)
    masks = [((torch.rand(4, 6, width, generator=g) >= 0.5).float() * 2.0).cuda() for _ in range(6)]
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    outs = []
    with torch.cuda.stream(st):
        for m in masks:
            _, logp = gm.step(x, lab, stream=st, dropout_mask=m)
            outs.append((logp.clone(), gm.grads.clone()))
    st.synchronize()
    for m, (logp, grads) in zip(masks, outs):
        _, l2 = ref.step(x, lab, dropout_mask=m)
        torch.cuda.synchronize()
        assert torch.equal(l2, logp) and torch.equal(ref.grads, grads)
    assert gm.ctx.graph_stats()[0] == 1


def test_graph_dropout_seed_replay_equals_eager(s2s):
    """In-kernel masks under replay: one capture for 15 steps with 15 seeds; the replayed step with
    seed 7 equals the eager step with seed 7 bitwise (so the seed is read at replay, not baked in at
    capture) and its mask drops a fraction ~p of the units with the 1/(1-p) scaling."""
    p = 0.5
    cfg = s2s.ModelConfig(**KW, dropout=p)
    gm = s2s.ChorowskiBaseline(cfg, graph=True, overlap=True)
    ref = s2s.ChorowskiBaseline(cfg)
    ref.params.copy_(gm.params)
    x, lab = _inputs(16, 20, 8, 5)
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        for seed in range(100, 114):
            gm.step(x, lab, stream=st, dropout_seed=seed)
        _, logp = gm.step(x, lab, stream=st, dropout_seed=7)
    st.synchronize()
    mask = gm.dropout_mask_used().clone()
    _, l2 = ref.step(x, lab, dropout_seed=7)
    torch.cuda.synchronize()
    assert torch.equal(l2, logp) and torch.equal(ref.grads, gm.grads)
    assert torch.equal(ref.dropout_mask_used(), mask)
    vals = set(torch.unique(mask).tolist())
    assert vals <= {0.0, 1.0 / (1.0 - p)}
    assert abs(float((mask == 0).float().mean()) - p) < 0.03
    assert gm.ctx.graph_stats()[:2] == (1, 15)


def test_default_dropout_seeds_differ_by_step_and_rank(s2s, monkeypatch):
    """Default seeds mix the init seed, the data-parallel rank and the step counter: two ranks draw
    different masks at the same step; the checkpoint restores the counter (no mask replay on resume)."""
    cfg = s2s.ModelConfig(**KW, dropout=0.5)
    monkeypatch.setenv("RANK", "0")
    a = s2s.ChorowskiBaseline(cfg)
    monkeypatch.setenv("RANK", "1")
    b = s2s.ChorowskiBaseline(cfg)
    x, lab = _inputs(2, 10, 4, 6)
    a.step(x, lab)
    ma = a.dropout_mask_used().clone()
    b.step(x, lab)
    mb = b.dropout_mask_used().clone()
    assert not torch.equal(ma, mb)
    a.step(x, lab)
    assert not torch.equal(a.dropout_mask_used(), ma)


def test_decoder_accessors_after_model_step(s2s):
    """decoder:alpha() / penalty() / Ws() / Vh.output of the model step's decoder against the oracle's
    forward on the same encoder output."""
    cfg_o = orc.ModelConfig(**KW)
    model = s2s.ChorowskiBaseline(s2s.ModelConfig(**KW))
    P = orc.unflatten(model.params.cpu().double().numpy(), cfg_o)
    x, labels = orc.synthetic_batch(cfg_o, 3, 18, 5, seed=2, pad=3, eos=7)
    model.step(torch.tensor(x, dtype=torch.float32, device="cuda"),
               torch.tensor(labels, dtype=torch.int32, device="cuda"))
    torch.cuda.synchronize()
    enc, _ = orc.encoder_fwd(x, P, cfg_o.numLayers)
    _, cache = orc.attention_fwd(enc, labels, P, cfg_o)

    def close(a, r, name):
        a = a.detach().cpu().double().numpy()
        err = np.abs(a - r).max() / max(np.abs(r).max(), 1e-30)
        assert err < 1e-4, (name, err)

    close(model.decoder_alpha(), cache["alpha"], "alpha")
    assert torch.equal(model.decoder_penalty(), model.decoder_alpha())
    ws = model.decoder_Ws()
    assert ws.shape == (3, 5, 18, cfg_o.scoreDepth)
    close(ws[:, :, 0], cache["ws"], "Ws")
    assert torch.equal(ws[:, :, 7], ws[:, :, 0])
    close(model.decoder_Vh(), cache["Vh"], "Vh.output")


def test_graph_step_on_explicit_stream_outside_its_context(s2s):
    """step(..., stream=st) called while the CURRENT stream is another one (the advisor's round-2 case): the
    injected dropout mask and the lengths are written into the model-owned buffers on `st`, after `st` has
    waited for the current stream that produced them, so each replay reads its own step's mask -- equal
    bitwise to an eager model stepping on the current stream."""
    cfg = s2s.ModelConfig(**KW, dropout=0.5)
    gm = s2s.ChorowskiBaseline(cfg, graph=True, overlap=True)
    ref = s2s.ChorowskiBaseline(cfg)
    ref.params.copy_(gm.params)
    S, A = cfg.stateDepth, cfg.annotationDepth
    st = torch.cuda.Stream()
    x, lab = _inputs(3, 16, 5, 11)
    g = torch.Generator(device="cuda").manual_seed(5)
    for i in range(5):
        mask = (torch.rand(3, 5, S + A, device="cuda", generator=g) > 0.5).float() * 2.0  # current stream
        nll, logp = gm.step(x, lab, stream=st, dropout_mask=mask, frame_lengths=[16, 12 + i, 9],
                            label_lengths=[5, 4, 3])
        torch.cuda.current_stream().wait_stream(st)
        got = (nll.clone(), logp.clone(), gm.grads.clone())
        n2, l2 = ref.step(x, lab, dropout_mask=mask, frame_lengths=[16, 12 + i, 9], label_lengths=[5, 4, 3])
        torch.cuda.synchronize()
        assert torch.equal(got[1], l2) and torch.equal(got[0], n2), i
        assert torch.equal(got[2], ref.grads), i
    assert gm.ctx.graph_stats()[0] == 1  # one capture: mask and lengths live in stable model-owned buffers
