"""GPU: a persistent launch that fails is a reported error, not silent garbage (SURVEY.md §8b "int status,
never abort"; the reference raises through error()/assert, RNN.lua:8-9, Attention.lua:316).

The persistent kernels hand data between workgroups with bounded waits.  A wait that times out, or a launch
that finds its sync region already aborted, sets the context's host-visible status words; every later compute
call of that context then fails until s2s_ctx_status(..., clear=1) has reported it.  Two deterministic
triggers: s2s_debug_handoff_timeout (one wave waits for a value nobody writes, with a short spin limit: the
timeout path itself) and s2s_debug_inject_abort (the next sync_prep starts its region aborted: the persistent
GRU / decoder launch behind it gives up its waits -- S2S_STATUS_ABORTED_REGION, or HANDOFF_TIMEOUT when a wave
gave up first).  The failure words are harvested into the status at the end of each call.  After the status is
cleared the same calls give the oracle's results again.
"""
import ctypes

import numpy as np
import pytest
import torch

from oracle import s2s_oracle as orc

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def s2s():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import s2s_amd
    from s2s_amd import _lib
    _lib.lib.s2s_debug_inject_abort.argtypes = [ctypes.c_int]
    _lib.lib.s2s_debug_inject_abort.restype = None
    _lib.lib.s2s_debug_handoff_timeout.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
    _lib.lib.s2s_debug_handoff_timeout.restype = ctypes.c_int
    yield s2s_amd
    _lib.lib.s2s_debug_inject_abort(0)


def _rel(g, r):
    return float(np.abs(np.asarray(g, np.float64) - r).max() / max(np.abs(r).max(), 1e-30))


def test_handoff_timeout_sets_status_and_blocks_calls(s2s):
    from s2s_amd import _lib
    ctx = s2s.Context(0)
    region = torch.zeros(1024, dtype=torch.uint8, device="cuda")
    assert ctx.status(clear=False) == 0
    _lib.check(_lib.lib.s2s_debug_handoff_timeout(ctx.handle, s2s.nn.stream_ptr(), ctypes.c_void_p(region.data_ptr())))
    assert ctx.status(clear=False) == _lib.S2S_STATUS_HANDOFF_TIMEOUT
    assert int(region[:4].view(torch.int32).item()) == 0  # the harvest reported the abort word and cleared it
    # every later compute call of this context fails loudly (and names the way out) ...
    with pytest.raises(_lib.S2SError, match="timed out"):
        _lib.check(_lib.lib.s2s_debug_handoff_timeout(ctx.handle, s2s.nn.stream_ptr(),
                                                     ctypes.c_void_p(region.data_ptr())))
    with pytest.raises(_lib.S2SError, match="persistent launch failure"):
        ctx.check_status()  # reports (and clears) it
    assert ctx.status() == 0
    # ... other contexts are unaffected
    assert s2s.nn.get_context(0).status(clear=False) == 0


def test_injected_abort_gru_layer_reports_then_recovers(s2s):
    """BiGRU layer on the persistent kernels (H = 64, B = 5): the injected abort hits the sync_prep in front of
    the forward launch; the status says so, the next call raises, and after clearing the status the same layer
    matches the oracle."""
    from s2s_amd import _lib
    ctx = s2s.nn.get_context(0)
    assert ctx.status() == 0
    rng = np.random.default_rng(7)
    B, L, D, H = 5, 16, 123, 64
    x = rng.standard_normal((B, L, D))
    cells = [s2s.GRU(D, H) for _ in range(2)]
    mod = s2s.BiRNN(cells[0], cells[1]).cuda()
    xs = torch.tensor(x, dtype=torch.float32, device="cuda")
    try:
        _lib.lib.s2s_debug_inject_abort(1)
        mod.forward(xs)
        torch.cuda.synchronize()
        _lib.lib.s2s_debug_inject_abort(0)
        assert ctx.status(clear=False) != 0
        with pytest.raises(_lib.S2SError, match="persistent launch of an earlier call failed"):
            mod.forward(xs)
    finally:
        _lib.lib.s2s_debug_inject_abort(0)
        st = ctx.status(clear=True)
    assert st & (_lib.S2S_STATUS_ABORTED_REGION | _lib.S2S_STATUS_HANDOFF_TIMEOUT)
    y = mod.forward(xs).cpu().numpy()
    assert ctx.status() == 0
    for i, rev in enumerate((False, True)):
        W = [w.detach().cpu().double().numpy() for w in cells[i].weight]
        yr, _ = orc.gru_seq_fwd(x, W[0], W[1], W[2], rev)
        assert _rel(y[:, :, i * H:(i + 1) * H], yr) < 1e-4


def test_injected_abort_model_step_reports_then_recovers(s2s):
    """Config-2-shaped model step (XCD-local decoder, persistent GRU launches) on its own overlap context:
    the first sync_prep of the step (the decoder's forward region, prepared in its prologue) starts aborted.
    The step completes (nothing waits forever), the status is set, the next step raises, and after clearing
    the status a step equals a fresh model's step bitwise."""
    from s2s_amd import _lib
    cfg = s2s.ModelConfig()
    m = s2s.ChorowskiBaseline(cfg, overlap=True)
    ref = s2s.ChorowskiBaseline(cfg, overlap=True)
    ref.params.copy_(m.params)
    g = torch.Generator().manual_seed(3)
    x = torch.randn(4, 24, cfg.inputFrameSize, generator=g).cuda()
    lab = torch.randint(0, cfg.outputDepth, (4, 6), generator=g).to(torch.int32).cuda()
    try:
        _lib.lib.s2s_debug_inject_abort(1)
        m.step(x, lab)
        torch.cuda.synchronize()
        _lib.lib.s2s_debug_inject_abort(0)
        assert m.ctx.status(clear=False) != 0
        with pytest.raises(_lib.S2SError):
            m.step(x, lab)
    finally:
        _lib.lib.s2s_debug_inject_abort(0)
        m.ctx.status(clear=True)
    nll, logp = m.step(x, lab)
    n2, l2 = ref.step(x, lab)
    torch.cuda.synchronize()
    assert m.ctx.status() == 0 and ref.ctx.status() == 0
    assert torch.equal(logp, l2) and torch.equal(nll, n2)
    assert torch.equal(m.grads, ref.grads)


def test_optimizer_queued_behind_failed_step_skips_update(s2s):
    """the host gate only sees a failure after the harvest has run, so an optimizer update already
    queued in program order behind the failed step would apply its invalid gradients.  The update reads the
    context's status words on the device and skips itself: parameters, optimizer state and the noise counter
    stay untouched.  A sleep kernel in front of the step keeps the host from seeing the status before the
    update is queued (the device-side path is the one exercised)."""
    from s2s_amd import _lib
    from s2s_amd.optim import Adadelta
    cfg = s2s.ModelConfig()
    m = s2s.ChorowskiBaseline(cfg, overlap=True)
    opt = Adadelta(m, gradnoise_eta=1e-3)
    assert opt.ctx is m.ctx
    g = torch.Generator().manual_seed(5)
    x = torch.randn(4, 24, cfg.inputFrameSize, generator=g).cuda()
    lab = torch.randint(0, cfg.outputDepth, (4, 6), generator=g).to(torch.int32).cuda()
    m.step(x, lab)  # a good step + update first: the state is non-trivial
    opt.step()
    torch.cuda.synchronize()
    p0, s0 = m.params.clone(), opt.state.clone()
    try:
        _lib.lib.s2s_debug_inject_abort(1)
        torch.cuda._sleep(50_000_000)  # ~25 ms of device time ahead of the failing step
        m.step(x, lab)
        opt.step()  # queued before the harvest has run
        _lib.lib.s2s_debug_inject_abort(0)
        torch.cuda.synchronize()
        assert m.ctx.status(clear=False) != 0
    finally:
        _lib.lib.s2s_debug_inject_abort(0)
        m.ctx.status(clear=True)
    assert torch.equal(m.params, p0)
    # state = v | u (nn floats each) | 512 norm partials | scal: v, u and scal[0..3] (norm, clip, sigma, noise t)
    nn = (opt.n + 63) // 64 * 64
    f, f0 = opt.state.view(torch.float32), s0.view(torch.float32)
    assert torch.equal(f[:2 * nn], f0[:2 * nn])
    assert torch.equal(f[2 * nn + 512:2 * nn + 516], f0[2 * nn + 512:2 * nn + 516])
    # after clearing, a good step updates again
    m.step(x, lab)
    opt.step()
    torch.cuda.synchronize()
    assert not torch.equal(m.params, p0)


def test_failure_on_one_replica_skips_every_replica(s2s):
    """ADVICE r4 (data parallel): two replicas (two contexts on this GPU) with identical parameters; replica A's
    step fails (injected abort), replica B's succeeds.  Their gradients would both go into the all-reduce, so both
    must skip the update.  Each replica's failure flag (s2s_ctx_status_flag, on the device) is summed as the
    all-reduce would (dist.reduce_failure_flag takes the MAX; any nonzero skips), and both optimizers run with it:
    neither replica's parameters change, so the replicas stay identical.  Without the reduced flag B would apply
    the update alone (checked: B's own flag is 0)."""
    from s2s_amd import _lib
    from s2s_amd.optim import Adadelta
    cfg = s2s.ModelConfig()
    a = s2s.ChorowskiBaseline(cfg, overlap=True)
    b = s2s.ChorowskiBaseline(cfg, overlap=True)
    b.params.copy_(a.params)
    assert a.ctx is not b.ctx
    oa, ob = Adadelta(a), Adadelta(b)
    g = torch.Generator().manual_seed(9)
    x = torch.randn(4, 24, cfg.inputFrameSize, generator=g).cuda()
    lab = torch.randint(0, cfg.outputDepth, (4, 6), generator=g).to(torch.int32).cuda()
    z = torch.zeros(1, dtype=torch.float32, device="cuda")
    for m, o in ((a, oa), (b, ob)):  # warm-up: every lazily sized buffer exists, so nothing below syncs the host
        m.step(x, lab)
        o.failure_flag()
        o.step(skip_flag=z)
    torch.cuda.synchronize()
    assert torch.equal(a.params, b.params)
    p0 = a.params.clone()
    try:
        _lib.lib.s2s_debug_inject_abort(1)
        torch.cuda._sleep(200_000_000)  # the host queues everything below before the failure is visible to it
        a.step(x, lab)
        _lib.lib.s2s_debug_inject_abort(0)
        b.step(x, lab)
        fa, fb = oa.failure_flag(), ob.failure_flag()
        flag = fa + fb  # the cross-rank reduction (a sum or a max: nonzero iff any replica failed)
        oa.step(skip_flag=flag)
        ob.step(skip_flag=flag)
        torch.cuda.synchronize()
        assert float(fa.item()) == 1.0 and float(fb.item()) == 0.0
        assert a.ctx.status(clear=False) != 0
    finally:
        _lib.lib.s2s_debug_inject_abort(0)
        a.ctx.status(clear=True)
    assert b.ctx.status() == 0
    assert torch.equal(a.params, p0) and torch.equal(b.params, p0)
    # a clear flag lets both replicas update again, identically
    a.step(x, lab)
    b.step(x, lab)
    oa.step(skip_flag=z)
    ob.step(skip_flag=z)
    torch.cuda.synchronize()
    assert not torch.equal(a.params, p0)
    assert torch.equal(a.params, b.params)
