"""GPU parity at the full shapes the bench reports (VERDICT r1 "next" 1): the whole training step of
BASELINE config 4 at its single-GPU shape and of the config-5 VGG model at full width, against the
float64 oracle.

* Config 4 (librispeech/model_chorowski_baseline.lua:10-83): F = 80, O = 29 chars, L = 400, T = 200, B = 25
  -- 7 XCD decoder chains of 4 utterances and a ragged last chain of 1, the streamed (Vh-resident,
  h-from-L2) decoder kernels the B = 32 bench runs, run exactly as the bench runs it (hipGraph replay,
  side-stream weight gradients).  Tolerance: the fp32 bar, max|gpu - ref| <= 1e-4 max|ref| per tensor.
* Config 5 (librispeech/model_vgg.lua:23-82): the VGG stack on (B, 3, 1024, 40), 1x1 layers 2048 wide,
  A = 512, S = 256, Sc = 512, T = 200 chars, default init (no rescaling), B = 2.  At the default init
  some gradients are sums whose terms cancel to ~1e-5 .. 1e-8 of their size (dWs max |.| ~1e-11: the
  attention is nearly uniform); the reference's own fp32 arithmetic cannot get those to 1e-4.  Per
  tensor the bar is max(1e-4, 16 e32), with e32 = the relative error of the fp32 run of the same
  restatement (identical algorithm, numpy's summation order) against float64 on these inputs: a
  tensor is pinned as tightly as fp32 evaluation of the reference algorithm allows, with a factor 16
  for a different (equally valid) fp32 summation order -- the weight-gradient GEMMs accumulate
  K ~ 1e4 products in blocked sequential MFMA chains plus split-K partials, numpy sums pairwise
  (measured: dvgg3.W 5.8e-4 on the GPU vs e32 = 8.3e-5).
"""
import numpy as np
import pytest
import torch

from oracle import s2s_oracle as orc

pytestmark = pytest.mark.gpu
RTOL = 1e-4
# ill-conditioned tensors: bar = max(RTOL, FLOOR_FACTOR x the fp32 restatement's own error), see
# tests/test_gpu_fullsize.py
FLOOR_FACTOR = 16


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


def test_model_step_config4_full_shape(s2s):
    kw = dict(inputFrameSize=80, outputDepth=29)
    B, L, T = 25, 400, 200
    cfg_o = orc.ModelConfig(**kw)
    model = s2s.ChorowskiBaseline(s2s.ModelConfig(**kw), graph=True, overlap=True)
    P = orc.unflatten(model.params.cpu().double().numpy(), cfg_o)
    x, labels = orc.synthetic_batch(cfg_o, B, L, T, seed=41, pad=1, eos=28)
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    xs, ls = cu(x), cu(labels, torch.int32)
    with torch.cuda.stream(st):
        for _ in range(2):  # capture, then a replay: the replay's results are checked
            nll, logp = model.step(xs, ls, stream=st)
    st.synchronize()
    assert model.ctx.graph_stats()[:2] == (1, 2)
    nll_ref, G, lref, enc = orc.training_step(x, labels, P, cfg_o)
    errs = {"logp": rel(logp.cpu().numpy(), lref), "encoder.output": rel(model.encoder_output().cpu().numpy(), enc)}
    Gg = orc.unflatten(model.grads.cpu().double().numpy(), cfg_o)
    errs.update({"grad " + k: rel(Gg[k], G[k]) for k in G})
    print("config 4 max rel errs:", {k: f"{v:.1e}" for k, v in errs.items()})
    bad = {k: f"{v:.2e}" for k, v in errs.items() if not v <= RTOL}
    assert not bad, bad
    assert abs(float(nll.mean()) - nll_ref) <= RTOL * abs(nll_ref)


def test_vgg_model_step_config5_full_width(s2s):
    import vgg_case as vc
    from s2s_amd import frontend as fe
    g = torch.Generator().manual_seed(5)
    B, L, T = 2, 1024, 200
    model = s2s.VGGAttentionModel(40, outputFrameSize=512, hidden=2048, outputDepth=29, generator=g).cuda()
    rng = np.random.default_rng(5)
    x = rng.standard_normal((B, 3, L, 40))
    labels = np.append(rng.integers(0, 28, (B, T - 1)), np.full((B, 1), 28), axis=1).astype(np.int32)
    model.zeroGradParameters()
    nll, logp = model.step(cu(x), cu(labels, torch.int32))
    torch.cuda.synchronize()
    nll64, logp64, G64, mg64 = vc.oracle_step(model, fe, x, labels, np.float64)
    nll32, logp32, G32, mg32 = vc.oracle_step(model, fe, x, labels, np.float32)
    floor = {"logp": rel(logp32, logp64), "nll": rel(nll32, nll64)}
    errs = {"logp": rel(logp.cpu().numpy(), logp64), "nll": rel(nll.cpu().numpy(), nll64)}
    pairs64 = vc.grad_pairs(model, fe, G64, mg64)
    pairs32 = vc.grad_pairs(model, fe, G32, mg32)
    for (name, gpu, r64), (_, _, r32) in zip(pairs64, pairs32):
        errs[name] = rel(gpu.detach().cpu().numpy(), r64)
        floor[name] = rel(r32, r64)
    print("config 5 max rel errs (fp32 floor):", {k: f"{errs[k]:.1e} ({floor[k]:.1e})" for k in errs})
    bad = {k: f"{errs[k]:.2e} (fp32 floor {floor[k]:.2e})" for k in errs if not errs[k] <= max(RTOL, FLOOR_FACTOR * floor[k])}
    assert not bad, bad
    # every tensor the fp32 restatement gets to 1e-5 must also be within the plain 1e-4 bar
    strict = {k: f"{errs[k]:.2e}" for k in errs if floor[k] <= 1e-5 and not errs[k] <= RTOL}
    assert not strict, strict
