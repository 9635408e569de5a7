"""GPU parity at the full shapes the bench reports (VERDICT r1 "next" 1): the whole training step of
BASELINE config 4 at its single-GPU shape and of the config-5 VGG model at full width, against the
float64 oracle.

* Config 4 (librispeech/model_chorowski_baseline.lua:10-83): F = 80, O = 29 chars, L = 400, T = 200, B = 25
  -- 7 XCD decoder chains of 4 utterances and a ragged last chain of 1, the streamed (Vh-resident,
  h-from-L2) decoder kernels the B = 32 bench runs, run exactly as the bench runs it (hipGraph replay,
  side-stream weight gradients).  Tolerance: the fp32 bar, max|gpu - ref| <= 1e-4 max|ref| per tensor.
* Config 5 (librispeech/model_vgg.lua:23-82): the VGG stack on (B, 3, 1024, 40), 1x1 layers 2048 wide,
  A = 512, S = 256, Sc = 512, T = 200 chars, B = 2, at the conditioned test point of tests/vgg_case.py
  (`condition`: He gain on the encoder weights -- at the default init the annotations are bias-dominated, the
  attention is uniform and the score layer's gradients cancel to ~1e-11, so they could not be judged).  Every
  tensor is held to 1e-4 except the encoder layers' weight / bias gradients (VGG convolutions and 1x1 layers), sums
  over ~1e4-1e5 pixels / frames whose fp32 evaluation in any order reaches ~1e-4 (the fp32 run of the same
  restatement against float64: e32 up to 6.3e-4, the first 1x1 layer): those are held to 16 e32 (a different,
  equally valid blocked summation order), and e32 itself must stay below 1e-3 so the escape is bounded.
"""
import numpy as np
import pytest
import torch

from oracle import s2s_oracle as orc

pytestmark = pytest.mark.gpu
RTOL = 1e-4
# the encoder layers' weight / bias gradients (long pixel / frame sums): bar = max(RTOL, FLOOR_FACTOR x the fp32
# restatement's own error), that error itself bounded by FLOOR_CAP
FLOOR_FACTOR = 16
FLOOR_CAP = 1e-3

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
    vc.condition(model, fe)
    rng = np.random.default_rng(5)
    x = rng.standard_normal((B, 3, L, 40)).astype(np.float32).astype(np.float64)
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
    # the attention score layer's gradients are conditioned at this test point: their fp32 floor is far below the bar
    att = {k: f"{floor[k]:.1e}" for k in ("dV", "dWs", "dbs", "dwe") if not floor[k] <= 1e-5}
    assert not att, att
    conv = {k for k in errs if k.startswith("dvgg") or k.startswith("dlin")}
    uncapped = {k: f"{floor[k]:.1e}" for k in conv if not floor[k] <= FLOOR_CAP}
    assert not uncapped, uncapped
    bad = {k: f"{errs[k]:.2e} (fp32 floor {floor[k]:.2e})" for k in errs
           if not errs[k] <= (max(RTOL, FLOOR_FACTOR * floor[k]) if k in conv else RTOL)}
    assert not bad, bad
