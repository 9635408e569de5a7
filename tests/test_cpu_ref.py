"""The C restatement of the training step (oracle/cpu_ref.c: bench.py's CPU baseline) against the float64 NumPy
oracle -- the same function restated twice, so it must agree to fp32 rounding: logp-level nll and every gradient
within 2e-4 of max|ref| (fp32 sums over L frames and T steps)."""
import subprocess

import numpy as np
import pytest

from oracle import cpu_ref
from oracle import s2s_oracle as orc


@pytest.fixture(scope="module", autouse=True)
def built():
    subprocess.run(["make", "-s", "-C", cpu_ref._HERE], check=True)


@pytest.mark.parametrize("B,L,T,penalty,drop", [(3, 17, 5, 0.0, False), (2, 12, 6, 0.3, False), (2, 9, 4, 0.0, True),
                                                (1, 10, 3, 0.0, False)])
def test_cpu_restatement_matches_oracle(B, L, T, penalty, drop):
    cfg = orc.ModelConfig(inputFrameSize=10, hiddenFrameSize=8, outputFrameSize=6, scoreDepth=12, stateDepth=7,
                          outputDepth=9, mlpDepth=3, maxoutWindow=4, penalty=penalty, numLayers=3)
    P = orc.init_params(cfg, seed=5)
    x, lab = orc.synthetic_batch(cfg, B, L, T, seed=7, pad=2, eos=cfg.outputDepth - 1)
    mask = None
    if drop:
        rng = np.random.default_rng(3)
        mask = ((rng.random((B, T, cfg.stateDepth + cfg.annotationDepth)) >= 0.5) / 0.5)
    flat = orc.flatten(P, cfg)
    nll, g = cpu_ref.training_step(x, lab, flat, cfg, dropout_mask=mask, threads=2)
    # the oracle's per-utterance nll (reference semantics: each utterance alone)
    nll_ref = [orc.training_step(x[b:b + 1], lab[b:b + 1], P, cfg, dropout_mask=None if mask is None else mask[b:b + 1])[0]
               for b in range(B)]
    np.testing.assert_allclose(nll, nll_ref, rtol=1e-4)
    _, G, _, _ = orc.training_step(x, lab, P, cfg, dropout_mask=mask)
    gref = orc.flatten(G, cfg)
    off = 0
    for name, shp in orc.param_shapes(cfg):
        n = int(np.prod(shp))
        a, r = g[off:off + n], gref[off:off + n]
        off += n
        assert np.abs(a - r).max() <= 2e-4 * max(np.abs(r).max(), 1e-6), name


def test_cpu_restatement_thread_count_independent():
    cfg = orc.ModelConfig(inputFrameSize=10, hiddenFrameSize=8, outputFrameSize=6, scoreDepth=12, stateDepth=7,
                          outputDepth=9, mlpDepth=3, maxoutWindow=4, numLayers=2)
    P = orc.init_params(cfg, seed=2)
    x, lab = orc.synthetic_batch(cfg, 5, 11, 4, seed=3, pad=2, eos=cfg.outputDepth - 1)
    flat = orc.flatten(P, cfg)
    n1, g1 = cpu_ref.training_step(x, lab, flat, cfg, threads=1)
    n4, g4 = cpu_ref.training_step(x, lab, flat, cfg, threads=4)
    np.testing.assert_array_equal(n1, n4)
    np.testing.assert_allclose(g1, g4, rtol=0, atol=1e-6 * np.abs(g1).max())
