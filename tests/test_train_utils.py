"""TrainUtils.orthogonalize (TrainUtils.lua:5-26) on host tensors: numpy's LAPACK QR is the checker."""
import numpy as np
import pytest
import torch

from s2s_amd import train_utils as tu
from s2s_amd.model import ModelConfig, param_shapes


def _lapack(w):
    """TrainUtils.lua:8-13 restated with numpy (geqrf / orgqr)."""
    if w.shape[0] < w.shape[1]:
        return np.linalg.qr(w.T, mode="reduced")[0].T
    return np.linalg.qr(w, mode="reduced")[0]


@pytest.mark.parametrize("shape,bias", [((8, 5), False), ((5, 8), False), ((8, 5), True), ((5, 8), True),
                                        ((6, 5), True), ((1, 12), False)])
def test_orthogonalize_matches_lapack_qr(shape, bias):
    g = torch.Generator().manual_seed(3)
    w = torch.rand(shape, generator=g, dtype=torch.float64) * 2 - 1
    b = torch.rand(shape[0], generator=g, dtype=torch.float64) * 2 - 1 if bias else None
    full = w.numpy() if b is None else np.concatenate([w.numpy(), b.numpy()[:, None]], 1)
    q = _lapack(full)
    tu.orthogonalize(w, b)
    np.testing.assert_allclose(w.numpy(), q[:, :shape[1]], atol=1e-12)
    if bias:
        np.testing.assert_allclose(b.numpy(), q[:, shape[1]], atol=1e-12)
    # TrainUtils.lua:29-49 checkOrthogonalization: the smaller Gram matrix is the identity
    m = q @ q.T if q.shape[0] <= q.shape[1] else q.T @ q
    np.testing.assert_allclose(m, np.eye(m.shape[0]), atol=1e-12)


@pytest.mark.parametrize("shape", [(8, 5), (5, 8), (1, 12)])
def test_zero_bias_module_equals_weight_only(shape):
    """TemporalConvolutionZeroBias: the re-zeroed bias column leaves the weight's Q columns unchanged, so the
    flat layout (which drops that bias) orthogonalizes V and we as weight-only modules."""
    g = torch.Generator().manual_seed(5)
    w = torch.rand(shape, generator=g, dtype=torch.float64) - 0.5
    a, b = w.clone(), torch.zeros(shape[0], dtype=torch.float64)
    tu.orthogonalize(a, b)
    tu.orthogonalize(w)
    np.testing.assert_allclose(a.numpy(), w.numpy(), atol=1e-12)


def test_modules_cover_every_weight_once():
    cfg = ModelConfig()
    names = [n for n, _ in param_shapes(cfg)]
    mods = tu.modules(cfg)
    seen = [w for w, _ in mods] + [b for _, b in mods if b]
    assert sorted(seen) == sorted(names)
