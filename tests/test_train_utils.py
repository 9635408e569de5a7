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


@pytest.mark.parametrize("shape", [(8, 5), (5, 8), (1, 12), (6, 6)])
def test_zero_bias_module_matches_reference_zero_column(shape):
    """TemporalConvolutionZeroBias (TrainUtils.lua:6-15 sees [W | 0]): the zero column leaves the weight's Q
    columns unchanged when W is tall or wide, but a square W becomes wide and takes the qr(w^T)^T branch --
    orthogonalize_model therefore passes an explicit zero column (ZERO_BIAS) and its result must equal the
    reference's [W | 0] QR in every case, the square one included."""
    g = torch.Generator().manual_seed(5)
    w = torch.rand(shape, generator=g, dtype=torch.float64) - 0.5
    ref = _lapack(np.concatenate([w.numpy(), np.zeros((shape[0], 1))], 1))[:, :shape[1]]
    a, b = w.clone(), torch.zeros(shape[0], dtype=torch.float64)
    tu.orthogonalize(a, b)
    np.testing.assert_allclose(a.numpy(), ref, atol=1e-12)
    if shape[0] != shape[1]:  # weight-only agrees off the square case
        tu.orthogonalize(w)
        np.testing.assert_allclose(a.numpy(), w.numpy(), atol=1e-12)


def test_orthogonalize_model_square_V_uses_zero_column():
    """At the default config V is (Sc, A) = (512, 512): orthogonalize_model must give the [V | 0] result."""
    from s2s_amd.model import ModelConfig as MC

    class _M:  # the flat views orthogonalize_model reads (no device needed)
        cfg = MC(inputFrameSize=5, hiddenFrameSize=4, outputFrameSize=4, scoreDepth=8, stateDepth=4,
                 outputDepth=7, mlpDepth=3, maxoutWindow=2, numLayers=1)

        def __init__(self):
            g = torch.Generator().manual_seed(9)
            self.shapes = param_shapes(self.cfg)
            n = sum(int(np.prod(s)) for _, s in self.shapes)
            self.flat = torch.rand(n, generator=g, dtype=torch.float64) - 0.5

        def views(self):
            out, off = {}, 0
            for name, shp in self.shapes:
                sz = int(np.prod(shp))
                out[name] = self.flat[off:off + sz].view(shp)
                off += sz
            return out

    m = _M()
    V0 = m.views()["V"].clone().numpy()
    assert V0.shape[0] == V0.shape[1]
    tu.orthogonalize_model(m)
    ref = _lapack(np.concatenate([V0, np.zeros((V0.shape[0], 1))], 1))[:, :V0.shape[1]]
    np.testing.assert_allclose(m.views()["V"].numpy(), ref, atol=1e-12)


def test_modules_cover_every_weight_once():
    cfg = ModelConfig()
    names = [n for n, _ in param_shapes(cfg)]
    mods = tu.modules(cfg)
    seen = [w for w, _ in mods] + [b for _, b in mods if b and b != tu.ZERO_BIAS]
    assert sorted(seen) == sorted(names)
