"""TrainUtils.orthogonalize / orthogonalizeGraph (TrainUtils.lua:5-26, 137-188) on the flat layout.

The reference applies `orthogonalize` to every weight-bearing leaf module of the autoencoder after
`reset(init_std)` when `opt.orthogonalize` is set (librispeech/exp0_scriptchecker.lua:49-52,
timit/exp_logmel7_chorowski_normNLL_colnorm.lua:39).  Per module: `w = [weight | bias]` (bias as one
more column when the module has one), Q of a Householder QR of w (of w^T when w has fewer rows than
columns, then transposed back), and the module's weight / bias take Q's columns.  Init-time host code,
outside the timed step; the QR runs where the parameters live (LAPACK geqrf / orgqr, the algorithm
Torch7's torch.qr calls, so Q's column signs follow the same convention).
"""
import torch

from .model import param_shapes

# bias slot of a TemporalConvolutionZeroBias module: a zero column that takes part in the QR and is thrown away
ZERO_BIAS = "<zero bias>"


def orthogonalize(weight, bias=None):
    """TrainUtils.lua:5-26 on one module, in place.  weight (rows, cols), bias (rows,) or None."""
    w = weight if bias is None else torch.cat([weight, bias.reshape(-1, 1)], 1)
    w = w.double()
    if w.shape[0] < w.shape[1]:
        q = torch.linalg.qr(w.t(), mode="reduced")[0].t()
    else:
        q = torch.linalg.qr(w, mode="reduced")[0]
    weight.copy_(q[:, :weight.shape[1]])
    if bias is not None:
        bias.copy_(q[:, weight.shape[1]])
    return weight, bias


def modules(cfg):
    """(weight name, bias name or None) of every leaf module of the Chorowski autoencoder that holds a
    weight, in the flat layout's naming (model.param_shapes).  The encoder's GRU gates are
    LinearZeroBias (weight only, GRU.lua:22-25).  V and we are TemporalConvolutionZeroBias: a bias
    that reset() and updateOutput zero (TemporalConvolutionZeroBias.lua:13-38) and the flat layout drops.
    TrainUtils.lua:6-15 still sees [W | 0]: a zero column changes neither Q's weight columns in the tall
    case (QR is column-sequential) nor Q^T's in the wide case (its row of w^T is zero), but a SQUARE W
    becomes wide and takes the qr(w^T)^T branch, a different Q (V is (Sc, A) = (512, 512) at the
    defaults).  So both carry ZERO_BIAS: orthogonalized with an explicit zero column, which is dropped.
    Ws / Wy / Wc / Wd / Wm / Wo are nn.Linear (weight + bias); the decoder GRU's gates are
    LinearZeroBias."""
    names = [n for n, _ in param_shapes(cfg)]
    out = []
    for n in names:
        if n.startswith("enc") or n.startswith("dec."):
            out.append((n, None))
        elif n in ("V", "we"):
            out.append((n, ZERO_BIAS))
    for w, b in (("Ws", "bs"), ("Wy", "by"), ("Wc", "bc"), ("Wd", "bd"), ("Wm", "bm"), ("Wo", "bo")):
        out.append((w, b))
    return out


@torch.no_grad()
def orthogonalize_model(model):
    """TrainUtils.orthogonalizeGraph(model.autoencoder) on a ChorowskiBaseline's flat parameters."""
    v = model.views()
    for w, b in modules(model.cfg):
        if b == ZERO_BIAS:
            orthogonalize(v[w], torch.zeros(v[w].shape[0], dtype=v[w].dtype, device=v[w].device))
        else:
            orthogonalize(v[w], v[b] if b is not None else None)
    return model
