"""The BASELINE config-5 model (librispeech/model_vgg.lua: VGG conv stack -> 1x1 TemporalConvolutions ->
attention decoder with the two-Maxout decoder_mlp, :23-82) as an oracle case: parameters of an
s2s_amd.VGGAttentionModel (default Torch7-style init, no rescaling) in the oracle's dict layout, and the
oracle step in float64 or float32 (the float32 run measures how far the reference's own fp32 arithmetic
can be from the exact result on this case -- the floor any fp32 implementation is judged against)."""
import numpy as np

from oracle import frontend_oracle as fo
from oracle import s2s_oracle as orc


def _np(t, dtype):
    return t.detach().cpu().numpy().astype(dtype)


def oracle_params(model, fe, dtype=np.float64):
    """-> (P, mlp layers, decoder cfg) of a VGGAttentionModel (s2s_amd.frontend as fe)."""
    enc_mods = model.encoder.seq.modules
    P = {}
    for l, m in enumerate([m for m in enc_mods if isinstance(m, fe.SpatialConvolutionMM)]):
        P[f"vgg{l}.W"], P[f"vgg{l}.b"] = _np(m.weight, dtype), _np(m.bias, dtype)
    for l, m in enumerate([m for m in enc_mods if isinstance(m, fe.TemporalConvolution)]):
        P[f"lin{l}.W"], P[f"lin{l}.b"] = _np(m.weight, dtype), _np(m.bias, dtype)
    dec = model.decoder
    names = ("V", "Ws", "bs", "we", "Wy", "by", "Wc", "bc", "Wd", "bd", "dec.Wz", "dec.Wr", "dec.Wh")
    for n, t in zip(names, dec._tensors(False)[:13]):
        P[n] = _np(t, dtype)
    layers = []
    for m in dec.decoder_mlp.modules:
        if isinstance(m, fe.Maxout):
            layers.append(("maxout", _np(m.linear.weight, dtype), _np(m.linear.bias, dtype), m.window))
        elif isinstance(m, fe.Linear):
            layers.append(("linear", _np(m.weight, dtype), _np(m.bias, dtype)))
        else:
            layers.append(("logsoftmax",))
    cfg = orc.ModelConfig(inputFrameSize=8, hiddenFrameSize=16, outputFrameSize=dec.annotationDepth // 2,
                          scoreDepth=dec.scoreDepth, stateDepth=dec.stateDepth, outputDepth=dec.outputDepth,
                          mlpDepth=8, maxoutWindow=7, numLayers=1)
    return P, layers, cfg


def grad_pairs(model, fe, G, mg):
    """[(name, gpu gradient tensor, oracle gradient)] over every parameter of the model."""
    enc_mods = model.encoder.seq.modules
    dec = model.decoder
    pairs = []
    for l, m in enumerate([m for m in enc_mods if isinstance(m, fe.SpatialConvolutionMM)]):
        pairs += [(f"dvgg{l}.W", m.gradWeight, G[f"vgg{l}.W"]), (f"dvgg{l}.b", m.gradBias, G[f"vgg{l}.b"])]
    for l, m in enumerate([m for m in enc_mods if isinstance(m, fe.TemporalConvolution)]):
        pairs += [(f"dlin{l}.W", m.gradWeight, G[f"lin{l}.W"]), (f"dlin{l}.b", m.gradBias, G[f"lin{l}.b"])]
    names = ("V", "Ws", "bs", "we", "Wy", "by", "Wc", "bc", "Wd", "bd", "dec.Wz", "dec.Wr", "dec.Wh")
    for n, g in zip(names, dec._tensors(True)[:13]):
        pairs.append(("d" + n, g, G[n]))
    mods = [m for m in dec.decoder_mlp.modules if not isinstance(m, fe.LogSoftMax)]
    for i, (m, g) in enumerate(zip(mods, [g for g in mg if g is not None])):
        lin = m.linear if isinstance(m, fe.Maxout) else m
        pairs += [(f"dmlp{i}.W", lin.gradWeight, g[0]), (f"dmlp{i}.b", lin.gradBias, g[1])]
    return pairs


def oracle_step(model, fe, x, labels, dtype=np.float64):
    P, layers, cfg = oracle_params(model, fe, dtype)
    return fo.vgg_model_step(x.astype(dtype), labels, P, layers, cfg)


def rel(a, r):
    a = np.asarray(a, np.float64)
    r = np.asarray(r, np.float64)
    return float(np.abs(a - r).max() / max(np.abs(r).max(), 1e-30))
