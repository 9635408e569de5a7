"""CPU oracle for the encoder front-ends.

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker; nothing in the product path
(`seq2seq-attention-asr_amd/`, `libs2s_hip.so`) imports or calls it.

NumPy restatement (float64) of the Torch7 `nn` operators (3p, no version pinned by the reference)
that the reference's two other encoders call, with their published semantics:
  * conv + BiLSTM encoder, timit/timit.lua:108-125: 3 x [TemporalConvolution(D, 256, 3) -> ReLU ->
    TemporalMaxPooling(2, 2)] shared by both directions (the same `convlayer` module is applied twice
    to the same input, :123-124, so its output is one tensor and its weight gradient the sum of both
    directions' contributions), then RNN(LSTM(256, 128)) forward and reverse, JoinTable(2,2);
  * VGG encoder, librispeech/model_vgg.lua:23-51: SpatialConvolutionMM(3,64,3,3) ReLU,
    (64,64,3,3) ReLU, SpatialMaxPooling(2,1,2,1), (64,128,3,3) ReLU, (128,128,3,3) ReLU,
    SpatialMaxPooling(2,2,2,2), Transpose2({1,2},3), View(-1, 128*H'), four TemporalConvolution(., ., 1)
    each followed by ReLU.
Operator semantics restated: TemporalConvolution y_t = W [x_t; ...; x_{t+kW-1}] + b, W (out, kW*in)
frame-major (pinned by Attention.ipynb cells 4-6, see s2s_oracle.temporal_conv);
TemporalMaxPooling / SpatialMaxPooling floor mode, first maximum wins (strict >), gradient to the
argmax; SpatialConvolutionMM weight (out, in*kH*kW) in (c, i, j) order, no padding, stride 1, input
(C, H, W) with H = time, W = frequency; ReLU dx = dy * 1[x > 0]; Transpose2 swaps dims 1 and 2 of
(nFeat, L, H) (Transpose2.lua:23-37).  Independently checked against torch.nn.functional autograd in
tests/test_frontend.py.
"""
from typing import Dict, Optional

import numpy as np

from . import s2s_oracle as orc

Array = np.ndarray


# ---------------------------------------------------------------- TemporalConvolution (3p)

def tconv_fwd(x: Array, W: Array, b: Optional[Array], kW: int) -> Array:
    """x (B, L, Din) -> (B, L - kW + 1, Dout); timit/timit.lua:113, model_vgg.lua:43-50."""
    return orc.temporal_conv(W, b, x, kW)


def tconv_bwd(x: Array, W: Array, dy: Array, kW: int):
    """Returns (dx, dW, db) of TemporalConvolution: dW = sum_t dy_t window_t^T, db = sum_t dy_t,
    dx[t] = sum_i (W^T dy_{t-i})[i*Din:(i+1)*Din]."""
    B, L, Din = x.shape
    Lo = L - kW + 1
    win = np.stack([x[:, j:j + Lo, :] for j in range(kW)], axis=-2).reshape(B, Lo, kW * Din)
    dW = np.einsum("blo,blk->ok", dy, win)
    db = dy.sum(axis=(0, 1))
    dU = dy @ W  # (B, Lo, kW*Din)
    dx = np.zeros_like(x)
    for i in range(kW):
        dx[:, i:i + Lo, :] += dU[:, :, i * Din:(i + 1) * Din]
    return dx, dW, db


# ---------------------------------------------------------------- TemporalMaxPooling (3p)

def tmaxpool_fwd(x: Array, kW: int, dW: int):
    """x (B, L, D) -> y (B, (L-kW)//dW + 1, D), idx = argmax offset (first maximum); timit/timit.lua:115."""
    B, L, D = x.shape
    Lo = (L - kW) // dW + 1
    win = np.stack([x[:, i:i + (Lo - 1) * dW + 1:dW, :] for i in range(kW)], axis=0)  # (kW, B, Lo, D)
    idx = np.argmax(win, axis=0)  # numpy argmax returns the first maximum
    y = np.take_along_axis(win, idx[None], axis=0)[0]
    return y, idx


def tmaxpool_bwd(idx: Array, dy: Array, L: int, kW: int, dW: int) -> Array:
    B, Lo, D = dy.shape
    dx = np.zeros((B, L, D), dy.dtype)
    bb, oo, cc = np.meshgrid(np.arange(B), np.arange(Lo), np.arange(D), indexing="ij")
    np.add.at(dx, (bb, oo * dW + idx, cc), dy)
    return dx


# ---------------------------------------------------------------- ReLU (3p)

def relu_fwd(x: Array) -> Array:
    return np.maximum(x, 0.0)


def relu_bwd(x: Array, dy: Array) -> Array:
    return np.where(x > 0, dy, 0.0)


def relu_gate(u: Array, mask: Optional[Array]):
    """ReLU with an optionally adopted decision mask: -> (output, gate), relu_bwd(gate, dy) being the backward.
    Without a mask the gate is u itself."""
    if mask is None:
        return np.maximum(u, 0.0), u
    return np.where(mask, u, 0.0), np.where(mask, 1.0, -1.0)


# ---------------------------------------------------------------- SpatialConvolutionMM (3p)

def _im2col(x: Array, kH: int, kW: int) -> Array:
    """x (B, C, H, W) -> (B, C*kH*kW, Ho*Wo) in (c, i, j) row order."""
    B, C, H, W = x.shape
    Ho, Wo = H - kH + 1, W - kW + 1
    cols = np.stack([x[:, :, i:i + Ho, j:j + Wo] for i in range(kH) for j in range(kW)], axis=2)  # (B,C,kHkW,Ho,Wo)
    return cols.reshape(B, C * kH * kW, Ho * Wo)


def sconv_fwd(x: Array, Wt: Array, b: Optional[Array], kH: int, kW: int) -> Array:
    """model_vgg.lua:24-32: y[b, o] = Wt[o] . unfold(x[b]) + b[o]."""
    B, C, H, W = x.shape
    Ho, Wo = H - kH + 1, W - kW + 1
    y = np.einsum("ok,bkn->bon", Wt, _im2col(x, kH, kW))
    if b is not None:
        y = y + b[None, :, None]
    return y.reshape(B, Wt.shape[0], Ho, Wo)


def sconv_bwd(x: Array, Wt: Array, dy: Array, kH: int, kW: int):
    B, C, H, W = x.shape
    Ho, Wo = H - kH + 1, W - kW + 1
    O = Wt.shape[0]
    d2 = dy.reshape(B, O, Ho * Wo)
    dW = np.einsum("bon,bkn->ok", d2, _im2col(x, kH, kW))
    db = d2.sum(axis=(0, 2))
    dcol = np.einsum("ok,bon->bkn", Wt, d2).reshape(B, C, kH, kW, Ho, Wo)
    dx = np.zeros_like(x)
    for i in range(kH):
        for j in range(kW):
            dx[:, :, i:i + Ho, j:j + Wo] += dcol[:, :, i, j]
    return dx, dW, db


# ---------------------------------------------------------------- SpatialMaxPooling (3p)

def smaxpool_fwd(x: Array, kW: int, kH: int, dW: int, dH: int, idx: Optional[Array] = None):
    """x (B, C, H, W) -> y (B, C, Ho, Wo); idx = i*kW + j of the window's first maximum (scan i then j).
    A given idx (a decision adopted from the implementation under test) is used instead of the argmax."""
    B, C, H, W = x.shape
    Ho, Wo = (H - kH) // dH + 1, (W - kW) // dW + 1
    win = np.stack([x[:, :, i:i + (Ho - 1) * dH + 1:dH, j:j + (Wo - 1) * dW + 1:dW]
                    for i in range(kH) for j in range(kW)], axis=0)
    if idx is None:
        idx = np.argmax(win, axis=0)
    y = np.take_along_axis(win, idx[None], axis=0)[0]
    return y, idx


def smaxpool_bwd(idx: Array, dy: Array, H: int, W: int, kW: int, kH: int, dW: int, dH: int) -> Array:
    B, C, Ho, Wo = dy.shape
    dx = np.zeros((B, C, H, W), dy.dtype)
    bb, cc, oh, ow = np.meshgrid(np.arange(B), np.arange(C), np.arange(Ho), np.arange(Wo), indexing="ij")
    np.add.at(dx, (bb, cc, oh * dH + idx // kW, ow * dW + idx % kW), dy)
    return dx


# ---------------------------------------------------------------- encoders

def conv_stack_fwd(x: Array, P: Dict[str, Array], nconv: int = 3, kW: int = 3):
    """The shared `convlayer` of timit/timit.lua:112-121 on x (B, L, D)."""
    cache = []
    h = x
    for l in range(nconv):
        u = tconv_fwd(h, P[f"conv{l}.W"], P[f"conv{l}.b"], kW)
        r = relu_fwd(u)
        p, idx = tmaxpool_fwd(r, 2, 2)
        cache.append((h, u, idx, r.shape[1]))
        h = p
    return h, cache


def conv_stack_bwd(P: Dict[str, Array], cache, dout: Array, G: Dict[str, Array], kW: int = 3, scale: float = 1.0):
    d = dout
    for l in reversed(range(len(cache))):
        h, u, idx, Lr = cache[l]
        dr = tmaxpool_bwd(idx, d, Lr, 2, 2)
        du = relu_bwd(u, dr)
        dx, dW, db = tconv_bwd(h, P[f"conv{l}.W"], du, kW)
        G[f"conv{l}.W"] += scale * dW
        G[f"conv{l}.b"] += scale * db
        d = dx
    return d


def _lstm_p(P, prefix):
    return {k[len(prefix):]: v for k, v in P.items() if k.startswith(prefix)}


def conv_bilstm_fwd(x: Array, P: Dict[str, Array]):
    """timit/timit.lua:108-125: conv stack -> [RNN(LSTM) fwd | RNN(LSTM) reverse] (JoinTable(2,2))."""
    c, ccache = conv_stack_fwd(x, P)
    yf, sf = orc.lstm_seq_fwd(c, _lstm_p(P, "f."), reverse=False)
    yb, sb = orc.lstm_seq_fwd(c, _lstm_p(P, "b."), reverse=True)
    return np.concatenate([yf, yb], axis=-1), (c, ccache, sf, sb)


def conv_bilstm_bwd(P: Dict[str, Array], cache, dout: Array, G: Dict[str, Array], scale: float = 1.0):
    c, ccache, sf, sb = cache
    H = dout.shape[-1] // 2
    gf, gb = {k: np.zeros_like(v) for k, v in _lstm_p(P, "f.").items()}, {k: np.zeros_like(v) for k, v in
                                                                          _lstm_p(P, "b.").items()}
    dcf = orc.lstm_seq_bwd(c, _lstm_p(P, "f."), sf, dout[..., :H], gf, reverse=False, scale=scale)
    dcb = orc.lstm_seq_bwd(c, _lstm_p(P, "b."), sb, dout[..., H:], gb, reverse=True, scale=scale)
    for k, v in gf.items():
        G["f." + k] += v
    for k, v in gb.items():
        G["b." + k] += v
    return conv_stack_bwd(P, ccache, dcf + dcb, G, scale=scale)


VGG_CONVS = ((3, 64), (64, 64), (64, 128), (128, 128))
VGG_POOLS = {1: (2, 1, 2, 1), 3: (2, 2, 2, 2)}  # after conv index: (kW, kH, dW, dH)


def vgg_dims(F: int, hidden: int = 2048, out: int = 512):
    Hf = ((F - 4) // 2 - 4) // 2
    return [(128 * Hf, hidden), (hidden, hidden), (hidden, hidden), (hidden, out)]


def vgg_fwd(x: Array, P: Dict[str, Array], decide: Optional[dict] = None, raw: Optional[dict] = None):
    """librispeech/model_vgg.lua:23-51 on x (B, 3, L, F) -> (B, (L-8)//2, out).
    decide (tests only): the discrete decisions of an implementation under test, run instead of the oracle's own
    -- {"conv": [ReLU mask per conv layer], "pool": {layer: SpatialMaxPooling idx}, "lin": [ReLU mask per 1x1
    layer]}; raw (a dict, filled) then receives the oracle's own pre-activations and pool argmaxes under those
    upstream decisions, for the caller to check that the two agree off the near-tie band."""
    cache = {"conv": [], "pool": {}, "lin": []}
    if raw is not None:
        raw.update({"conv": [], "pool": {}, "pool_in": {}, "lin": []})
    dc = decide or {}
    h = x
    for l in range(4):
        u = sconv_fwd(h, P[f"vgg{l}.W"], P[f"vgg{l}.b"], 3, 3)
        r, gate = relu_gate(u, dc["conv"][l] if "conv" in dc else None)
        cache["conv"].append((h, gate))
        if raw is not None:
            raw["conv"].append(u)
        h = r
        if l in VGG_POOLS:
            kW, kH, dW, dH = VGG_POOLS[l]
            if raw is not None:
                raw["pool"][l] = smaxpool_fwd(h, kW, kH, dW, dH)[1]
                raw["pool_in"][l] = h
            p, idx = smaxpool_fwd(h, kW, kH, dW, dH, dc["pool"][l] if "pool" in dc else None)
            cache["pool"][l] = (idx, h.shape)
            h = p
    B, C, Lq, Hf = h.shape
    cache["tshape"] = h.shape
    h = h.transpose(0, 2, 1, 3).reshape(B, Lq, C * Hf)  # Transpose2({1,2},3) + View(-1, 128*H)
    for l in range(4):
        u = tconv_fwd(h, P[f"lin{l}.W"], P[f"lin{l}.b"], 1)
        r, gate = relu_gate(u, dc["lin"][l] if "lin" in dc else None)
        cache["lin"].append((h, gate))
        if raw is not None:
            raw["lin"].append(u)
        h = r
    return h, cache


def vgg_bwd(P: Dict[str, Array], cache, dout: Array, G: Dict[str, Array], scale: float = 1.0):
    d = dout
    for l in reversed(range(4)):
        h, u = cache["lin"][l]
        du = relu_bwd(u, d)
        dx, dW, db = tconv_bwd(h, P[f"lin{l}.W"], du, 1)
        G[f"lin{l}.W"] += scale * dW
        G[f"lin{l}.b"] += scale * db
        d = dx
    B, C, Lq, Hf = cache["tshape"]
    d = d.reshape(B, Lq, C, Hf).transpose(0, 2, 1, 3)
    for l in reversed(range(4)):
        if l in VGG_POOLS:
            kW, kH, dW, dH = VGG_POOLS[l]
            idx, shp = cache["pool"][l]
            d = smaxpool_bwd(idx, d, shp[2], shp[3], kW, kH, dW, dH)
        h, u = cache["conv"][l]
        du = relu_bwd(u, d)
        dx, dW, db = sconv_bwd(h, P[f"vgg{l}.W"], du, 3, 3)
        G[f"vgg{l}.W"] += scale * dW
        G[f"vgg{l}.b"] += scale * db
        d = dx
    return d


# ---------------------------------------------------------------- decoder_mlp stacks (3p nn + Maxout.lua)

def mlp_fwd(v: Array, layers, maxout_idx=None, raw: Optional[list] = None):
    """A decoder_mlp Sequential on rows v (N, D): layers are ("maxout", W, b, window) (Maxout.lua:14-18:
    Linear + TemporalMaxPooling(window, window) over consecutive groups), ("linear", W, b), ("relu",),
    ("logsoftmax",).  maxout_idx (tests only): one adopted winner array (N, out) per Maxout layer, in order,
    run instead of the argmax; raw (a list, filled) then receives each Maxout's pre-activations (N, out, window)."""
    cache = []
    h = v
    mi = 0
    for L in layers:
        if L[0] == "maxout":
            _, W, b, k = L
            u = h @ W.T + b
            g = u.reshape(u.shape[0], -1, k)
            if raw is not None:
                raw.append(g)
            am = np.argmax(g, axis=2) if maxout_idx is None else maxout_idx[mi]
            mi += 1
            cache.append((h, am, u.shape))
            h = np.take_along_axis(g, am[..., None], axis=2)[..., 0]
        elif L[0] == "linear":
            cache.append((h,))
            h = h @ L[1].T + L[2]
        elif L[0] == "relu":
            cache.append((h,))
            h = relu_fwd(h)
        else:
            h = orc.log_softmax(h, 1)
            cache.append((h,))
    return h, cache


def mlp_bwd(layers, cache, dout: Array, grads, scale: float = 1.0) -> Array:
    """grads: list of (dW, db) per maxout / linear layer (None for relu / logsoftmax), accumulated."""
    d = dout
    for L, c, gr in zip(reversed(layers), reversed(cache), reversed(grads)):
        if L[0] == "maxout":
            _, W, b, k = L
            h, am, ushape = c
            du = np.zeros(ushape, d.dtype).reshape(ushape[0], -1, k)
            np.put_along_axis(du, am[..., None], d[..., None], axis=2)
            du = du.reshape(ushape)
            gr[0][...] += scale * (du.T @ h)
            gr[1][...] += scale * du.sum(0)
            d = du @ W
        elif L[0] == "linear":
            (h,) = c
            gr[0][...] += scale * (d.T @ h)
            gr[1][...] += scale * d.sum(0)
            d = d @ L[1]
        elif L[0] == "relu":
            d = relu_bwd(c[0], d)
        else:
            (y,) = c
            d = d - np.exp(y) * d.sum(1, keepdims=True)
    return d


def vgg_model_step(x: Array, labels: Array, P: Dict[str, Array], mlp_layers, cfg, decide: Optional[dict] = None,
                   maxout_idx=None, raw: Optional[dict] = None):
    """librispeech/model_vgg.lua end to end + the trainer's loss seed (train.lua:139-165): VGG encoder,
    attention decoder (GRU recurrence) with the external decoder_mlp stack, nll = -sum onehot * logp,
    dlogp = -onehot, gradients summed over the batch then / B.  P holds the encoder (vgg*/lin*) and the
    decoder's own parameters; cfg an s2s_oracle.ModelConfig for the decoder dims.
    decide / maxout_idx / raw (tests only): adopted decisions and the oracle's own pre-decision values, as in
    vgg_fwd and mlp_fwd (raw["mlp"] holds the Maxout pre-activations).
    Returns (nll per utterance, logp, G encoder+decoder, mlp grads)."""
    B = x.shape[0]
    h, ecache = vgg_fwd(x, P, decide, raw)
    Pd = dict(P)
    S, A, M, k, O = cfg.stateDepth, cfg.annotationDepth, cfg.mlpDepth, cfg.maxoutWindow, cfg.outputDepth
    for name, shp in (("Wm", (M * k, S + A)), ("bm", (M * k,)), ("Wo", (O, M)), ("bo", (O,))):
        Pd.setdefault(name, np.zeros(shp))  # the fused MLP is not used (external decoder_mlp)
    _, acache = orc.attention_fwd(h, labels, Pd, cfg)
    T = labels.shape[1]
    v = acache["v"].reshape(B * T, -1)
    mraw = raw.setdefault("mlp", []) if raw is not None else None
    logp, mcache = mlp_fwd(v, mlp_layers, maxout_idx, mraw)
    logp = logp.reshape(B, T, O)
    onehot = np.zeros_like(logp)
    np.put_along_axis(onehot, labels[..., None].astype(np.int64), 1.0, axis=2)
    nll = -(onehot * logp).sum(axis=(1, 2))
    scale = 1.0 / B if B > 1 else 1.0
    mgrads = [(np.zeros_like(L[1]), np.zeros_like(L[2])) if L[0] != "logsoftmax" else None for L in mlp_layers]
    dv = mlp_bwd(mlp_layers, mcache, (-onehot).reshape(B * T, O), mgrads, scale)
    G = {kk: np.zeros_like(vv) for kk, vv in Pd.items()}
    dh = orc.attention_bwd(Pd, cfg, acache, None, G, scale, dmlp_in=dv.reshape(B, T, -1))
    vgg_bwd(P, ecache, dh, G, scale)
    return nll, logp, G, mgrads


def vgg_random_case(F: int = 40, hidden: int = 2048, out: int = 512, S: int = 256, Sc: int = 512, O: int = 29,
                    M: int = 64, seed: int = 1234, dtype=np.float32):
    """Parameters of a librispeech/model_vgg.lua model at the reference's default init (U(+-1/sqrt(fan_in)),
    nn.Linear / SpatialConvolutionMM / TemporalConvolution resets) as (P, mlp layers, decoder cfg) for
    vgg_model_step: the CPU-baseline workload of bench.py's config-5 line (a port of the reference, timed)."""
    rng = np.random.default_rng(seed)

    def u(shape, fan_in):
        return (rng.uniform(-1.0, 1.0, shape) / np.sqrt(fan_in)).astype(dtype)

    P = {}
    for l, (ci, co) in enumerate(VGG_CONVS):
        P[f"vgg{l}.W"], P[f"vgg{l}.b"] = u((co, ci * 9), ci * 9), u((co,), ci * 9)
    for l, (di, do) in enumerate(vgg_dims(F, hidden, out)):
        P[f"lin{l}.W"], P[f"lin{l}.b"] = u((do, di), di), u((do,), di)
    A = out
    for name, shape, fan in (("V", (Sc, A), A), ("Ws", (Sc, S), S), ("bs", (Sc,), S), ("we", (1, Sc), Sc),
                             ("Wy", (S, O), O), ("by", (S,), O), ("Wc", (S, A), A), ("bc", (S,), A),
                             ("Wd", (S, 2 * S), 2 * S), ("bd", (S,), 2 * S), ("dec.Wz", (S, 2 * S), 2 * S),
                             ("dec.Wr", (S, 2 * S), 2 * S), ("dec.Wh", (S, 2 * S), 2 * S)):
        P[name] = u(shape, fan)
    k = 7
    layers = [("maxout", u((M * k, S + A), S + A), u((M * k,), S + A), k), ("linear", u((M, M), M), u((M,), M)),
              ("maxout", u((M * k, M), M), u((M * k,), M), k), ("linear", u((O, M), M), u((O,), M)),
              ("logsoftmax",)]
    cfg = orc.ModelConfig(inputFrameSize=8, hiddenFrameSize=16, outputFrameSize=A // 2, scoreDepth=Sc, stateDepth=S,
                          outputDepth=O, mlpDepth=M, maxoutWindow=k, numLayers=1)
    return P, layers, cfg
