"""CPU oracle for the attention-seq2seq ASR training step (forward + backward).

TEST INFRASTRUCTURE ONLY.  Nothing in the product path (`seq2seq-attention-asr_amd/`,
`libs2s_hip.so`) imports, links or calls this module.  Only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg use it, and only as
the checker / the timed CPU baseline.

What it is
----------
A NumPy restatement (float64 by default, float32 on request) of the reference's
Torch7 hot path, module by module, following the Lua sources in
Ajay-Wong/seq2seq-attention-asr.  Every function cites the reference file:line
it restates.  The arithmetic of the un-vendored Torch7 packages (`nn`, `nngraph`)
that those Lua files call is restated from their published semantics (marked 3p):
`nn.Linear` y = W x + b, W (out, in); `nn.TemporalConvolution` W (out, in*kW);
`nn.SoftMax` / `nn.LogSoftMax` max-subtracted; `nn.Sigmoid` / `nn.Tanh` backward
from their outputs; `nn.TemporalMaxPooling` first maximum wins; `nn.Dropout`
(v2) inverted scaling.  No Torch7 version is pinned by the reference.

Parity status
-------------
The reference (Lua/Torch7) cannot run in this container or on the GPU box (no
`th`/`luajit`/Torch7).  The restatement is pinned by
  * the reference notebooks' known answers (TemporalConvolution iota layout
    -> rows of [15, 40, 65, 90]; hybrid-attention padding shapes; the
    "-sum(labelmask*logprobs) == ClassNLL" loss identity), see
    tests/test_oracle.py;
  * the batched-vs-per-utterance identity the notebooks exercise
    (Attention.ipynb cells 43-44);
  * an independent PyTorch-CPU autograd formulation of the same forward pass
    and central finite differences in float64 (tests/test_oracle.py).
It is NOT pinned against outputs of Torch7 itself: "parity unpinned against
Torch7" in the sense of the task statement.

Batch semantics
---------------
The reference forwards one utterance at a time as a 2-D (L x F) tensor and
accumulates gradients over `opt.batchSize` utterances, then divides by B
(timit/timit.lua:240-295).  Here every function takes a leading batch axis B;
each batch row is computed exactly as the reference computes one utterance
(rows never interact), so B=1 is the reference's own call and B>1 equals the
per-utterance loop.
"""
from __future__ import annotations

import dataclasses
from typing import Dict, Optional

import numpy as np

Array = np.ndarray


# ----------------------------------------------------------------------------
# (3p) nn pointwise semantics
# ----------------------------------------------------------------------------

def sigmoid(x: Array) -> Array:
    """nn.Sigmoid (3p): 1 / (1 + exp(-x))."""
    return 1.0 / (1.0 + np.exp(-x))


def softmax(x: Array, axis: int = -1) -> Array:
    """nn.SoftMax (3p): exp(x - max) / sum(exp(x - max))."""
    m = np.max(x, axis=axis, keepdims=True)
    e = np.exp(x - m)
    return e / np.sum(e, axis=axis, keepdims=True)


def log_softmax(x: Array, axis: int = -1) -> Array:
    """nn.LogSoftMax (3p): x - max - log(sum(exp(x - max)))."""
    m = np.max(x, axis=axis, keepdims=True)
    return x - m - np.log(np.sum(np.exp(x - m), axis=axis, keepdims=True))


# ----------------------------------------------------------------------------
# LinearZeroBias / TemporalConvolutionZeroBias
# ----------------------------------------------------------------------------

def linear_zero_bias_fwd(W: Array, x: Array) -> Array:
    """LinearZeroBias.lua:31-48: y = W x (addmv for 1-D, addmm x W^T for 2-D)."""
    return x @ W.T


def linear_zero_bias_bwd(W: Array, x: Array, dy: Array, dW: Array, scale: float = 1.0) -> Array:
    """LinearZeroBias.lua:50-74: dx = W^T dy; dW += scale * dy (x) x."""
    dW += scale * (dy.reshape(-1, dy.shape[-1]).T @ x.reshape(-1, x.shape[-1]))
    return dy @ W


def temporal_conv(W: Array, b: Optional[Array], x: Array, kW: int) -> Array:
    """nn.TemporalConvolution (3p) with dW=1, no padding, as called by
    TemporalConvolutionZeroBias.lua:37-40 and Attention.lua:66,90.

    x (..., L_in, inFrame) -> y (..., L_in - kW + 1, outFrame); W is (out, in*kW) with
    the window laid out frame-major (pinned by Attention.ipynb cells 4-6: weights
    1..20 row-major on ones(10,5) give rows of [15, 40, 65, 90])."""
    L_in, fin = x.shape[-2], x.shape[-1]
    L_out = L_in - kW + 1
    cols = np.stack([x[..., j:j + L_out, :] for j in range(kW)], axis=-2)  # (..., L_out, kW, fin)
    cols = cols.reshape(cols.shape[:-2] + (kW * fin,))
    y = cols @ W.T
    if b is not None:
        y = y + b
    return y


# ----------------------------------------------------------------------------
# GRU cell + nn.RNN unroll
# ----------------------------------------------------------------------------

def gru_seq_fwd(x: Array, Wz: Array, Wr: Array, Wh: Array, reverse: bool = False,
                h0: Optional[Array] = None):
    """nn.RNN(nn.GRU(D, H), reverse) forward.

    GRU.lua:16-38 (cell): hx = [h; x] (h FIRST, :22); z = sig(Wz hx) (:23);
    r = sig(Wr hx) (:24); hh = tanh(Wh [r*h; x]) (:25-26); h' = (1-z)*h + z*hh (:27-30).
    No biases (LinearZeroBias).  Recurrent.lua:104-127 supplies zeros for the first
    prev_h; RNN.lua:120-167 runs t = 1..L, or L..1 when reverse (:142-145), passing
    y_{t-1} as prev_h.

    x (B, L, D); W* (H, H+D).  Returns y (B, L, H) and the saved activations."""
    B, L, D = x.shape
    H = Wz.shape[0]
    h = np.zeros((B, H), x.dtype) if h0 is None else h0
    y = np.zeros((B, L, H), x.dtype)
    sv = {k: np.zeros((B, L, H), x.dtype) for k in ("z", "r", "hh", "hprev")}
    order = range(L - 1, -1, -1) if reverse else range(L)
    for t in order:
        xt = x[:, t]
        hx = np.concatenate([h, xt], axis=1)
        z = sigmoid(hx @ Wz.T)
        r = sigmoid(hx @ Wr.T)
        rhx = np.concatenate([r * h, xt], axis=1)
        hh = np.tanh(rhx @ Wh.T)
        sv["z"][:, t], sv["r"][:, t], sv["hh"][:, t], sv["hprev"][:, t] = z, r, hh, h
        h = (1.0 - z) * h + z * hh
        y[:, t] = h
    return y, sv


def gru_seq_bwd(x: Array, Wz: Array, Wr: Array, Wh: Array, sv: Dict[str, Array], dy: Array,
                grads: Dict[str, Array], reverse: bool = False, scale: float = 1.0):
    """nn.RNN:updateGradInput (RNN.lua:169-201) over nn.GRU / nn.Recurrent
    (GRU.lua:45-51 uses only gradOutput[1]; Recurrent.lua:129-151).

    BPTT: dEdy_t += dEdpy from step t+1 (RNN.lua:194); gradInput[t] = dx_t (:196).
    Weight grads accumulate into grads['Wz'|'Wr'|'Wh'] (LinearZeroBias.lua:67-74).
    Returns dx (B, L, D) and dh0 (grad w.r.t. the zero initial state)."""
    B, L, D = x.shape
    H = Wz.shape[0]
    dx = np.zeros_like(x)
    dnext = np.zeros((B, H), x.dtype)
    order = range(L) if reverse else range(L - 1, -1, -1)
    for t in order:
        z, r, hh, hp = sv["z"][:, t], sv["r"][:, t], sv["hh"][:, t], sv["hprev"][:, t]
        xt = x[:, t]
        dh = dy[:, t] + dnext
        dz = dh * (hh - hp)
        dhh = dh * z
        dhp = dh * (1.0 - z)
        dah = dhh * (1.0 - hh * hh)
        rhx = np.concatenate([r * hp, xt], axis=1)
        grads["Wh"] += scale * (dah.T @ rhx)
        drhx = dah @ Wh
        drh = drhx[:, :H]
        dxt = drhx[:, H:].copy()
        dr = drh * hp
        dhp += drh * r
        daz = dz * z * (1.0 - z)
        dar = dr * r * (1.0 - r)
        hx = np.concatenate([hp, xt], axis=1)
        grads["Wz"] += scale * (daz.T @ hx)
        grads["Wr"] += scale * (dar.T @ hx)
        dhx = daz @ Wz + dar @ Wr
        dhp += dhx[:, :H]
        dxt += dhx[:, H:]
        dx[:, t] = dxt
        dnext = dhp
    return dx, dnext


# ----------------------------------------------------------------------------
# LSTM cell + nn.RNN unroll (BiLSTM variant)
# ----------------------------------------------------------------------------

LSTM_GATES = ("i", "f", "g", "o")


def lstm_seq_fwd(x: Array, P: Dict[str, Array], reverse: bool = False, peepholes: bool = False):
    """nn.RNN(nn.LSTM(D, H, peepholes), reverse) forward.

    LSTM.lua:16-58: each gate is Linear(D,H)(x) + Linear(H,H)(prev_h) [+ Linear(H,H)(c)
    peephole] with biases (:25-36); in_gate, forget_gate = sig (:42-43, peek prev_c);
    in2cell = tanh (:44, never peeks); next_c = f*c + i*g (:45-46); out_gate = sig
    peeking next_c (:47-50); next_h = o * tanh(next_c) (:51).  nn.RNN passes
    {x, y_{t-1}, h_{t-1}} so prev_h = y_{t-1} and prev_c = the carried cell
    (RNN.lua:155-163, LSTM.lua:100-116).

    P keys: W{g}x (H,D), b{g}x (H), W{g}h (H,H), b{g}h (H), and W{g}c, b{g}c (H,H)/(H)
    for g in i,f,o when peepholes."""
    B, L, D = x.shape
    H = P["Wix"].shape[0]
    h = np.zeros((B, H), x.dtype)
    c = np.zeros((B, H), x.dtype)
    y = np.zeros((B, L, H), x.dtype)
    sv = {k: np.zeros((B, L, H), x.dtype) for k in ("i", "f", "g", "o", "c", "cprev", "hprev", "tc")}
    order = range(L - 1, -1, -1) if reverse else range(L)
    for t in order:
        xt = x[:, t]

        def pre(gname, peek):
            a = xt @ P[f"W{gname}x"].T + P[f"b{gname}x"] + h @ P[f"W{gname}h"].T + P[f"b{gname}h"]
            if peepholes and peek is not None:
                a = a + peek @ P[f"W{gname}c"].T + P[f"b{gname}c"]
            return a

        i = sigmoid(pre("i", c))
        f = sigmoid(pre("f", c))
        g = np.tanh(pre("g", None))
        cn = f * c + i * g
        o = sigmoid(pre("o", cn))
        tc = np.tanh(cn)
        hn = o * tc
        for k, v in (("i", i), ("f", f), ("g", g), ("o", o), ("c", cn), ("cprev", c), ("hprev", h), ("tc", tc)):
            sv[k][:, t] = v
        h, c = hn, cn
        y[:, t] = h
    return y, sv


def lstm_seq_bwd(x: Array, P: Dict[str, Array], sv: Dict[str, Array], dy: Array,
                 grads: Dict[str, Array], reverse: bool = False, peepholes: bool = False,
                 scale: float = 1.0):
    """LSTM:updateGradInput (LSTM.lua:118-136) under nn.RNN's BPTT (RNN.lua:169-201):
    dEdh = dy_t + d prev_h from t+1, dEdc = d prev_c from t+1."""
    B, L, D = x.shape
    H = P["Wix"].shape[0]
    dx = np.zeros_like(x)
    dh_next = np.zeros((B, H), x.dtype)
    dc_next = np.zeros((B, H), x.dtype)
    order = range(L) if reverse else range(L - 1, -1, -1)
    for t in order:
        i, f, g, o = sv["i"][:, t], sv["f"][:, t], sv["g"][:, t], sv["o"][:, t]
        cn, cp, hp, tc = sv["c"][:, t], sv["cprev"][:, t], sv["hprev"][:, t], sv["tc"][:, t]
        xt = x[:, t]
        dh = dy[:, t] + dh_next
        do = dh * tc
        dcn = dc_next + dh * o * (1.0 - tc * tc)
        dao = do * o * (1.0 - o)
        dxt = np.zeros_like(xt)
        dhp = np.zeros_like(hp)
        dcp = np.zeros_like(cp)

        def acc(gname, da, peek_val):
            nonlocal dxt, dhp
            grads[f"W{gname}x"] += scale * (da.T @ xt)
            grads[f"b{gname}x"] += scale * da.sum(0)
            grads[f"W{gname}h"] += scale * (da.T @ hp)
            grads[f"b{gname}h"] += scale * da.sum(0)
            dxt = dxt + da @ P[f"W{gname}x"]
            dhp = dhp + da @ P[f"W{gname}h"]
            if peepholes and peek_val is not None:
                grads[f"W{gname}c"] += scale * (da.T @ peek_val)
                grads[f"b{gname}c"] += scale * da.sum(0)
                return da @ P[f"W{gname}c"]
            return None

        dpeek = acc("o", dao, cn)
        if dpeek is not None:
            dcn = dcn + dpeek
        di = dcn * g
        df = dcn * cp
        dg = dcn * i
        dcp = dcp + dcn * f
        dai = di * i * (1.0 - i)
        daf = df * f * (1.0 - f)
        dag = dg * (1.0 - g * g)
        for gname, da in (("i", dai), ("f", daf)):
            dpk = acc(gname, da, cp)
            if dpk is not None:
                dcp = dcp + dpk
        acc("g", dag, None)
        dx[:, t] = dxt
        dh_next, dc_next = dhp, dcp
    return dx


# ----------------------------------------------------------------------------
# Bidirectional encoder (timit/model_chorowski_baseline.lua:20-34)
# ----------------------------------------------------------------------------

def encoder_fwd(x: Array, P: Dict[str, Array], nlayers: int = 3):
    """3 x [fwd GRU || bwd GRU] joined on features, fwd first (JoinTable(2,2),
    model_chorowski_baseline.lua:24,28,32)."""
    caches = []
    inp = x
    for l in range(1, nlayers + 1):
        yf, svf = gru_seq_fwd(inp, P[f"enc{l}f.Wz"], P[f"enc{l}f.Wr"], P[f"enc{l}f.Wh"], False)
        yb, svb = gru_seq_fwd(inp, P[f"enc{l}b.Wz"], P[f"enc{l}b.Wr"], P[f"enc{l}b.Wh"], True)
        caches.append((inp, svf, svb))
        inp = np.concatenate([yf, yb], axis=2)
    return inp, caches


def encoder_bwd(P: Dict[str, Array], caches, dout: Array, G: Dict[str, Array], scale: float = 1.0):
    d = dout
    for l in range(len(caches), 0, -1):
        inp, svf, svb = caches[l - 1]
        H = P[f"enc{l}f.Wz"].shape[0]
        gf = {k: G[f"enc{l}f.{k}"] for k in ("Wz", "Wr", "Wh")}
        gb = {k: G[f"enc{l}b.{k}"] for k in ("Wz", "Wr", "Wh")}
        dxf, _ = gru_seq_bwd(inp, P[f"enc{l}f.Wz"], P[f"enc{l}f.Wr"], P[f"enc{l}f.Wh"], svf, d[:, :, :H], gf, False, scale)
        dxb, _ = gru_seq_bwd(inp, P[f"enc{l}b.Wz"], P[f"enc{l}b.Wr"], P[f"enc{l}b.Wh"], svb, d[:, :, H:], gb, True, scale)
        d = dxf + dxb
    return d


# ----------------------------------------------------------------------------
# Attention decoder (Attention.lua + RNNAttention.lua + MonotonicAlignment.lua)
# ----------------------------------------------------------------------------

def hybrid_pads(kW: int):
    """Attention.lua:77-86: odd kW pads (kW-1)/2 on both sides; even kW pads kW/2 on the left
    (nn.Padding(1, -pad_left, 2)) and kW/2 - 1 on the right, so the conv returns L frames."""
    if kW % 2 == 1:
        return (kW - 1) // 2, (kW - 1) // 2
    return kW // 2, kW // 2 - 1


def hybrid_features(alpha_prev: Array, P: Dict[str, Array], kW: int):
    """Location features of the hybrid attention (Attention.lua:75-97): alpha_{t-1} (B, L) as an
    (L, 1) sequence, zero-padded (hybrid_pads), -> F = TemporalConvolution(1, nF, kW) with bias
    (:90) -> UF = TCZB(nF, Sc, 1) (:91, zero bias).  Returns (UF (B, L, Sc), F (B, L, nF), the
    padded sequence (B, L + kW - 1))."""
    pl, pr = hybrid_pads(kW)
    B, L = alpha_prev.shape
    apad = np.concatenate([np.zeros((B, pl), alpha_prev.dtype), alpha_prev, np.zeros((B, pr), alpha_prev.dtype)], 1)
    Fm = temporal_conv(P["hybW"], P["hybb"], apad[..., None], kW)   # (B, L, nF)
    UF = temporal_conv(P["hybU"], None, Fm, 1)                       # (B, L, Sc)
    return UF, Fm, apad


def attention_fwd(h: Array, labels: Array, P: Dict[str, Array], cfg: "ModelConfig",
                  dropout_mask: Optional[Array] = None, maxout_idx: Optional[Array] = None):
    """nn.Attention:updateOutput (Attention.lua:305-322) = decoder gModule
    {h, labelmask} -> RNNAttention over T steps (RNNAttention.lua:144-185).

    h (B, L, A) annotations; labels (B, T) int in [0, O) (0-based; the reference is
    1-based).  Teacher forcing: prev_y = zeros at t=1, else onehot(labels[t-1])
    (RNNAttention.lua:172-176).  Hidden carried = {alpha, s, mem}, zeros at t=1
    (Recurrent.lua:79-112 with dimhidden {L, S, S}, Attention.lua:318).

    Per step (decoder_base_, Attention.lua:51-184):
      ws = Ws s + bs            TemporalConvolution(1,Sc,S) on View(S,1) (:65-66)
      Z = expand_L(ws) + Vh [+ UF] ExpandAs + CAddTable (:67,95-98); UF = hybrid_features(alpha_prev)
                                 when cfg.hybridAttendFeatureMaps > 0 (:75-94)
      e = we . tanh(Z)           TCZB(Sc,1,1) (:104-110)
      alpha = softmax_L(e)       (:117)
      alpha = MonoAlign(alpha, alpha_prev) identity fwd (:122-125, MonotonicAlignment.lua:19-42)
      c = alpha^T h              Replicate + MM + View (:132-134)
      y_in = Wy y + by; c_in = Wc c + bc; d = Wd [c_in; y_in] + bd   (:149-151)
      s = GRU(d, s_prev)         decoder_recurrent (model_chorowski_baseline.lua:48-51)
      logp = LogSoftMax(Wo Maxout([s; c]) + bo)   decoder_mlp (:53-59, Maxout.lua:14-18)
    Vh = h V^T once per utterance (TCZB(A, Sc, 1), Attention.lua:43-47,202).
    maxout_idx (B, T, M) ints (optional): take these Maxout winners instead of the argmax -- to compare an
    implementation under ITS OWN discrete decisions (a reduced-precision run flips near ties)."""
    B, L, A = h.shape
    T = labels.shape[1]
    S, Sc, O, M, k = cfg.stateDepth, cfg.scoreDepth, cfg.outputDepth, cfg.mlpDepth, cfg.maxoutWindow
    dt = h.dtype
    Vh = temporal_conv(P["V"], None, h, 1)                      # (B, L, Sc)
    s = np.zeros((B, S), dt)
    alpha_prev = np.zeros((B, L), dt)
    keys = ["ws", "alpha", "c", "cin", "yin", "d", "sprev", "mono_ind", "u", "argmax", "m", "logp", "v",
            "alpha_prev"]
    keys += ["li", "lf", "lg", "lo", "mprev", "mnew"] if cfg.decoderLSTM else ["z", "r", "hh"]
    cache = {key: [] for key in keys}
    mem = np.zeros((B, S), dt)  # the LSTM decoder's carried cell (mem, Attention.lua:152)
    logp_all = np.zeros((B, T, O), dt)
    Wg = {g: P[f"dec.W{g}"] for g in ("z", "r", "h")} if not cfg.decoderLSTM else {}
    hyb = cfg.hybridAttendFeatureMaps > 0
    for t in range(T):
        yprev = np.zeros((B, O), dt)
        if t > 0:
            yprev[np.arange(B), labels[:, t - 1]] = 1.0
        ws = s @ P["Ws"].T + P["bs"]                               # (B, Sc)
        Z = ws[:, None, :] + Vh
        if hyb:
            Z = Z + hybrid_features(alpha_prev, P, cfg.hybridAttendFilterSize)[0]
        th = np.tanh(Z)
        e = (th @ P["we"].T)[..., 0]                               # (B, L)
        alpha = softmax(e, axis=1)
        # MonotonicAlignment.lua:27-39: penalty = lambda * max(sum_j(cumsum a - cumsum a_prev), 0)
        diff = np.sum(np.cumsum(alpha, 1) - np.cumsum(alpha_prev, 1), axis=1)
        pen = cfg.penalty * np.maximum(diff, 0.0)
        ind = (pen > 0).astype(dt)
        c = np.einsum("bl,bla->ba", alpha, h)
        yin = yprev @ P["Wy"].T + P["by"]
        cin = c @ P["Wc"].T + P["bc"]
        d = np.concatenate([cin, yin], 1) @ P["Wd"].T + P["bd"]
        if cfg.decoderLSTM:
            # LSTM.lua:16-51 with x = d, prev_h = s, prev_c = mem: each gate Linear(x) + Linear(h), biases
            pre = {q: d @ P[f"dec.W{q}x"].T + P[f"dec.b{q}x"] + s @ P[f"dec.W{q}h"].T + P[f"dec.b{q}h"]
                   for q in "ifgo"}
            li, lf, lo = sigmoid(pre["i"]), sigmoid(pre["f"]), sigmoid(pre["o"])
            lg = np.tanh(pre["g"])
            mnew = lf * mem + li * lg
            s_new = lo * np.tanh(mnew)
            for key, val in (("li", li), ("lf", lf), ("lg", lg), ("lo", lo), ("mprev", mem), ("mnew", mnew)):
                cache[key].append(val)
            mem = mnew
        else:
            hx = np.concatenate([s, d], 1)
            z = sigmoid(hx @ Wg["z"].T)
            r = sigmoid(hx @ Wg["r"].T)
            hh = np.tanh(np.concatenate([r * s, d], 1) @ Wg["h"].T)
            s_new = (1.0 - z) * s + z * hh
            for key, val in (("z", z), ("r", r), ("hh", hh)):
                cache[key].append(val)
        v = np.concatenate([s_new, c], 1)
        if dropout_mask is not None:
            v = v * dropout_mask[:, t]
        u = v @ P["Wm"].T + P["bm"]
        ug = u.reshape(B, M, k)
        am = np.argmax(ug, axis=2) if maxout_idx is None else np.asarray(maxout_idx[:, t], np.int64)  # first max wins
        m = np.take_along_axis(ug, am[..., None], 2)[..., 0]
        o = m @ P["Wo"].T + P["bo"]
        logp = log_softmax(o, 1)
        logp_all[:, t] = logp
        for key, val in (("ws", ws), ("alpha", alpha), ("c", c), ("cin", cin), ("yin", yin), ("d", d),
                         ("sprev", s), ("mono_ind", ind), ("u", u),
                         ("argmax", am), ("m", m), ("logp", logp), ("v", v), ("alpha_prev", alpha_prev)):
            cache[key].append(val)
        s = s_new
        alpha_prev = alpha
    cache = {key: np.stack(vals, 1) for key, vals in cache.items()}
    cache["Vh"] = Vh
    cache["h"] = h
    cache["labels"] = labels
    return logp_all, cache


def _gru_dec_bwd(P, G, Wg, g_, ds, sp, d, S, scale):
    """decoder GRU backward (GRU.lua:16-38), x = d, h = s_prev: returns (dd, dL/ds_prev from the cell)."""
    z, r, hh = g_("z"), g_("r"), g_("hh")
    dz = ds * (hh - sp)
    dah = ds * z * (1 - hh * hh)
    dsp = ds * (1 - z)
    rhx = np.concatenate([r * sp, d], 1)
    G["dec.Wh"] += scale * (dah.T @ rhx)
    drhx = dah @ Wg["h"]
    dd = drhx[:, S:].copy()
    dr = drhx[:, :S] * sp
    dsp += drhx[:, :S] * r
    daz = dz * z * (1 - z)
    dar = dr * r * (1 - r)
    hx = np.concatenate([sp, d], 1)
    G["dec.Wz"] += scale * (daz.T @ hx)
    G["dec.Wr"] += scale * (dar.T @ hx)
    dhx = daz @ Wg["z"] + dar @ Wg["r"]
    dsp += dhx[:, :S]
    dd += dhx[:, S:]
    return dd, dsp


def attention_bwd(P: Dict[str, Array], cfg: "ModelConfig", cache, dlogp: Array, G: Dict[str, Array],
                  scale: float = 1.0, dropout_mask: Optional[Array] = None, dmlp_in: Optional[Array] = None):
    """nn.Attention:updateGradInput (Attention.lua:324-327): RNNAttention's reverse BPTT
    (RNNAttention.lua:203-253) accumulating d{Vh, h} over all t (:247); dy discarded
    (:248).  MonotonicAlignment.lua:44-77 adds lambda*(L+1-j)*ind to d alpha and its
    negation to d alpha_prev.  Returns dh (B, L, A)."""
    h, Vh, labels = cache["h"], cache["Vh"], cache["labels"]
    B, L, A = h.shape
    T = (dlogp if dmlp_in is None else dmlp_in).shape[1]
    S, Sc, O, M, k = cfg.stateDepth, cfg.scoreDepth, cfg.outputDepth, cfg.mlpDepth, cfg.maxoutWindow
    dt = h.dtype
    dh = np.zeros_like(h)
    dVh = np.zeros_like(Vh)
    ds_carry = np.zeros((B, S), dt)
    dmem_carry = np.zeros((B, S), dt)
    dalpha_carry = np.zeros((B, L), dt)
    jw = (L + 1 - np.arange(1, L + 1)).astype(dt)               # (L+1-j), j 1-based
    Wg = {g: P[f"dec.W{g}"] for g in ("z", "r", "h")} if not cfg.decoderLSTM else {}
    hyb = cfg.hybridAttendFeatureMaps > 0
    kW = cfg.hybridAttendFilterSize
    for t in range(T - 1, -1, -1):
        g_ = lambda key: cache[key][:, t]
        if dmlp_in is not None:  # an external decoder_mlp's gradient w.r.t. its input [s_t; c_t]
            dv = dmlp_in[:, t].copy()
        else:
            logp = g_("logp")
            # LogSoftMax backward (3p): do = dlogp - exp(logp) * sum(dlogp)
            dl = dlogp[:, t]
            do = dl - np.exp(logp) * dl.sum(1, keepdims=True)
            G["Wo"] += scale * (do.T @ g_("m"))
            G["bo"] += scale * do.sum(0)
            dm = do @ P["Wo"]
            du = np.zeros((B, M * k), dt)
            idx = np.arange(M) * k + g_("argmax")
            np.put_along_axis(du, idx, dm, axis=1)
            v = g_("v")
            G["Wm"] += scale * (du.T @ v)
            G["bm"] += scale * du.sum(0)
            dv = du @ P["Wm"]
        if dropout_mask is not None:
            dv = dv * dropout_mask[:, t]
        ds = dv[:, :S] + ds_carry
        dc = dv[:, S:].copy()
        sp, d = g_("sprev"), g_("d")
        if cfg.decoderLSTM:
            # LSTM backward (LSTM.lua:118-136): ds = dL/dh_t, dmem_carry = dL/dc_t from step t+1
            li, lf, lg, lo, mp, mn = (g_(key) for key in ("li", "lf", "lg", "lo", "mprev", "mnew"))
            tc = np.tanh(mn)
            dcell = dmem_carry + ds * lo * (1 - tc * tc)
            dpre = {"i": dcell * lg * li * (1 - li), "f": dcell * mp * lf * (1 - lf),
                    "g": dcell * li * (1 - lg * lg), "o": ds * tc * lo * (1 - lo)}
            dmem_carry = dcell * lf
            dd = np.zeros_like(d)
            dsp = np.zeros_like(sp)
            for q, da in dpre.items():
                G[f"dec.W{q}x"] += scale * (da.T @ d)
                G[f"dec.b{q}x"] += scale * da.sum(0)
                G[f"dec.W{q}h"] += scale * (da.T @ sp)
                G[f"dec.b{q}h"] += scale * da.sum(0)
                dd += da @ P[f"dec.W{q}x"]
                dsp += da @ P[f"dec.W{q}h"]
        else:
            dd, dsp = _gru_dec_bwd(P, G, Wg, g_, ds, sp, d, S, scale)
        # d = Wd [c_in; y_in] + bd
        cin, yin = g_("cin"), g_("yin")
        G["Wd"] += scale * (dd.T @ np.concatenate([cin, yin], 1))
        G["bd"] += scale * dd.sum(0)
        dcy = dd @ P["Wd"]
        dcin, dyin = dcy[:, :S], dcy[:, S:]
        c = g_("c")
        G["Wc"] += scale * (dcin.T @ c)
        G["bc"] += scale * dcin.sum(0)
        dc += dcin @ P["Wc"]
        yprev = np.zeros((B, O), dt)
        if t > 0:
            yprev[np.arange(B), labels[:, t - 1]] = 1.0
        G["Wy"] += scale * (dyin.T @ yprev)
        G["by"] += scale * dyin.sum(0)
        # c = alpha^T h
        alpha = g_("alpha")
        dalpha = np.einsum("ba,bla->bl", dc, h) + dalpha_carry
        dh += alpha[:, :, None] * dc[:, None, :]
        # MonotonicAlignment backward
        gdiff = cfg.penalty * jw[None, :] * g_("mono_ind")[:, None]
        dalpha = dalpha + gdiff
        dalpha_carry = -gdiff
        # softmax backward (3p)
        de = alpha * (dalpha - np.sum(alpha * dalpha, 1, keepdims=True))
        ws = g_("ws")
        Z = ws[:, None, :] + Vh
        if hyb:
            UF, Fm, apad = hybrid_features(g_("alpha_prev"), P, kW)
            Z = Z + UF
        th = np.tanh(Z)
        G["we"] += scale * np.einsum("bl,blk->k", de, th)[None, :]
        dZ = de[:, :, None] * P["we"][0][None, None, :] * (1 - th * th)
        dVh += dZ
        if hyb:
            # UF = TCZB(F -> Sc) of F = conv(alpha_{t-1}): grads of U, the conv, and d alpha_{t-1}
            # (alpha is part of the carried hidden state, RNNAttention.lua:233-250)
            G["hybU"] += scale * np.einsum("bls,blf->sf", dZ, Fm)
            dF = dZ @ P["hybU"]                                      # (B, L, nF)
            G["hybb"] += scale * dF.sum((0, 1))
            win = np.stack([apad[:, i:i + L] for i in range(kW)], 2)  # (B, L, kW)
            G["hybW"] += scale * np.einsum("blf,bli->fi", dF, win)
            dq = dF @ P["hybW"]                                      # (B, L, kW): d apad[l + i]
            dapad = np.zeros_like(apad)
            for i in range(kW):
                dapad[:, i:i + L] += dq[:, :, i]
            pl, _ = hybrid_pads(kW)
            dalpha_carry = dalpha_carry + dapad[:, pl:pl + L]
        dws = dZ.sum(1)
        G["Ws"] += scale * (dws.T @ sp)
        G["bs"] += scale * dws.sum(0)
        ds_carry = dsp + dws @ P["Ws"]
    # Vh = h V^T  (TCZB k=1)
    G["V"] += scale * np.einsum("bls,bla->sa", dVh, h)
    dh += dVh @ P["V"]
    return dh


# ----------------------------------------------------------------------------
# Model config, init, full training step (timit/timit.lua:240-295)
# ----------------------------------------------------------------------------

@dataclasses.dataclass
class ModelConfig:
    """Mirrors loadmodel(opt) field names (timit/model_chorowski_baseline.lua:14-46)."""
    inputFrameSize: int = 123
    hiddenFrameSize: int = 256
    outputFrameSize: int = 256
    scoreDepth: int = 512
    stateDepth: int = 256
    outputDepth: int = 62          # opt.numPhonemes (TIMIT) / opt.outputDepth (LibriSpeech)
    mlpDepth: int = 64
    maxoutWindow: int = 7          # Maxout(..., 7) (model_chorowski_baseline.lua:56)
    penalty: float = 0.0           # MonotonicAlignment lambda
    numLayers: int = 3
    hybridAttendFilterSize: int = 0    # Attention(..., hybridAttendFilterSize, hybridAttendFeatureMaps, ...):
    hybridAttendFeatureMaps: int = 0   # 0 maps = content-only attention (model_chorowski_baseline.lua:39-40)
    decoderLSTM: bool = False      # decoder_recurrent = nn.LSTM(S, S) (timit/timit.lua:137) instead of GRU(S, S)

    @property
    def annotationDepth(self) -> int:
        return 2 * self.outputFrameSize


def param_shapes(cfg: ModelConfig):
    """Canonical parameter list, in flat-buffer order (see DESIGN.md §Data layout)."""
    shapes = []
    D = cfg.inputFrameSize
    for l in range(1, cfg.numLayers + 1):
        H = cfg.outputFrameSize if l == cfg.numLayers else cfg.hiddenFrameSize
        for dname in ("f", "b"):
            for g in ("Wz", "Wr", "Wh"):
                shapes.append((f"enc{l}{dname}.{g}", (H, H + D)))
        D = 2 * H
    A, Sc, S, O, M, k = cfg.annotationDepth, cfg.scoreDepth, cfg.stateDepth, cfg.outputDepth, cfg.mlpDepth, cfg.maxoutWindow
    shapes += [("V", (Sc, A)), ("Ws", (Sc, S)), ("bs", (Sc,)), ("we", (1, Sc)),
               ("Wy", (S, O)), ("by", (S,)), ("Wc", (S, A)), ("bc", (S,)),
               ("Wd", (S, 2 * S)), ("bd", (S,)),
               ("dec.Wz", (S, 2 * S)), ("dec.Wr", (S, 2 * S)), ("dec.Wh", (S, 2 * S)),
               ("Wm", (M * k, S + A)), ("bm", (M * k,)), ("Wo", (O, M)), ("bo", (O,))]
    if cfg.hybridAttendFeatureMaps > 0:  # Attention.lua:90-91: conv (nF, kW) + bias, UF TCZB (Sc, nF)
        nF, kW = cfg.hybridAttendFeatureMaps, cfg.hybridAttendFilterSize
        shapes += [("hybW", (nF, kW)), ("hybb", (nF,)), ("hybU", (Sc, nF))]
    return shapes


def fan_in(name: str, shape, cfg: ModelConfig) -> int:
    """Default reset() stdv = 1/sqrt(fan_in): LinearZeroBias.lua:12-29 (in),
    TemporalConvolutionZeroBias.lua:21-35 (kW*inFrame), nn.Linear / nn.TemporalConvolution (3p)."""
    S, Sc, A, O, M, k = cfg.stateDepth, cfg.scoreDepth, cfg.annotationDepth, cfg.outputDepth, cfg.mlpDepth, cfg.maxoutWindow
    table = {"V": A, "Ws": S, "bs": S, "we": Sc, "Wy": O, "by": O, "Wc": A, "bc": A, "Wd": 2 * S, "bd": 2 * S,
             "Wm": S + A, "bm": S + A, "Wo": M, "bo": M, "hybW": cfg.hybridAttendFilterSize,
             "hybb": cfg.hybridAttendFilterSize, "hybU": cfg.hybridAttendFeatureMaps}
    if name in table:
        return table[name]
    return shape[1]


def init_params(cfg: ModelConfig, seed: int = 1234, dtype=np.float64) -> Dict[str, Array]:
    rng = np.random.default_rng(seed)
    P = {}
    for name, shape in param_shapes(cfg):
        stdv = 1.0 / np.sqrt(fan_in(name, shape, cfg))
        P[name] = rng.uniform(-stdv, stdv, size=shape).astype(dtype)
    return P


def zeros_like_params(P: Dict[str, Array]) -> Dict[str, Array]:
    return {k: np.zeros_like(v) for k, v in P.items()}


def flatten(P: Dict[str, Array], cfg: ModelConfig) -> Array:
    return np.concatenate([P[n].reshape(-1) for n, _ in param_shapes(cfg)])


def unflatten(flat: Array, cfg: ModelConfig) -> Dict[str, Array]:
    out, off = {}, 0
    for n, shp in param_shapes(cfg):
        sz = int(np.prod(shp))
        out[n] = flat[off:off + sz].reshape(shp)
        off += sz
    assert off == flat.size
    return out


def training_step(x: Array, labels: Array, P: Dict[str, Array], cfg: ModelConfig,
                  normalizeNLL: bool = True, dropout_mask: Optional[Array] = None,
                  maxout_idx: Optional[Array] = None):
    """timit/timit.lua:240-295 for one optimizer step's gradient, B utterances of
    equal length: per utterance logp = fwd({X, onehot(Y)}) (:262-265);
    nll_b = -sum(onehot * logp) [/T] (:268-272, reporting only); dlogp = -onehot (:278);
    backward accumulates; then nll /= B and grad /= B when B > 1 (:292-295).
    Returns (nll, grads dict, logp, enc_out)."""
    B, L, F = x.shape
    T = labels.shape[1]
    O = cfg.outputDepth
    enc, ecache = encoder_fwd(x, P, cfg.numLayers)
    logp, acache = attention_fwd(enc, labels, P, cfg, dropout_mask, maxout_idx)
    onehot = np.zeros((B, T, O), x.dtype)
    np.put_along_axis(onehot, labels[..., None], 1.0, axis=2)
    nll_b = -(onehot * logp).sum((1, 2))
    if normalizeNLL:
        nll_b = nll_b / T
    scale = 1.0 / B if B > 1 else 1.0
    G = zeros_like_params(P)
    denc = attention_bwd(P, cfg, acache, -onehot, G, scale, dropout_mask)
    encoder_bwd(P, ecache, denc, G, scale)
    return float(nll_b.mean()), G, logp, enc


def training_step_ragged(x: Array, labels: Array, flen, tlen, P: Dict[str, Array], cfg: ModelConfig,
                         normalizeNLL: bool = True):
    """timit/timit.lua:239-295 literally: a minibatch of variable-length utterances is forwarded and
    back-propagated ONE UTTERANCE AT A TIME at its own length ("data is variable length", :239-240),
    gradients summed, then / B (:292-295).  x (B, Lmax, F) and labels (B, Tmax) are padded; utterance b
    is x[b, :flen[b]], labels[b, :tlen[b]].  Returns (nll per utterance (B,), grads dict,
    [logp_b (T_b, O)], [enc_b (L_b, A)])."""
    B = x.shape[0]
    G = zeros_like_params(P)
    nlls, logps, encs = [], [], []
    for b in range(B):
        Lb, Tb = int(flen[b]), int(tlen[b])
        nll_b, G_b, logp_b, enc_b = training_step(x[b:b + 1, :Lb], labels[b:b + 1, :Tb], P, cfg, normalizeNLL)
        for k in G:
            G[k] += G_b[k]
        nlls.append(nll_b)
        logps.append(logp_b[0])
        encs.append(enc_b[0])
    if B > 1:
        for k in G:
            G[k] /= B
    return np.array(nlls), G, logps, encs


def timit_like_lengths(n: int, seed: int = 0, frames_per_s: float = 16000 / 512, pad: int = 20,
                       phones_per_s: float = 12.3, max_frames: int = None):
    """Synthetic TIMIT-like utterance lengths: durations ~ N(3.1 s, 0.9 s) clipped to
    [1.0, 7.8] s; frames at the reference's hop (librosa hop 512 at 16 kHz, timit/preprocess_timit.py:
    196-209) plus 10 zero pad frames each side (:274-276); one label per phone (~12.3 phones/s) plus EOS.
    Returns (frames, labels) int arrays."""
    rng = np.random.default_rng(seed)
    dur = np.clip(rng.normal(3.1, 0.9, n), 1.0, 7.8)
    frames = np.rint(dur * frames_per_s).astype(int) + pad
    labels = np.maximum(np.rint(dur * phones_per_s).astype(int), 1) + 1
    if max_frames is not None:
        frames = np.minimum(frames, max_frames)
    return frames, labels


def synthetic_batch(cfg: ModelConfig, B: int, L: int, T: int, seed: int = 1234, pad: int = 10,
                    eos: int = 23, dtype=np.float64):
    """x ~ N(0,1), zero pad frames each side (timit/preprocess_timit.py:274-276);
    labels uniform over non-EOS classes, last label = EOS (TIMIT EOS = 24 1-based,
    timit/phonemes.txt:25 -> 23 0-based)."""
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((B, L, cfg.inputFrameSize)).astype(dtype)
    if pad > 0 and L > 2 * pad:
        x[:, :pad] = 0
        x[:, L - pad:] = 0
    O = cfg.outputDepth
    choices = np.array([c for c in range(O) if c != eos])
    labels = choices[rng.integers(0, len(choices), size=(B, T))]
    labels[:, -1] = eos
    return x, labels.astype(np.int32)


# ----------------------------------------------------------------------------
# Optimizer step (timit/timit.lua:292-347; optim.adadelta (3p); TrainUtils.lua:52-104)
# ----------------------------------------------------------------------------

def column_norm_constraint(W: Array, maxval: float = 1.0) -> Array:
    """TrainUtils.columnNormConstraint (TrainUtils.lua:52-104): norm = W:norm(2,2) + 1e-8 (per
    output row of W (out, in)); rows with norm >= maxval are divided by norm / maxval (:64-79)."""
    norm = np.sqrt((W * W).sum(1, keepdims=True)) + 1e-8
    div = np.where(norm >= maxval, norm / maxval, 1.0)
    return W / div


_GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def _mix64(z):
    """splitmix64's finaliser on uint64 arrays (wrapping arithmetic)."""
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def gradient_noise(n: int, seed: int, t: int) -> Array:
    """The N(0, 1) draws of gradient-noise step t (timit.lua:310-315 uses torch.randn; the device
    optimizer uses this counter-based form so every rank and launch geometry agree): key =
    mix64(seed * G + t); h_i = mix64(key + i * G); u1 = (h >> 40 + 1) / 2^24, u2 = ((h >> 16) & 0xffffff)
    / 2^24; z = sqrt(-2 ln u1) cos(2 pi u2).  Restates csrc/optim.hip noise_normal."""
    with np.errstate(over="ignore"):
        key = _mix64(np.array([seed], dtype=np.uint64) * _GOLDEN + np.uint64(t))[0]
        h = _mix64(key + np.arange(n, dtype=np.uint64) * _GOLDEN)
    u1 = ((h >> np.uint64(40)) + np.uint64(1)).astype(np.float64) / 16777216.0
    u2 = ((h >> np.uint64(16)) & np.uint64(0xFFFFFF)).astype(np.float64) / 16777216.0
    return np.sqrt(-2.0 * np.log(u1)) * np.cos(2.0 * np.pi * u2)


def optimizer_step(x: Array, g: Array, state: Dict[str, Array], rho: float = 0.95, eps: float = 1e-8,
                   maxnorm: float = 1e20, weightDecay: float = 0.0, colnorm_max: float = 0.0, mats=(),
                   gradnoise_eta: float = 0.0, gradnoise_gamma: float = 0.55, gradnoise_seed: int = 0x5EED):
    """One optimizer step on the flat buffers after the (1/B-scaled) backward:
    clip on the global norm (timit.lua:297-302), L2 (:305-308), optim.adadelta (3p) -- v = rho v +
    (1-rho) g^2; delta = sqrt(u + eps) / sqrt(v + eps) * g; x -= delta; u = rho u + (1-rho) delta^2 --
    and the column-norm constraint on every weight matrix (:344-346).  mats: (offset, rows, cols).
    Gradient noise (:310-315) when gradnoise_eta != 0: t += 1 (state["gradnoise_t"]), g += N(0, 1) *
    (eta / (1 + t)^gamma)^0.5 with the draws of gradient_noise.
    Updates x, g, state in place; returns ||g|| before clipping."""
    gn = float(np.sqrt((g * g).sum()))
    if gn > maxnorm:
        g *= maxnorm / gn
    if weightDecay > 0:
        g += weightDecay * x
    if gradnoise_eta != 0:
        t = state["gradnoise_t"] = state.get("gradnoise_t", 0) + 1
        sigma = (gradnoise_eta / (1 + t) ** gradnoise_gamma) ** 0.5
        g += gradient_noise(g.size, gradnoise_seed, t) * sigma
    v = state.setdefault("paramVariance", np.zeros_like(x))
    u = state.setdefault("accDelta", np.zeros_like(x))
    v *= rho
    v += (1 - rho) * g * g
    delta = np.sqrt(u + eps) / np.sqrt(v + eps) * g
    x -= delta
    u *= rho
    u += (1 - rho) * delta * delta
    if colnorm_max > 0:
        for off, r, c in mats:
            W = x[off:off + r * c].reshape(r, c)
            W[...] = column_norm_constraint(W, colnorm_max)
    return gn


# ----------------------------------------------------------------------------
# Decode path: Attention:BeamSearch (Attention.lua:332-438) and WagnerFischer (utils.lua:3-27)
# ----------------------------------------------------------------------------

def decoder_step(h: Array, Vh: Array, state, yprev: int, P: Dict[str, Array], cfg: "ModelConfig", mlp=None):
    """One decoder_base forward for one utterance (Attention.lua:51-184) in evaluate() mode, the step of
    attention_fwd above for a single row: h (L, A), Vh (L, Sc), state = the reference's hidden
    {alpha_prev (L), s (S), mem (S)} (Attention.lua:360-403; mem is the LSTM decoder's cell, unused by the
    GRU), yprev the previous label (-1 = zeros_y).  mlp: an external decoder_mlp, v = [s; c] (S + A) ->
    log-probabilities (O); None = the fused MaxoutMLP.  Returns (logp (O), new state)."""
    alpha_prev, s, mem = state
    O, M, k = cfg.outputDepth, cfg.mlpDepth, cfg.maxoutWindow
    ws = P["Ws"] @ s + P["bs"]
    Z = ws[None, :] + Vh
    if cfg.hybridAttendFeatureMaps > 0:
        Z = Z + hybrid_features(alpha_prev[None], P, cfg.hybridAttendFilterSize)[0][0]
    e = np.tanh(Z) @ P["we"][0]
    alpha = softmax(e, axis=0)
    c = alpha @ h
    y = np.zeros(O, h.dtype)
    if yprev >= 0:
        y[yprev] = 1.0
    yin = P["Wy"] @ y + P["by"]
    cin = P["Wc"] @ c + P["bc"]
    d = P["Wd"] @ np.concatenate([cin, yin]) + P["bd"]
    if cfg.decoderLSTM:  # LSTM.lua:16-51, x = d, prev_h = s, prev_c = mem
        pre = {q: P[f"dec.W{q}x"] @ d + P[f"dec.b{q}x"] + P[f"dec.W{q}h"] @ s + P[f"dec.b{q}h"] for q in "ifgo"}
        mem = sigmoid(pre["f"]) * mem + sigmoid(pre["i"]) * np.tanh(pre["g"])
        s_new = sigmoid(pre["o"]) * np.tanh(mem)
    else:
        hx = np.concatenate([s, d])
        z = sigmoid(P["dec.Wz"] @ hx)
        r = sigmoid(P["dec.Wr"] @ hx)
        hh = np.tanh(P["dec.Wh"] @ np.concatenate([r * s, d]))
        s_new = (1.0 - z) * s + z * hh
    v = np.concatenate([s_new, c])
    if mlp is not None:
        logp = np.asarray(mlp(v)).reshape(-1)
    else:
        u = P["Wm"] @ v + P["bm"]
        m = u.reshape(M, k).max(1)
        logp = log_softmax(P["Wo"] @ m + P["bo"], 0)
    return logp, (alpha, s_new, mem)


def decoder_zero_state(L: int, S: int, dtype=np.float64):
    """zeros_hidden (Recurrent.lua:112) of the dimhidden {L, S, S} hidden (Attention.lua:318)."""
    return np.zeros(L, dtype), np.zeros(S, dtype), np.zeros(S, dtype)


def beam_search(h: Array, P: Dict[str, Array], cfg: "ModelConfig", eos: int, K: int = 5,
                maxseqlength: Optional[int] = None, mlp=None):
    """Attention:BeamSearch (Attention.lua:332-438) for one utterance h (L, A), 0-based labels.
    Step 0 from zeros_y / zero hidden (:356-367), torch.topk(K) sorted (:369); then while fewer
    than K hypotheses finished and count < maxseqlength (:384): every active hypothesis k is
    extended (p_next[k] = logp + p_beam[k], :386-399), topk(K) over the flattened candidates
    (:400-402), of which the first K - finished are taken (:408): eos or count == maxseqlength
    finishes (:413-417), else it survives with its parent's hidden {alpha, s, mem}.  mlp: an external
    decoder_mlp (decoder_step).  Returns (prediction = the finished hypothesis of highest score
    (first maximum, :432-434), score)."""
    L = h.shape[0]
    maxlen = maxseqlength or L
    Vh = h @ P["V"].T
    logp, st = decoder_step(h, Vh, decoder_zero_state(L, cfg.stateDepth, h.dtype), -1, P, cfg, mlp)
    order = np.argsort(-logp, kind="stable")[:K]
    beams, fin = [], []
    for j in order:
        if j == eos:
            fin.append(([int(j)], float(logp[j])))
        else:
            beams.append(([int(j)], st, float(logp[j])))
    count = 0
    while len(fin) < K and count < maxlen:
        count += 1
        nexts = []
        for seq, sp, pb in beams:
            lp, sn = decoder_step(h, Vh, sp, seq[-1], P, cfg, mlp)
            nexts.append((lp + pb, sn))
        flat = np.concatenate([n[0] for n in nexts])
        O = nexts[0][0].size
        top = np.argsort(-flat, kind="stable")[:K]
        new_beams = []
        for idx in top[:len(beams)]:
            i, j = divmod(int(idx), O)
            seq = beams[i][0] + [j]
            if j == eos or count == maxlen:
                fin.append((seq, float(flat[idx])))
            else:
                new_beams.append((seq, nexts[i][1], float(flat[idx])))
        beams = new_beams
    best = int(np.argmax([f[1] for f in fin]))
    return fin[best][0], fin[best][1]


def wagner_fischer(a, b) -> int:
    """utils.lua:3-27: Levenshtein distance (substitution, insertion, deletion cost 1)."""
    m, n = len(a) + 1, len(b) + 1
    d = np.zeros((m, n), np.int64)
    d[:, 0] = np.arange(m)
    d[0, :] = np.arange(n)
    for j in range(1, n):
        for i in range(1, m):
            if a[i - 1] == b[j - 1]:
                d[i, j] = d[i - 1, j - 1]
            else:
                d[i, j] = min(d[i - 1, j] + 1, d[i, j - 1] + 1, d[i - 1, j - 1] + 1)
    return int(d[m - 1, n - 1])
