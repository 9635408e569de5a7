"""Independent PyTorch-CPU autograd formulation of the Chorowski baseline forward
pass, written directly from the Lua graphs (not from oracle/s2s_oracle.py) so
that the oracle's hand-derived backward can be checked against autograd.

Test infrastructure only.
"""
import torch


def gru_cell(x, h, Wz, Wr, Wh):
    # GRU.lua:22-30
    hx = torch.cat([h, x], -1)
    z = torch.sigmoid(hx @ Wz.t())
    r = torch.sigmoid(hx @ Wr.t())
    hh = torch.tanh(torch.cat([r * h, x], -1) @ Wh.t())
    return (1 - z) * h + z * hh


def rnn(x, Wz, Wr, Wh, reverse):
    # RNN.lua:120-167
    B, L, _ = x.shape
    h = x.new_zeros(B, Wz.shape[0])
    out = [None] * L
    ts = range(L - 1, -1, -1) if reverse else range(L)
    for t in ts:
        h = gru_cell(x[:, t], h, Wz, Wr, Wh)
        out[t] = h
    return torch.stack(out, 1)


def lstm_rnn(x, P, reverse, peepholes=False):
    # LSTM.lua:16-58 driven by RNN.lua
    B, L, _ = x.shape
    H = P["Wix"].shape[0]
    h = x.new_zeros(B, H)
    c = x.new_zeros(B, H)
    out = [None] * L
    ts = range(L - 1, -1, -1) if reverse else range(L)

    def gate(g, xt, hp, peek):
        a = xt @ P[f"W{g}x"].t() + P[f"b{g}x"] + hp @ P[f"W{g}h"].t() + P[f"b{g}h"]
        if peepholes and peek is not None:
            a = a + peek @ P[f"W{g}c"].t() + P[f"b{g}c"]
        return a

    for t in ts:
        xt = x[:, t]
        i = torch.sigmoid(gate("i", xt, h, c))
        f = torch.sigmoid(gate("f", xt, h, c))
        g = torch.tanh(gate("g", xt, h, None))
        cn = f * c + i * g
        o = torch.sigmoid(gate("o", xt, h, cn))
        h = o * torch.tanh(cn)
        c = cn
        out[t] = h
    return torch.stack(out, 1)


def model_forward(x, labels, P, cfg, dropout_mask=None):
    """Returns logp (B, T, O).  P: dict of torch tensors (requires_grad as desired)."""
    inp = x
    for l in range(1, cfg.numLayers + 1):
        yf = rnn(inp, P[f"enc{l}f.Wz"], P[f"enc{l}f.Wr"], P[f"enc{l}f.Wh"], False)
        yb = rnn(inp, P[f"enc{l}b.Wz"], P[f"enc{l}b.Wr"], P[f"enc{l}b.Wh"], True)
        inp = torch.cat([yf, yb], 2)
    h = inp
    B, L, A = h.shape
    T = labels.shape[1]
    O, S, M, k = cfg.outputDepth, cfg.stateDepth, cfg.mlpDepth, cfg.maxoutWindow
    Vh = h @ P["V"].t()
    s = h.new_zeros(B, S)
    aprev = h.new_zeros(B, L)
    jw = torch.arange(L, 0, -1, dtype=h.dtype)
    outs = []
    penalties = []
    for t in range(T):
        y = h.new_zeros(B, O)
        if t > 0:
            y = torch.nn.functional.one_hot(torch.as_tensor(labels[:, t - 1]).long(), O).to(h.dtype)
        ws = s @ P["Ws"].t() + P["bs"]
        Z = ws[:, None, :] + Vh
        nF = getattr(cfg, "hybridAttendFeatureMaps", 0)
        if nF > 0:  # Attention.lua:75-98 via torch's conv1d (cross-correlation = TemporalConvolution)
            kW = cfg.hybridAttendFilterSize
            pl, pr = (kW - 1) // 2, (kW - 1) // 2 if kW % 2 else None
            if kW % 2 == 0:
                pl, pr = kW // 2, kW // 2 - 1
            apad = torch.nn.functional.pad(aprev, (pl, pr))
            Fm = torch.nn.functional.conv1d(apad[:, None, :], P["hybW"][:, None, :], P["hybb"])  # (B, nF, L)
            Z = Z + Fm.transpose(1, 2) @ P["hybU"].t()
        e = (torch.tanh(Z) @ P["we"].t())[..., 0]
        a = torch.softmax(e, 1)
        # MonotonicAlignment as a loss-free regulariser: its backward equals the
        # gradient of lambda * (sum_j (L+1-j)(a_j - aprev_j)) where the indicator is on.
        diff = ((a - aprev) * jw).sum(1)
        penalties.append((diff, a, aprev))
        c = torch.einsum("bl,bla->ba", a, h)
        yin = y @ P["Wy"].t() + P["by"]
        cin = c @ P["Wc"].t() + P["bc"]
        d = torch.cat([cin, yin], 1) @ P["Wd"].t() + P["bd"]
        s = gru_cell(d, s, P["dec.Wz"], P["dec.Wr"], P["dec.Wh"])
        v = torch.cat([s, c], 1)
        if dropout_mask is not None:
            v = v * dropout_mask[:, t]
        u = (v @ P["Wm"].t() + P["bm"]).view(B, M, k)
        m = u.max(2).values
        o = m @ P["Wo"].t() + P["bo"]
        outs.append(torch.log_softmax(o, 1))
        aprev = a
    return torch.stack(outs, 1), penalties
