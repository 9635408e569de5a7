"""Diagnostic: a captured module / model step replayed against the eager step (modes: interleave noeager junk poison parts mods rnn).
Found that hipMemsetAsync nodes did not clear their range on the second replay (the library now clears with fill kernels)."""
import sys
import numpy as np
import torch
sys.path.insert(0, "seq2seq-attention-asr_amd")
import s2s_amd  # noqa: E402

rng = np.random.default_rng(8)
B, L, D, T, O = 3, 64, 20, 7, 11


def make():
    return s2s_amd.ConvBiLSTMAttentionModel(D, numPhonemes=O, hiddenFrameSize=32, outputFrameSize=16, stateDepth=48,
                                            scoreDepth=30, penalty=0.1, generator=torch.Generator().manual_seed(2)).cuda()


def cu(a, dt=torch.float32):
    return torch.tensor(a, dtype=dt, device="cuda")


def inter(m):
    enc = m.encoder
    out = {"dh": m.decoder.gradInput[0], "dc": enc.rnn.gradInput}
    for i, mod in enumerate(enc.convlayer.modules):
        if mod.gradInput is not None:
            out[f"conv{i}.gi"] = mod.gradInput
        out[f"conv{i}.out"] = mod.output
    return out


def report(tag, e, g):
    ie, ig = inter(e), inter(g)
    bad = [k for k in ie if not torch.equal(ie[k], ig[k])]
    pb = [i for i, (a, b) in enumerate(zip(e.parameters()[1], g.parameters()[1])) if not torch.equal(a, b)]
    print(tag, "bad intermediates:", bad, "bad grads:", pb, flush=True)


x = cu(rng.standard_normal((B, L, D)))
labels = cu(rng.integers(0, O, (B, T)), torch.int32)
mode = sys.argv[1] if len(sys.argv) > 1 else "interleave"
eager, graphed = make(), make()
xg, lg = x.clone(), labels.clone()
if mode == "interleave":
    for it in range(3):
        eager.zeroGradParameters()
        eager.step(x, labels)
        graphed.graph_step(xg, lg)
        torch.cuda.synchronize()
        report(f"it{it}", eager, graphed)
elif mode == "noeager":
    eager.zeroGradParameters()
    eager.step(x, labels)
    for it in range(3):
        graphed.graph_step(xg, lg)
        torch.cuda.synchronize()
        report(f"it{it}", eager, graphed)
elif mode == "junk":
    eager.zeroGradParameters()
    eager.step(x, labels)
    for it in range(3):
        graphed.graph_step(xg, lg)
        torch.cuda.synchronize()
        report(f"it{it}", eager, graphed)
        junk = [torch.full((1 << 20,), float("nan"), device="cuda") for _ in range(64)]
        del junk
elif mode == "poison":
    eager.zeroGradParameters()
    eager.step(x, labels)
    s2s_amd.nn._POISON = True
    _empty, _empty_like = torch.empty, torch.empty_like

    def pe(*a, **k):
        t = _empty(*a, **k)
        if t.is_cuda and t.is_floating_point():
            t.fill_(float("nan"))
        return t

    def pel(*a, **k):
        t = _empty_like(*a, **k)
        if t.is_cuda and t.is_floating_point():
            t.fill_(float("nan"))
        return t
    torch.empty, torch.empty_like = pe, pel
    graphed.zeroGradParameters()
    graphed.step(xg, lg)
    torch.cuda.synchronize()
    report("poison", eager, graphed)
    ie = inter(graphed)
    print({k: bool(torch.isnan(v).any()) for k, v in ie.items()})
    print([i for i, gg in enumerate(graphed.parameters()[1]) if torch.isnan(gg).any()])
elif mode == "parts":
    def cap(fn):
        fn(); torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph(); side = torch.cuda.Stream(); side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.graph(graph, stream=side, capture_error_mode="thread_local"):
            out = fn()
        torch.cuda.current_stream().wait_stream(side)
        return graph, out
    from s2s_amd.nn import nll_seed
    h = cu(rng.standard_normal((B, 8, 32)))
    dh0 = cu(rng.standard_normal((B, 8, 32)))

    def dec_step(m):
        dec = m.decoder
        dec.zeroGradParameters()
        logp = dec.forward([h, labels])
        nll, dlogp = nll_seed(logp, labels, False)
        return dec.backward([h, labels], dlogp, 0.5)[0]

    def enc_step(m):
        m.encoder.zeroGradParameters()
        m.encoder.forward(x)
        return m.encoder.backward(x, dh0, 0.5)

    for name, fn, sl in (("decoder", dec_step, slice(22, None)), ("encoder", enc_step, slice(0, 22))):
        e, g = make(), make()
        gr, outg = cap(lambda: fn(g))
        for it in range(3):
            oute = fn(e)
            gr.replay(); torch.cuda.synchronize()
            pe_, pg_ = e.parameters()[1][sl], g.parameters()[1][sl]
            print(name, it, "out eq", torch.equal(oute, outg) if oute is not None else None,
                  "bad grads", [i for i, (a, b) in enumerate(zip(pe_, pg_)) if not torch.equal(a, b)], flush=True)
elif mode == "mods":
    from s2s_amd import frontend as F
    from s2s_amd.nn import nll_seed

    def cap(fn):
        fn(); torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph(); side = torch.cuda.Stream(); side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.graph(graph, stream=side, capture_error_mode="thread_local"):
            out = fn()
        torch.cuda.current_stream().wait_stream(side)
        return graph, out

    def run(name, mk, inp, gy):
        def fn(m):
            m.zeroGradParameters()
            y = m.forward(inp)
            gi = m.backward(inp, gy, 0.5)
            return [y, gi]
        e, g = mk(), mk()
        gr, outg = cap(lambda: fn(g))
        for it in range(3):
            oute = fn(e)
            gr.replay(); torch.cuda.synchronize()
            eqo = [torch.equal(a, b) if a is not None else None for a, b in zip(oute, outg)]
            bad = [i for i, (a, b) in enumerate(zip(e.parameters()[1], g.parameters()[1])) if not torch.equal(a, b)]
            print(name, it, "y/gi eq", eqo, "bad grads", bad, flush=True)

    gen = lambda: torch.Generator().manual_seed(5)
    x3 = cu(rng.standard_normal((3, 64, 20)))
    run("tconv_k3_relu", lambda: F.TemporalConvolution(20, 32, 3, relu=True, generator=gen()).cuda(), x3,
        cu(rng.standard_normal((3, 62, 32))))
    run("tconv_k3_relu_nogi", lambda: F.TemporalConvolution(20, 32, 3, relu=True, need_gradInput=False, generator=gen()).cuda(), x3,
        cu(rng.standard_normal((3, 62, 32))))
    run("tmaxpool", lambda: F.TemporalMaxPooling(2, 2), x3, cu(rng.standard_normal((3, 32, 20))))
    x2 = cu(rng.standard_normal((21, 64)))
    run("linear", lambda: F.Linear(64, 22, generator=gen()).cuda(), x2, cu(rng.standard_normal((21, 22))))
    run("logsoftmax", lambda: F.LogSoftMax(), x2, cu(rng.standard_normal((21, 64))))
    run("seq_mlp", lambda: F.Sequential(F.Linear(64, 22, generator=gen()), F.ReLU(), F.Linear(22, 11, generator=gen()), F.LogSoftMax()).cuda(),
        x2, cu(rng.standard_normal((21, 11))))
    run("convstack", lambda: F.Sequential(F.TemporalConvolution(20, 32, 3, relu=True, need_gradInput=False, generator=gen()), F.TemporalMaxPooling(2, 2),
                                          F.TemporalConvolution(32, 32, 3, relu=True, generator=gen()), F.TemporalMaxPooling(2, 2)).cuda(),
        x3, cu(rng.standard_normal((3, 14, 32))))
elif mode == "rnn":
    from s2s_amd import frontend as F

    def cap(fn):
        fn(); torch.cuda.synchronize()
        graph = torch.cuda.CUDAGraph(); side = torch.cuda.Stream(); side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.graph(graph, stream=side, capture_error_mode="thread_local"):
            out = fn()
        torch.cuda.current_stream().wait_stream(side)
        return graph, out

    def run(name, mk, inp, gy):
        def fn(m):
            m.zeroGradParameters()
            y = m.forward(inp)
            gi = m.backward(inp, gy, 0.5)
            return [y, gi]
        e, g = mk(), mk()
        gr, outg = cap(lambda: fn(g))
        for it in range(3):
            oute = fn(e)
            gr.replay(); torch.cuda.synchronize()
            eqo = [torch.equal(a, b) if a is not None else None for a, b in zip(oute, outg)]
            bad = [i for i, (a, b) in enumerate(zip(e.parameters()[1], g.parameters()[1])) if not torch.equal(a, b)]
            print(name, it, "y/gi eq", eqo, "bad grads", bad, flush=True)

    gen = lambda s: torch.Generator().manual_seed(s)
    for (Bq, Lq, Dq, Hq) in ((3, 6, 32, 16), (3, 64, 20, 16)):
        xq = cu(rng.standard_normal((Bq, Lq, Dq)))
        gyq = cu(rng.standard_normal((Bq, Lq, 2 * Hq)))
        run(f"bilstm B{Bq} L{Lq}", lambda: s2s_amd.BiRNN(s2s_amd.LSTM(Dq, Hq, False, gen(1)), s2s_amd.LSTM(Dq, Hq, False, gen(2))).cuda(), xq, gyq)
        run(f"lstm1 B{Bq} L{Lq}", lambda: s2s_amd.RNN(s2s_amd.LSTM(Dq, Hq, False, gen(1))).cuda(), xq, gyq[:, :, :Hq].contiguous())
        run(f"bigru B{Bq} L{Lq}", lambda: s2s_amd.BiRNN(s2s_amd.GRU(Dq, Hq, gen(1)), s2s_amd.GRU(Dq, Hq, gen(2))).cuda(), xq, gyq)
    enc = lambda: F.ConvBiLSTMEncoder(20, 32, 16, 3, generator=gen(3)).cuda()
    run("encoder", enc, x, cu(rng.standard_normal((B, 6, 32))))
