"""nn.Module mirrors of the encoder front-ends over libs2s_hip.so.

Operators (Torch7 nn semantics, include/s2s_hip.h "encoder front-ends"): TemporalConvolution,
TemporalMaxPooling, ReLU, SpatialConvolutionMM, SpatialMaxPooling, Transpose2 and a Sequential
container; and the two encoders the reference builds from them:
  * ConvBiLSTMEncoder -- timit/timit.lua:108-125 (conv stack shared by both LSTM directions);
  * VGGEncoder        -- librispeech/model_vgg.lua:23-51.
A convolution built with relu=True is the reference's `conv -> nn.ReLU()` pair fused (the ReLU runs in
the GEMM epilogue; its backward masks by the conv output).  Gradients accumulate; backward returns
gradInput (None for a module built with need_gradInput=False: the encoder input needs none).
"""
import contextlib
import math

import torch

from ._lib import check, lib
from .nn import (LSTM, BiRNN, Module, S2SArgumentError, _bytes, _require_cuda_f32, _uniform, dptr, get_context,
                 overlap_param_grads, side_uses, stream_ptr)


def _ctx(t):
    return get_context(t.device.index).handle


class TemporalConvolution(Module):
    """nn.TemporalConvolution(inputFrameSize, outputFrameSize, kW) (dW = 1): weight (out, kW*in), bias (out);
    reset U(+-1/sqrt(kW*in)).  bias=False gives TemporalConvolutionZeroBias (TemporalConvolutionZeroBias.lua)."""

    def __init__(self, inputFrameSize, outputFrameSize, kW, relu=False, bias=True, need_gradInput=True,
                 generator=None):
        super().__init__()
        self.inputFrameSize, self.outputFrameSize, self.kW = inputFrameSize, outputFrameSize, kW
        self.relu, self.need_gradInput = bool(relu), need_gradInput
        stdv = 1.0 / math.sqrt(kW * inputFrameSize)
        self.weight = _uniform((outputFrameSize, kW * inputFrameSize), stdv, generator)
        self.bias = _uniform((outputFrameSize,), stdv, generator) if bias else None
        self.gradWeight = torch.zeros_like(self.weight)
        self.gradBias = torch.zeros_like(self.bias) if bias else None

    def parameters(self):
        ws = [self.weight] + ([self.bias] if self.bias is not None else [])
        gs = [self.gradWeight] + ([self.gradBias] if self.gradBias is not None else [])
        return ws, gs

    def updateOutput(self, input):
        _require_cuda_f32(input, "input")
        self._check_params(input)
        x = input if input.dim() == 3 else input.unsqueeze(0)
        if x.dim() != 3 or x.shape[2] != self.inputFrameSize:
            raise S2SArgumentError("TemporalConvolution: input must be (L, inputFrameSize) or (B, L, inputFrameSize)")
        B, L, _ = x.shape
        y = torch.empty((B, L - self.kW + 1, self.outputFrameSize), device=x.device, dtype=torch.float32)
        check(lib.s2s_tconv_fwd(_ctx(x), stream_ptr(), B, L, self.inputFrameSize, self.outputFrameSize, self.kW,
                                int(self.relu), dptr(x), dptr(self.weight), dptr(self.bias), dptr(y)))
        self.output = y if input.dim() == 3 else y[0]
        return self.output

    def backward(self, input, gradOutput, scale=1.0):
        x = input if input.dim() == 3 else input.unsqueeze(0)
        B, L, _ = x.shape
        go = (gradOutput if gradOutput.dim() == 3 else gradOutput.unsqueeze(0)).contiguous()
        y = self.output if self.output.dim() == 3 else self.output.unsqueeze(0)
        dx = torch.empty_like(x) if self.need_gradInput else None
        scr = _bytes(lib.s2s_tconv_scratch_bytes(B, L, self.inputFrameSize, self.outputFrameSize, self.kW), x.device)
        check(lib.s2s_tconv_bwd(_ctx(x), stream_ptr(), B, L, self.inputFrameSize, self.outputFrameSize, self.kW,
                                int(self.relu), dptr(x), dptr(self.weight), dptr(y), dptr(go), dptr(dx), 0,
                                dptr(self.gradWeight), dptr(self.gradBias), float(scale), dptr(scr), scr.numel()))
        side_uses(x.device, scr)
        self.gradInput = None if dx is None else (dx if input.dim() == 3 else dx[0])
        return self.gradInput


class TemporalMaxPooling(Module):
    """nn.TemporalMaxPooling(kW, dW): floor mode, first maximum wins."""

    def __init__(self, kW, dW=None):
        super().__init__()
        self.kW, self.dW = kW, dW or kW

    def updateOutput(self, input):
        _require_cuda_f32(input, "input")
        self._check_params(input)
        x = input if input.dim() == 3 else input.unsqueeze(0)
        B, L, D = x.shape
        Lo = (L - self.kW) // self.dW + 1
        y = torch.empty((B, Lo, D), device=x.device, dtype=torch.float32)
        self.indices = torch.empty((B, Lo, D), device=x.device, dtype=torch.int32)
        check(lib.s2s_tmaxpool_fwd(_ctx(x), stream_ptr(), B, L, D, self.kW, self.dW, dptr(x), dptr(y),
                                   dptr(self.indices)))
        self.output = y if input.dim() == 3 else y[0]
        return self.output

    def backward(self, input, gradOutput, scale=1.0):
        x = input if input.dim() == 3 else input.unsqueeze(0)
        B, L, D = x.shape
        go = (gradOutput if gradOutput.dim() == 3 else gradOutput.unsqueeze(0)).contiguous()
        dx = torch.empty_like(x)
        check(lib.s2s_tmaxpool_bwd(_ctx(x), stream_ptr(), B, L, D, self.kW, self.dW, dptr(self.indices), dptr(go),
                                   dptr(dx)))
        self.gradInput = dx if input.dim() == 3 else dx[0]
        return self.gradInput


class ReLU(Module):
    """nn.ReLU: y = max(x, 0); dx = dy * 1[x > 0]."""

    def updateOutput(self, input):
        _require_cuda_f32(input, "input")
        self._check_params(input)
        self.output = torch.empty_like(input)
        check(lib.s2s_relu_fwd(_ctx(input), stream_ptr(), input.numel(), dptr(input), dptr(self.output)))
        return self.output

    def backward(self, input, gradOutput, scale=1.0):
        go = gradOutput.contiguous()
        self.gradInput = torch.empty_like(input)
        check(lib.s2s_relu_bwd(_ctx(input), stream_ptr(), input.numel(), dptr(input), dptr(go),
                               dptr(self.gradInput)))
        return self.gradInput


class Linear(TemporalConvolution):
    """nn.Linear(inputSize, outputSize): weight (out, in), bias (out), reset U(+-1/sqrt(in)); rows (N, in) or
    (B, T, in).  Runs as TemporalConvolution(in, out, 1) (one GEMM over the rows, bias in the epilogue)."""

    def __init__(self, inputSize, outputSize, relu=False, generator=None):
        super().__init__(inputSize, outputSize, 1, relu=relu, generator=generator)


class Maxout(Module):
    """nn.Maxout(inputDimension, outputDimension, window) (Maxout.lua:5-19): Linear(in, out*window) ->
    View(out*window, 1) -> TemporalMaxPooling(window, window) -> View(out), on rows (N, in)."""

    def __init__(self, inputDimension, outputDimension, window=4, generator=None):
        super().__init__()
        self.inputDim, self.outputDim, self.window = inputDimension, outputDimension, window
        self.linear = Linear(inputDimension, outputDimension * window, generator=generator)
        self.pool = TemporalMaxPooling(window, window)

    def parameters(self):
        return self.linear.parameters()

    def updateOutput(self, input):
        if input.dim() != 2:
            raise S2SArgumentError("Maxout: rows (N, inputDimension)")
        self._u = self.linear.forward(input)
        N = input.shape[0]
        self.output = self.pool.forward(self._u.reshape(N, -1, 1)).reshape(N, self.outputDim)
        return self.output

    def backward(self, input, gradOutput, scale=1.0):
        N = input.shape[0]
        du = self.pool.backward(self._u.reshape(N, -1, 1), gradOutput.reshape(N, self.outputDim, 1).contiguous())
        self.gradInput = self.linear.backward(input, du.reshape(N, -1), scale)
        return self.gradInput


class LogSoftMax(Module):
    """nn.LogSoftMax over the last dimension."""

    def updateOutput(self, input):
        _require_cuda_f32(input, "input")
        self._check_params(input)
        n = input.shape[-1]
        self.output = torch.empty_like(input)
        check(lib.s2s_logsoftmax_fwd(_ctx(input), stream_ptr(), input.numel() // n, n, dptr(input),
                                     dptr(self.output)))
        return self.output

    def backward(self, input, gradOutput, scale=1.0):
        n = input.shape[-1]
        go = gradOutput.contiguous()
        self.gradInput = torch.empty_like(input)
        check(lib.s2s_logsoftmax_bwd(_ctx(input), stream_ptr(), input.numel() // n, n, dptr(self.output), dptr(go),
                                     dptr(self.gradInput)))
        return self.gradInput


class SpatialConvolutionMM(Module):
    """nn.SpatialConvolutionMM(nInputPlane, nOutputPlane, kW, kH) (stride 1, no padding): weight
    (out, in*kH*kW), bias (out); reset U(+-1/sqrt(kW*kH*in)).  Input (B, C, H, W) or (C, H, W)."""

    def __init__(self, nInputPlane, nOutputPlane, kW, kH=None, relu=False, need_gradInput=True, generator=None):
        super().__init__()
        self.nInputPlane, self.nOutputPlane, self.kW, self.kH = nInputPlane, nOutputPlane, kW, kH or kW
        self.relu, self.need_gradInput = bool(relu), need_gradInput
        stdv = 1.0 / math.sqrt(self.kW * self.kH * nInputPlane)
        self.weight = _uniform((nOutputPlane, nInputPlane * self.kH * self.kW), stdv, generator)
        self.bias = _uniform((nOutputPlane,), stdv, generator)
        self.gradWeight = torch.zeros_like(self.weight)
        self.gradBias = torch.zeros_like(self.bias)

    def parameters(self):
        return [self.weight, self.bias], [self.gradWeight, self.gradBias]

    def _dims(self, x):
        if x.dim() != 4 or x.shape[1] != self.nInputPlane:
            raise S2SArgumentError("SpatialConvolutionMM: input must be (C, H, W) or (B, C, H, W) with C = nInputPlane")
        return x.shape

    def updateOutput(self, input):
        _require_cuda_f32(input, "input")
        self._check_params(input)
        x = input if input.dim() == 4 else input.unsqueeze(0)
        B, C, H, W = self._dims(x)
        y = torch.empty((B, self.nOutputPlane, H - self.kH + 1, W - self.kW + 1), device=x.device,
                        dtype=torch.float32)
        scr = _bytes(lib.s2s_sconv_scratch_bytes(B, C, H, W, self.nOutputPlane, self.kH, self.kW), x.device)
        self._scr = (scr, x.data_ptr(), x.shape)  # the im2col panel, reused by the backward on the same input
        check(lib.s2s_sconv_fwd(_ctx(x), stream_ptr(), B, C, H, W, self.nOutputPlane, self.kH, self.kW,
                                int(self.relu), dptr(x), dptr(self.weight), dptr(self.bias), dptr(y), dptr(scr),
                                scr.numel()))
        self.output = y if input.dim() == 4 else y[0]
        return self.output

    def backward(self, input, gradOutput, scale=1.0):
        x = input if input.dim() == 4 else input.unsqueeze(0)
        B, C, H, W = self._dims(x)
        go = (gradOutput if gradOutput.dim() == 4 else gradOutput.unsqueeze(0)).contiguous()
        y = self.output if self.output.dim() == 4 else self.output.unsqueeze(0)
        dx = torch.empty_like(x) if self.need_gradInput else None
        saved = getattr(self, "_scr", None)
        reuse = saved is not None and saved[1] == x.data_ptr() and saved[2] == x.shape
        scr = saved[0] if reuse else _bytes(lib.s2s_sconv_scratch_bytes(B, C, H, W, self.nOutputPlane, self.kH,
                                                                         self.kW), x.device)
        check(lib.s2s_sconv_bwd(_ctx(x), stream_ptr(), B, C, H, W, self.nOutputPlane, self.kH, self.kW,
                                int(self.relu), dptr(x), dptr(self.weight), dptr(y), dptr(go), dptr(dx), 0,
                                dptr(self.gradWeight), dptr(self.gradBias), float(scale), dptr(scr), scr.numel(),
                                int(reuse)))
        self._scr = None
        self.gradInput = None if dx is None else (dx if input.dim() == 4 else dx[0])
        return self.gradInput


class SpatialMaxPooling(Module):
    """nn.SpatialMaxPooling(kW, kH, dW, dH) (floor mode, first maximum wins)."""

    def __init__(self, kW, kH, dW=None, dH=None):
        super().__init__()
        self.kW, self.kH, self.dW, self.dH = kW, kH, dW or kW, dH or kH

    def updateOutput(self, input):
        _require_cuda_f32(input, "input")
        self._check_params(input)
        x = input if input.dim() == 4 else input.unsqueeze(0)
        B, C, H, W = x.shape
        Ho, Wo = (H - self.kH) // self.dH + 1, (W - self.kW) // self.dW + 1
        y = torch.empty((B, C, Ho, Wo), device=x.device, dtype=torch.float32)
        self.indices = torch.empty((B, C, Ho, Wo), device=x.device, dtype=torch.int32)
        check(lib.s2s_smaxpool_fwd(_ctx(x), stream_ptr(), B, C, H, W, self.kW, self.kH, self.dW, self.dH, dptr(x),
                                   dptr(y), dptr(self.indices)))
        self.output = y if input.dim() == 4 else y[0]
        return self.output

    def backward(self, input, gradOutput, scale=1.0):
        x = input if input.dim() == 4 else input.unsqueeze(0)
        B, C, H, W = x.shape
        go = (gradOutput if gradOutput.dim() == 4 else gradOutput.unsqueeze(0)).contiguous()
        dx = torch.empty_like(x)
        check(lib.s2s_smaxpool_bwd(_ctx(x), stream_ptr(), B, C, H, W, self.kW, self.kH, self.dW, self.dH,
                                   dptr(self.indices), dptr(go), dptr(dx)))
        self.gradInput = dx if input.dim() == 4 else dx[0]
        return self.gradInput


class Transpose2(Module):
    """nn.Transpose2({1,2},3) (Transpose2.lua): (nFeat, L, H) -> (L, nFeat, H), batched (B, nFeat, L, H) ->
    (B, L, nFeat, H).  Only this permutation (the one model_vgg.lua:41 uses) runs on this path."""

    def __init__(self, *perms):
        super().__init__()
        if perms not in (((1, 2), 3), ([1, 2], 3)):
            raise S2SArgumentError("Transpose2: only ({1,2}, 3) is implemented")

    def updateOutput(self, input):
        _require_cuda_f32(input, "input")
        self._check_params(input)
        if input.dim() not in (3, 4):
            raise S2SArgumentError("inconsistent tensor size")  # Transpose2.lua:29
        x = input if input.dim() == 4 else input.unsqueeze(0)
        B, D1, D2, D3 = x.shape
        y = torch.empty((B, D2, D1, D3), device=x.device, dtype=torch.float32)
        check(lib.s2s_swap12(_ctx(x), stream_ptr(), B, D1, D2, D3, dptr(x), dptr(y)))
        self.output = y if input.dim() == 4 else y[0]
        return self.output

    def backward(self, input, gradOutput, scale=1.0):
        x = input if input.dim() == 4 else input.unsqueeze(0)
        B, D1, D2, D3 = x.shape
        go = (gradOutput if gradOutput.dim() == 4 else gradOutput.unsqueeze(0)).contiguous()
        dx = torch.empty_like(x)
        check(lib.s2s_swap12(_ctx(x), stream_ptr(), B, D2, D1, D3, dptr(go), dptr(dx)))
        self.gradInput = dx if input.dim() == 4 else dx[0]
        return self.gradInput


class View(Module):
    """nn.View(-1, n):setNumInputDims(3) on a batch: (B, L, C, H) -> (B, L, C*H) (a free reshape)."""

    def updateOutput(self, input):
        self.output = input.reshape(input.shape[0], input.shape[1], -1)
        return self.output

    def backward(self, input, gradOutput, scale=1.0):
        self.gradInput = gradOutput.reshape(input.shape)
        return self.gradInput


class Sequential(Module):
    """nn.Sequential: forward in order, backward in reverse (each module's backward = updateGradInput +
    accGradParameters)."""

    def __init__(self, *modules):
        super().__init__()
        self.modules = list(modules)

    def add(self, m):
        self.modules.append(m)
        return self

    def parameters(self):
        ws, gs = [], []
        for m in self.modules:
            w, g = m.parameters()
            ws += w
            gs += g
        return ws, gs

    def updateOutput(self, input):
        self._inputs = []
        h = input
        for m in self.modules:
            self._inputs.append(h)
            h = m.forward(h)
        self.output = h
        return h

    def backward(self, input, gradOutput, scale=1.0):
        d = gradOutput
        for m, x in zip(reversed(self.modules), reversed(self._inputs)):
            d = m.backward(x, d, scale)
        self.gradInput = d
        return d


class ConvBiLSTMEncoder(Module):
    """timit/timit.lua:108-125: convlayer = 3 x [TemporalConvolution(D, hidden, kW) -> ReLU ->
    TemporalMaxPooling(2, 2)], applied once and read by both RNN(LSTM(hidden, out, peepholes=nil))
    directions (the reference calls the same module on the same input twice, :123-124, so the
    forward is one conv stack and its weight gradients sum both directions' contributions), then
    JoinTable(2,2).  x (B, L, D) -> (B, L', 2*out), L' = three times (L - kW + 1) // 2."""

    def __init__(self, inputFrameSize, hiddenFrameSize=256, outputFrameSize=128, kW=3, generator=None):
        super().__init__()
        convs = []
        for l in range(3):
            convs += [TemporalConvolution(inputFrameSize if l == 0 else hiddenFrameSize, hiddenFrameSize, kW, relu=True,
                                          need_gradInput=l > 0, generator=generator),
                      TemporalMaxPooling(2, 2)]
        self.convlayer = Sequential(*convs)
        self.rnn = BiRNN(LSTM(hiddenFrameSize, outputFrameSize, False, generator),
                         LSTM(hiddenFrameSize, outputFrameSize, False, generator))

    def parameters(self):
        w1, g1 = self.convlayer.parameters()
        w2, g2 = self.rnn.parameters()
        return w1 + w2, g1 + g2

    def updateOutput(self, input):
        self._c = self.convlayer.forward(input)
        self.output = self.rnn.forward(self._c)
        return self.output

    def backward(self, input, gradOutput, scale=1.0):
        dc = self.rnn.backward(self._c, gradOutput, scale)  # sum of both directions' dx
        self.gradInput = self.convlayer.backward(input, dc, scale)
        return self.gradInput


class VGGEncoder(Module):
    """librispeech/model_vgg.lua:23-51 on x (B, 3, L, F) (H = time, W = frequency) -> (B, (L-8)//2, out):
    SpatialConvolutionMM(3,64,3,3)+ReLU, (64,64)+ReLU, SpatialMaxPooling(2,1,2,1), (64,128)+ReLU,
    (128,128)+ReLU, SpatialMaxPooling(2,2,2,2), Transpose2({1,2},3), View(-1, 128*H'), then
    TemporalConvolution(128*H', hidden, 1), (hidden, hidden, 1) x 2, (hidden, out, 1), each + ReLU."""

    def __init__(self, inputFrameSize=40, outputFrameSize=512, hidden=2048, generator=None):
        super().__init__()
        Hf = ((inputFrameSize - 4) // 2 - 4) // 2
        if Hf < 1:
            raise S2SArgumentError("VGGEncoder: inputFrameSize too small for the conv stack")
        g = generator
        self.seq = Sequential(
            SpatialConvolutionMM(3, 64, 3, 3, relu=True, need_gradInput=False, generator=g),
            SpatialConvolutionMM(64, 64, 3, 3, relu=True, generator=g),
            SpatialMaxPooling(2, 1, 2, 1),
            SpatialConvolutionMM(64, 128, 3, 3, relu=True, generator=g),
            SpatialConvolutionMM(128, 128, 3, 3, relu=True, generator=g),
            SpatialMaxPooling(2, 2, 2, 2),
            Transpose2((1, 2), 3),
            View(),
            TemporalConvolution(128 * Hf, hidden, 1, relu=True, generator=g),
            TemporalConvolution(hidden, hidden, 1, relu=True, generator=g),
            TemporalConvolution(hidden, hidden, 1, relu=True, generator=g),
            TemporalConvolution(hidden, outputFrameSize, 1, relu=True, generator=g))

    def parameters(self):
        return self.seq.parameters()

    def updateOutput(self, input):
        self.output = self.seq.forward(input)
        return self.output

    def backward(self, input, gradOutput, scale=1.0):
        self.gradInput = self.seq.backward(input, gradOutput, scale)
        return self.gradInput


class GraphStep:
    """graph_step() for the host-side models (VGGAttentionModel, ConvBiLSTMAttentionModel): their step is a
    sequence of module calls from Python (front-end Sequential, decoder, decoder_mlp, loss seed and every
    backward), hundreds of launches -- the per-step decoder kernels of the conv + BiLSTM model alone launch a
    handful per decoder step -- replayed from one captured HIP graph."""

    def graph_step(self, x, labels, scale=None, normalizeNLL=False):
        """zeroGradParameters() + step() replayed from a captured HIP graph: every launch of the host-side
        step (front-end, decoder, decoder_mlp, loss seed and every backward) becomes one graph launch.  The
        capture is keyed by the input / label buffers (pointers and shapes): refill x and labels in place to
        train on new data.  The first call of a key runs one eager step
        (which sizes every lazily grown buffer, so the capture allocates only from its graph pool), then
        captures and replays; the returned (nll, logp) are the graph's own buffers, rewritten by every
        replay.  grads = this step's gradient (the graph zeroes them first)."""
        key = (x.data_ptr(), tuple(x.shape), labels.data_ptr(), tuple(labels.shape), scale, normalizeNLL)
        graphs = self.__dict__.setdefault("_graphs", {})
        g = graphs.get(key)
        if g is None:
            # the eager step runs on the capture stream: the library's lazily grown per-stream buffers (the big
            # bf16 GEMMs' staging copies) are sized for THAT stream before the capture, which cannot allocate them
            # one capture stream per model: the library keeps a few per-stream staging buffers, so a
            # fresh stream per key would use them up with shapes (ragged batches) and leave dead streams' buffers
            cur = torch.cuda.current_stream(x.device)
            side = self.__dict__.get("_capture_stream")
            if side is None or side.device != x.device:
                side = self.__dict__["_capture_stream"] = torch.cuda.Stream(x.device)
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                self.zeroGradParameters()
                self.step(x, labels, scale, normalizeNLL)
            side.synchronize()
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=side, capture_error_mode="thread_local"):
                self.zeroGradParameters()
                out = self.step(x, labels, scale, normalizeNLL)
            cur.wait_stream(side)
            graphs[key] = g = (graph, out)
        g[0].replay()
        return g[1]



class VGGAttentionModel(GraphStep, Module):
    """librispeech/model_vgg.lua:loadmodel(opt) end to end: VGGEncoder -> nn.Attention(GRU(S, S),
    decoder_mlp = Maxout(S+A, M, 7) -> Linear(M, M) -> Maxout(M, M, 7) -> Linear(M, O) -> LogSoftMax
    (:71-77), scoreDepth, hybrid (off by default), S, A, O, monoAlignPenalty = true, penalty) with the
    loss seed of librispeech/train.lua (nll = -sum labelmask * logp, dlogp = -labelmask, grads / B).
    The decoder_mlp runs outside the decoder launches on the saved [s_t; c_t] rows (external_mlp)."""

    def __init__(self, inputFrameSize=40, outputFrameSize=512, hidden=2048, scoreDepth=512, stateDepth=256,
                 outputDepth=62, mlpDepth=64, penalty=0.0, generator=None, precision="fp32"):
        from .nn import GRU, Attention
        super().__init__()
        # "bf16": every hoisted GEMM of the step (the VGG convolutions and 1x1 layers, Vh, decoder folds, the
        # decoder_mlp Linears, all weight gradients) on bf16 MFMA with fp32 accumulation (BASELINE config 5)
        self.precision = precision
        self.overlap = True  # parameter gradients on the side stream during the backward (overlap_param_grads)
        g = generator
        S, A, M, O = stateDepth, outputFrameSize, mlpDepth, outputDepth
        self.encoder = VGGEncoder(inputFrameSize, outputFrameSize, hidden, generator=g)
        mlp = Sequential(Maxout(S + A, M, 7, generator=g), Linear(M, M, generator=g), Maxout(M, M, 7, generator=g),
                         Linear(M, O, generator=g), LogSoftMax())
        self.decoder = Attention(GRU(S, S, generator=g), mlp, scoreDepth, 10, 0, S, A, O, True, penalty, generator=g)

    def parameters(self):
        w1, g1 = self.encoder.parameters()
        w2, g2 = self.decoder.parameters()
        return w1 + w2, g1 + g2

    def step(self, x, labels, scale=None, normalizeNLL=False):
        """One training step on x (B, 3, L, F), labels (B, T) 0-based: forward, nll, backward with
        gradients accumulated at scale (default 1/B).  Returns (nll (B,), logp (B, T, O))."""
        from .nn import nll_seed, precision
        B = x.shape[0]
        scale = (1.0 / B if B > 1 else 1.0) if scale is None else scale
        with precision(self.precision, x.device.index):
            h = self.encoder.forward(x)
            lab = labels.to(torch.int32).contiguous()
            logp = self.decoder.forward([h, lab])
            nll, dlogp = nll_seed(logp, lab, normalizeNLL)
            # each module's parameter gradients beside the next module's backward (bitwise the serial sums)
            with overlap_param_grads(x.device.index) if self.overlap else contextlib.nullcontext():
                dh = self.decoder.backward([h, lab], dlogp, scale)[0]
                self.encoder.backward(x, dh, scale)
        return nll, logp

class ConvBiLSTMAttentionModel(GraphStep, Module):
    """The conv + BiLSTM model timit/timit.lua builds when no model file is given (:106-145), end to end:
    ConvBiLSTMEncoder (3 x conv(k=3, 256) + ReLU + TemporalMaxPooling(2, 2), BiLSTM 2 x 128) ->
    nn.Attention(decoder_recurrent = LSTM(400, 400), decoder_mlp = Linear(400 + 256, 2*O) -> ReLU ->
    Linear(2*O, O) -> LogSoftMax, scoreDepth 150, hybrid attention kW = 5 / 16 maps, monoAlignPenalty
    true, opt.penalty), with the trainer's loss seed (timit/timit.lua:262-295)."""

    def __init__(self, inputFrameSize=123, numPhonemes=62, hiddenFrameSize=256, outputFrameSize=128,
                 stateDepth=400, scoreDepth=150, hybridAttendFilterSize=5, hybridAttendFeatureMaps=16, penalty=0.0,
                 generator=None, precision="fp32"):
        from .nn import Attention
        super().__init__()
        self.precision = precision  # "fp32" | "bf16" | "bf16-all" (s2s_amd.precision) for the step's GEMMs
        self.overlap = True  # parameter gradients on the side stream during the backward (overlap_param_grads)
        g = generator
        S, A, O = stateDepth, 2 * outputFrameSize, numPhonemes
        self.encoder = ConvBiLSTMEncoder(inputFrameSize, hiddenFrameSize, outputFrameSize, 3, generator=g)
        mlp = Sequential(Linear(S + A, 2 * O, generator=g), ReLU(), Linear(2 * O, O, generator=g), LogSoftMax())
        self.decoder = Attention(LSTM(S, S, False, g), mlp, scoreDepth, hybridAttendFilterSize,
                                 hybridAttendFeatureMaps, S, A, O, True, penalty, generator=g)

    def parameters(self):
        w1, g1 = self.encoder.parameters()
        w2, g2 = self.decoder.parameters()
        return w1 + w2, g1 + g2

    def step(self, x, labels, scale=None, normalizeNLL=False):
        """One training step on x (B, L, D), labels (B, T) 0-based; gradients accumulate at scale
        (default 1/B).  Returns (nll (B,), logp (B, T, O))."""
        from .nn import nll_seed, precision
        B = x.shape[0]
        scale = (1.0 / B if B > 1 else 1.0) if scale is None else scale
        with precision(self.precision, x.device.index):
            h = self.encoder.forward(x)
            lab = labels.to(torch.int32).contiguous()
            logp = self.decoder.forward([h, lab])
            nll, dlogp = nll_seed(logp, lab, normalizeNLL)
            # each module's parameter gradients beside the next module's backward (bitwise the serial sums)
            with overlap_param_grads(x.device.index) if self.overlap else contextlib.nullcontext():
                dh = self.decoder.backward([h, lab], dlogp, scale)[0]
                self.encoder.backward(x, dh, scale)
        return nll, logp
