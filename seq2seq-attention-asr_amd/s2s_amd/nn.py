"""nn.Module-protocol mirrors of the reference's hot-path modules, on libs2s_hip.so.

Protocol kept from Torch7: `forward(input)` = `updateOutput`,
`backward(input, gradOutput, scale)` = `updateGradInput` + `accGradParameters`,
`parameters()` -> ([weights], [gradWeights]), `zeroGradParameters()`, gradients
accumulate, `training()` / `evaluate()`.  2-D inputs are one utterance (the reference's
SGD mode, Recurrent.lua:67-77); 3-D inputs are a batch of equal-length utterances.
"""
import contextlib
import ctypes
import os
import math

import torch

from . import _lib
from ._lib import check, lib, ptr_array


# --------------------------------------------------------------------------- context / memory

class Context:
    """One s2s_ctx per device (s2s_ctx_create)."""

    def __init__(self, device: int = 0, graph: bool = False, overlap: bool = False):
        self.device = device
        h = ctypes.c_void_p()
        check(lib.s2s_ctx_create(device, ctypes.byref(h)))
        self.handle = h
        flags = (_lib.S2S_CTX_GRAPH if graph else 0) | (_lib.S2S_CTX_OVERLAP if overlap else 0)
        if flags:
            check(lib.s2s_ctx_set_flags(h, flags))

    def set_precision(self, precision: str):
        """"fp32" (default), "bf16" (forward / data-gradient GEMMs on bf16 operands, weight gradients fp32) or
        "bf16-all" (weight gradients too): operand precision of the hoisted GEMMs (s2s_ctx_set_precision)."""
        p = {"fp32": _lib.S2S_PREC_FP32, "bf16": _lib.S2S_PREC_BF16_GEMM, "bf16-all": _lib.S2S_PREC_BF16_ALL}[precision]
        check(lib.s2s_ctx_set_precision(self.handle, p))
        self.precision = precision

    def set_graph_cache(self, capacity: int):
        """How many captured steps (one per shape / buffer set) the context keeps (default 8)."""
        check(lib.s2s_ctx_set_graph_cache(self.handle, int(capacity)))

    def status(self, stream=None, clear=True):
        """Failure status of this context's persistent launches (s2s_ctx_status), after synchronising `stream`
        (default: the current stream): 0, or S2S_STATUS_HANDOFF_TIMEOUT | S2S_STATUS_ABORTED_REGION.  While it
        is nonzero every compute call of the context raises S2SError; clear=True resets it."""
        st = ctypes.c_void_p(stream.cuda_stream) if stream is not None else stream_ptr()
        if not hasattr(lib, "s2s_ctx_status"):  # an older A/B build (S2S_HIP_LIB) has no status words
            return 0
        v = ctypes.c_int()
        check(lib.s2s_ctx_status(self.handle, st, ctypes.byref(v), 1 if clear else 0))
        return v.value

    def check_status(self, stream=None):
        """Raise S2SError when a persistent launch of this context failed since the last check (and clear it)."""
        v = self.status(stream, clear=True)
        if v:
            raise _lib.S2SError(f"persistent launch failure (status {v}): the results since the last check are invalid")

    def graph_stats(self):
        """-> (graphs captured, replays launched, graphs cached) of this context."""
        c, r, n = ctypes.c_long(), ctypes.c_long(), ctypes.c_int()
        check(lib.s2s_ctx_graph_stats(self.handle, ctypes.byref(c), ctypes.byref(r), ctypes.byref(n)))
        return c.value, r.value, n.value

    def __del__(self):
        try:
            if self.handle:
                lib.s2s_ctx_destroy(self.handle)
        except Exception:
            pass


_CTX = {}


@contextlib.contextmanager
def precision(p: str, device=None):
    """with s2s_amd.precision("bf16"): the default context's hoisted GEMMs (front-end convolutions,
    x-projections, Vh, decoder MLP, weight-gradient / dX GEMMs) take bf16 operands with fp32
    accumulation inside the block (s2s_ctx_set_precision); "fp32" restores exact f32 MFMA."""
    ctx = get_context(device)
    prev = getattr(ctx, "precision", "fp32")
    ctx.set_precision(p)
    try:
        yield ctx
    finally:
        ctx.set_precision(prev)


@contextlib.contextmanager
def overlap_param_grads(device=None):
    """with s2s_amd.overlap_param_grads(): inside the block the module backward calls (Attention, the LSTM layers,
    TemporalConvolution) issue their parameter gradients on the context's side stream, beside the next module's
    backward (s2s_ctx_set_wgrad_overlap: Torch's accGradParameters made asynchronous); leaving the block joins them
    into the current stream, so from then on the gradients are final in its order.  The same kernels in the same
    order per gradient: the results are bitwise those of the serial calls."""
    ctx = get_context(device)
    if getattr(ctx, "_wgrad_side", None) is not None:  # nested: the outer block joins
        yield ctx
        return
    side = getattr(ctx, "_side_stream", None)
    if side is None:
        side = ctx._side_stream = torch.cuda.ExternalStream(lib.s2s_ctx_side_stream(ctx.handle),
                                                            device=torch.device("cuda", ctx.device))
    check(lib.s2s_ctx_set_wgrad_overlap(ctx.handle, 1))
    ctx._wgrad_side = side
    try:
        yield ctx
    finally:
        ctx._wgrad_side = None
        check(lib.s2s_ctx_set_wgrad_overlap(ctx.handle, 0))
        check(lib.s2s_ctx_join_wgrad(ctx.handle, stream_ptr()))


@contextlib.contextmanager
def serial_param_grads(device=None):
    """Inside overlap_param_grads: the block's parameter gradients stay on the call's stream (small products the
    side stream would only queue behind a persistent launch that holds every CU)."""
    ctx = _CTX.get(device)
    side = getattr(ctx, "_wgrad_side", None) if ctx is not None else None
    if side is None:
        yield
        return
    check(lib.s2s_ctx_set_wgrad_overlap(ctx.handle, 0))
    ctx._wgrad_side = None
    try:
        yield
    finally:
        check(lib.s2s_ctx_set_wgrad_overlap(ctx.handle, 1))
        ctx._wgrad_side = side


def side_uses(device, *tensors):
    """Inside overlap_param_grads: the side stream reads these buffers after the call returns -- keep the caching
    allocator from handing them out again before it has (record_stream; under graph capture the free is deferred to
    the capture's end)."""
    ctx = _CTX.get(device.index)
    side = getattr(ctx, "_wgrad_side", None) if ctx is not None else None
    if side is not None:
        for t in tensors:
            if t is not None:
                t.record_stream(side)


def get_context(device=None) -> Context:
    dev = torch.cuda.current_device() if device is None else int(device)
    if dev not in _CTX:
        _CTX[dev] = Context(dev)
    return _CTX[dev]


def stream_ptr():
    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def dptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


_POISON = os.environ.get("S2S_POISON_SCRATCH") == "1"  # diagnostic: fill every scratch / saved buffer with NaN


def _bytes(n, device):
    t = torch.empty(max(int(n), 1), dtype=torch.uint8, device=device)
    if _POISON:
        t.fill_(0xFF)  # all-ones words: NaN in every float view -- a read before write shows up in the outputs
    return t


def _require_cuda_f32(t, name):
    if not (t.is_cuda and t.dtype == torch.float32 and t.is_contiguous()):
        raise S2SArgumentError(f"{name} must be a contiguous float32 CUDA tensor")


class S2SArgumentError(ValueError):
    pass


def lengths_tensor(lengths, n, maxlen, device):
    """(n,) int32 device tensor of per-utterance lengths, each in [1, maxlen] (checked on the host: the
    kernels trust them)."""
    t = torch.as_tensor(lengths).to(torch.int64).reshape(-1)
    if t.numel() != n:
        raise S2SArgumentError(f"lengths: {t.numel()} values for {n} utterances")
    tc = t.cpu()
    if int(tc.min()) < 1 or int(tc.max()) > maxlen:
        raise S2SArgumentError(f"lengths must be in [1, {maxlen}]")
    return tc.to(torch.int32).to(device)


def _uniform(shape, stdv, gen=None):
    return (torch.rand(shape, generator=gen, dtype=torch.float64) * 2 - 1).mul_(stdv).float()


class Module:
    def __init__(self):
        self.output = None
        self.gradInput = None
        self.train = True

    def parameters(self):
        return [], []

    def zeroGradParameters(self):
        gs = [g for g in self.parameters()[1] if g is not None]
        if gs:
            torch._foreach_zero_(gs)  # one multi-tensor launch (a model has 30-60 gradient tensors)

    def forward(self, input):
        return self.updateOutput(input)

    def backward(self, input, gradOutput, scale=1.0):
        self.updateGradInput(input, gradOutput, scale)
        return self.gradInput

    def training(self):
        self.train = True

    def evaluate(self):
        self.train = False

    def _check_params(self, x):
        """every parameter / gradient buffer must be a contiguous float32 tensor on x's device: the kernels take
        raw device pointers, and a host tensor's pointer would fault on the GPU (call .cuda() first)"""
        ws, gs = self.parameters()
        for i, t in enumerate(ws + gs):
            if t is None:
                continue
            if not (t.is_cuda and t.device == x.device and t.dtype == torch.float32 and t.is_contiguous()):
                raise S2SArgumentError(f"{type(self).__name__}: parameter {i} must be a contiguous float32 tensor on "
                                       f"{x.device} (is {t.device}, {t.dtype}); call .cuda() first")

    def cuda(self, device=None):
        dev = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        ws, gs = self.parameters()
        for t in ws + gs:
            t.data = t.data.to(dev)
        return self


# --------------------------------------------------------------------------- GRU / RNN

class GRU(Module):
    """nn.GRU(diminput, dimoutput) cell parameters (GRU.lua:8-43): three LinearZeroBias
    (dimoutput, diminput+dimoutput) for z, r, h, columns [h | x]; reset U(+-1/sqrt(in))
    (LinearZeroBias.lua:12-29).  The cell runs inside RNN / Attention sequence kernels."""

    def __init__(self, diminput, dimoutput, generator=None):
        super().__init__()
        assert diminput is not None, "diminput must be specified"
        assert dimoutput is not None, "dimoutput must be specified"
        self.diminput, self.dimoutput = diminput, dimoutput
        stdv = 1.0 / math.sqrt(diminput + dimoutput)
        self.weight = [_uniform((dimoutput, diminput + dimoutput), stdv, generator) for _ in range(3)]
        self.gradWeight = [torch.zeros_like(w) for w in self.weight]

    def parameters(self):
        return list(self.weight), list(self.gradWeight)


class LSTM(Module):
    """nn.LSTM(inputSize, outputSize, peepholes) cell parameters (LSTM.lua:6-60): for each gate
    q in (i, f, g, o) a Linear(D, H) on x and a Linear(H, H) on h (both with bias); peepholes add
    Linear(H, H) on the cell for i, f (previous cell) and o (new cell).  nn.Linear reset:
    U(+-1/sqrt(in)) for weight and bias.  Flat order = the C ABI's (include/s2s_hip.h)."""

    GATES = ("i", "f", "g", "o")

    def __init__(self, inputSize, outputSize, peepholes=False, generator=None):
        super().__init__()
        self.diminput, self.dimoutput, self.peepholes = inputSize, outputSize, bool(peepholes)
        D, H = inputSize, outputSize
        sx, sh = 1.0 / math.sqrt(D), 1.0 / math.sqrt(H)
        self.names, self.weight = [], []
        for q in self.GATES:
            for name, shape, sd in ((f"W{q}x", (H, D), sx), (f"b{q}x", (H,), sx), (f"W{q}h", (H, H), sh),
                                    (f"b{q}h", (H,), sh)):
                self.names.append(name)
                self.weight.append(_uniform(shape, sd, generator))
        if self.peepholes:
            for q in ("i", "f", "o"):
                for name, shape in ((f"W{q}c", (H, H)), (f"b{q}c", (H,))):
                    self.names.append(name)
                    self.weight.append(_uniform(shape, sh, generator))
        self.gradWeight = [torch.zeros_like(w) for w in self.weight]

    def parameters(self):
        return list(self.weight), list(self.gradWeight)

    def named(self, grads=False):
        return dict(zip(self.names, self.gradWeight if grads else self.weight))


class _GruSeq(Module):
    """Shared driver of s2s_{gru,lstm}_{fwd,bwd} for 1 or 2 directions over the same input (all
    cells GRU, or all LSTM with the same peephole setting)."""

    def __init__(self, cells, reverses):
        super().__init__()
        self.cells = cells
        self.reverses = reverses
        self.dimoutput = cells[0].dimoutput
        self.lstm = isinstance(cells[0], LSTM)
        self.peep = int(self.lstm and cells[0].peepholes)
        for c in cells:
            if c.dimoutput % 16 != 0:
                raise S2SArgumentError("recurrent dimoutput must be a multiple of 16 on this path")
            if isinstance(c, LSTM) != self.lstm or (self.lstm and int(c.peepholes) != self.peep):
                raise S2SArgumentError("all directions must use the same cell type")

    def parameters(self):
        ws, gs = [], []
        for c in self.cells:
            w, g = c.parameters()
            ws += w
            gs += g
        return ws, gs

    def _shape(self, input):
        if input.dim() == 2:
            return 1, input.shape[0], input.shape[1]
        if input.dim() == 3:
            return input.shape
        raise S2SArgumentError("input dimension must be 2D or 3D")  # RNN.lua:128

    # variable-length batch: (B,) frames per utterance (the reference forwards each utterance alone,
    # timit/timit.lua:239-240); None = every utterance has all L frames
    lengths = None

    def _lengths_ptr(self, B, L, dev):
        if self.lengths is None:
            return ctypes.c_void_p(0)
        self._len_dev = lengths_tensor(self.lengths, B, L, dev)
        return dptr(self._len_dev)

    def updateOutput(self, input):
        _require_cuda_f32(input, "input")
        self._check_params(input)
        B, L, D = self._shape(input)
        H, nd = self.dimoutput, len(self.cells)
        if D != self.cells[0].diminput:
            raise S2SArgumentError(f"input frame size {D} != diminput {self.cells[0].diminput}")
        dev = input.device
        out = torch.empty((B, L, nd * H), device=dev, dtype=torch.float32)
        W = ptr_array([w.data_ptr() for c in self.cells for w in c.weight])
        y = ptr_array([out.data_ptr() + 4 * H * d for d in range(nd)])
        rev = ptr_array([int(r) for r in self.reverses], ctypes.c_int)
        ctx = get_context(dev.index).handle
        if self.lstm:
            self._saved = [_bytes(lib.s2s_lstm_saved_bytes(B, L, H), dev) for _ in range(nd)]
            scr = _bytes(lib.s2s_lstm_scratch_bytes(nd, B, L, D, H, self.peep), dev)
            sv = ptr_array([s.data_ptr() for s in self._saved])
            check(lib.s2s_lstm_fwd(ctx, stream_ptr(), nd, B, L, D, H, self.peep, rev, dptr(input), D, W, y, nd * H, sv,
                                   self._lengths_ptr(B, L, dev), dptr(scr), scr.numel()))
        else:
            self._saved = [_bytes(lib.s2s_gru_saved_bytes(B, L, H), dev) for _ in range(nd)]
            scr = _bytes(lib.s2s_gru_scratch_bytes(nd, B, L, D, H), dev)
            sv = ptr_array([s.data_ptr() for s in self._saved])
            check(lib.s2s_gru_fwd(ctx, stream_ptr(), nd, B, L, D, H, rev, dptr(input), D, W, y, nd * H, sv,
                                  self._lengths_ptr(B, L, dev), dptr(scr), scr.numel()))
        self._dims = (B, L, D)
        self.output = out if input.dim() == 3 else out[0]
        return self.output

    def updateGradInput(self, input, gradOutput, scale=1.0):
        B, L, D = self._dims
        H, nd = self.dimoutput, len(self.cells)
        dev = input.device
        go = gradOutput.contiguous()
        dx = torch.empty((B, L, D), device=dev, dtype=torch.float32)
        W = ptr_array([w.data_ptr() for c in self.cells for w in c.weight])
        dW = ptr_array([g.data_ptr() for c in self.cells for g in c.gradWeight])
        dy = ptr_array([go.data_ptr() + 4 * H * d for d in range(nd)])
        sv = ptr_array([s.data_ptr() for s in self._saved])
        rev = ptr_array([int(r) for r in self.reverses], ctypes.c_int)
        ctx = get_context(dev.index).handle
        if self.lstm:
            scr = _bytes(lib.s2s_lstm_scratch_bytes(nd, B, L, D, H, self.peep), dev)
            check(lib.s2s_lstm_bwd(ctx, stream_ptr(), nd, B, L, D, H, self.peep, rev, dptr(input), D, W, sv, dy, nd * H,
                                   dptr(dx), D, 0, dW, float(scale), self._lengths_ptr(B, L, dev), dptr(scr),
                                   scr.numel()))
            side_uses(dev, scr)
        else:
            scr = _bytes(lib.s2s_gru_scratch_bytes(nd, B, L, D, H), dev)
            check(lib.s2s_gru_bwd(ctx, stream_ptr(), nd, B, L, D, H, rev, dptr(input), D, W, sv, dy, nd * H, dptr(dx),
                                  D, 0, dW, float(scale), self._lengths_ptr(B, L, dev), dptr(scr), scr.numel()))
        self.gradInput = dx if input.dim() == 3 else dx[0]
        return self.gradInput

    def accGradParameters(self, input, gradOutput, scale=1.0):
        pass  # accumulated inside updateGradInput, as Recurrent's inner gModule:backward does


class RNN(_GruSeq):
    """nn.RNN(recurrent, reverse) (RNN.lua:3-201) over an nn.GRU or nn.LSTM cell."""

    def __init__(self, recurrent, reverse=False):
        assert recurrent is not None, "recurrent cannot be nil"
        assert getattr(recurrent, "dimoutput", None) is not None, "recurrent must specify dimoutput"
        if not isinstance(recurrent, (GRU, LSTM)):
            raise S2SArgumentError("this path runs nn.GRU and nn.LSTM cells")
        super().__init__([recurrent], [bool(reverse)])
        self.recurrent = recurrent
        self.reverse = bool(reverse)


class BiRNN(_GruSeq):
    """JoinTable(2,2)({RNN(cell, false)(x), RNN(cell, true)(x)}) -- one bidirectional encoder layer
    (timit/model_chorowski_baseline.lua:22-24; BiLSTM: timit/timit.lua:108-125) with both
    directions in the same launches."""

    def __init__(self, fwd_cell, bwd_cell):
        super().__init__([fwd_cell, bwd_cell], [False, True])


# --------------------------------------------------------------------------- Attention decoder

class MaxoutMLP(Module):
    """decoder_mlp of timit/model_chorowski_baseline.lua:53-59:
    [Dropout(p) ->] Maxout(inDim, mlpDepth, window) -> Linear(mlpDepth, outputDepth) -> LogSoftMax.
    Maxout = Linear(in, out*window) + TemporalMaxPooling(window, window) over consecutive groups
    (Maxout.lua:14-18); dropout > 0 is timit/model_chorowski_baseline_dropout.lua:56 (Torch7
    nn.Dropout: training mode scales kept inputs by 1/(1-p), evaluate() is the identity)."""

    def __init__(self, inputDimension, mlpDepth, window, outputDepth, generator=None, dropout=0.0):
        super().__init__()
        self.inputDim, self.mlpDepth, self.window, self.outputDepth = inputDimension, mlpDepth, window, outputDepth
        if not 0.0 <= dropout < 1.0:
            raise S2SArgumentError("dropout must be in [0, 1)")
        self.dropout = float(dropout)
        s1 = 1.0 / math.sqrt(inputDimension)
        s2 = 1.0 / math.sqrt(mlpDepth)
        self.weight = [_uniform((mlpDepth * window, inputDimension), s1, generator),
                       _uniform((mlpDepth * window,), s1, generator),
                       _uniform((outputDepth, mlpDepth), s2, generator),
                       _uniform((outputDepth,), s2, generator)]
        self.gradWeight = [torch.zeros_like(w) for w in self.weight]

    def parameters(self):
        return list(self.weight), list(self.gradWeight)


class Attention(Module):
    """nn.Attention (Attention.lua:15-211) for the Chorowski decoder: decoder_recurrent = GRU(S,S)
    (model_chorowski_baseline.lua:48-51), decoder_mlp = MaxoutMLP.  Input {h, y}: h (L, A) or
    (B, L, A) annotations, y the (T, O)/(B, T, O) labelmask or (B, T) int labels."""

    PARAM_NAMES = ("V", "Ws", "bs", "we", "Wy", "by", "Wc", "bc", "Wd", "bd", "Wz", "Wr", "Wh", "Wm", "bm", "Wo",
                   "bo")

    def __init__(self, decoder_recurrent, decoder_mlp, scoreDepth, hybridAttendFilterSize, hybridAttendFeatureMaps,
                 stateDepth, annotationDepth, outputDepth, monoAlignPenalty=False, penaltyLambda=0.0,
                 generator=None):
        super().__init__()
        nF = int(hybridAttendFeatureMaps or 0)
        if nF > 0 and not 1 <= int(hybridAttendFilterSize or 0) <= 8:
            raise S2SArgumentError("hybridAttendFilterSize must be in [1, 8] with hybrid attention")
        # decoder_recurrent: GRU(S, S) (the Chorowski models) or LSTM(S, S) without peepholes (the conv +
        # BiLSTM model, timit/timit.lua:137; per-step decoder kernels)
        self.decoder_lstm = isinstance(decoder_recurrent, LSTM)
        if self.decoder_lstm:
            if decoder_recurrent.peepholes or decoder_recurrent.diminput != stateDepth or \
                    decoder_recurrent.dimoutput != stateDepth:
                raise S2SArgumentError("decoder_recurrent LSTM must be LSTM(stateDepth, stateDepth) without peepholes")
        elif not isinstance(decoder_recurrent, GRU) or decoder_recurrent.dimoutput != stateDepth:
            raise S2SArgumentError("decoder_recurrent must be GRU(stateDepth, stateDepth) or LSTM(stateDepth, stateDepth)")
        # MaxoutMLP (Maxout -> Linear -> LogSoftMax, model_chorowski_baseline.lua:53-59) runs fused in the
        # decoder launches; any other decoder_mlp module (e.g. the two-Maxout MLP of librispeech/
        # model_vgg.lua:71-77, built from s2s_amd.frontend) runs outside on the saved [s_t; c_t] rows
        self.external_mlp = not isinstance(decoder_mlp, MaxoutMLP)
        if not self.external_mlp and decoder_mlp.inputDim != stateDepth + annotationDepth:
            raise S2SArgumentError("decoder_mlp must be MaxoutMLP(stateDepth + annotationDepth, ...)")
        if self.external_mlp and not (hasattr(decoder_mlp, "forward") and hasattr(decoder_mlp, "backward")):
            raise S2SArgumentError("decoder_mlp must be an nn.Module mirror")
        self.scoreDepth, self.stateDepth, self.annotationDepth, self.outputDepth = (scoreDepth, stateDepth,
                                                                                    annotationDepth, outputDepth)
        self.hybridAttendFilterSize, self.hybridAttendFeatureMaps = hybridAttendFilterSize, hybridAttendFeatureMaps
        self.MonotonicAlignmentPenalty = bool(monoAlignPenalty)
        self.penalty = float(penaltyLambda or 0.0) if monoAlignPenalty else 0.0
        self.decoder_recurrent, self.decoder_mlp = decoder_recurrent, decoder_mlp
        Sc, S, A, O = scoreDepth, stateDepth, annotationDepth, outputDepth
        g = generator
        own = {"V": _uniform((Sc, A), 1 / math.sqrt(A), g),            # TCZB(A, Sc, 1)
               "Ws": _uniform((Sc, S), 1 / math.sqrt(S), g),           # TemporalConvolution(1, Sc, S)
               "bs": _uniform((Sc,), 1 / math.sqrt(S), g),
               "we": _uniform((1, Sc), 1 / math.sqrt(Sc), g),          # TCZB(Sc, 1, 1)
               "Wy": _uniform((S, O), 1 / math.sqrt(O), g), "by": _uniform((S,), 1 / math.sqrt(O), g),
               "Wc": _uniform((S, A), 1 / math.sqrt(A), g), "bc": _uniform((S,), 1 / math.sqrt(A), g),
               "Wd": _uniform((S, 2 * S), 1 / math.sqrt(2 * S), g), "bd": _uniform((S,), 1 / math.sqrt(2 * S), g)}
        if nF > 0:  # Attention.lua:90-91: TemporalConvolution(1, nF, kW) + TCZB(nF, Sc, 1)
            kW = int(hybridAttendFilterSize)
            own.update({"hybW": _uniform((nF, kW), 1 / math.sqrt(kW), g), "hybb": _uniform((nF,), 1 / math.sqrt(kW), g),
                        "hybU": _uniform((Sc, nF), 1 / math.sqrt(nF), g)})
        self.own = own
        self.own_grad = {k: torch.zeros_like(v) for k, v in own.items()}
        # scoreDepth not a multiple of 16 (the conv model's 150, timit/timit.lua:128): the kernels run on
        # score channels zero-padded to the next multiple of 16 -- padded rows of V / Ws / hybU, bs and
        # columns of we are zero, so each padded channel adds we_j tanh(0) = 0 to every score (exact)
        self._scp = (scoreDepth + 15) // 16 * 16
        self._pad = None

    _PADDED = {"V": 0, "Ws": 0, "bs": 0, "we": 1, "hybU": 0}  # parameter -> score-channel axis

    def _pad_bound(self):
        return self._pad is not None and all(
            self.own[n].data_ptr() == t.data_ptr() and self.own_grad[n].data_ptr() == self._pad[1][n].data_ptr()
            for n, t in self._pad[0].items())

    def _sync_pad(self, grads_zero=False):
        """The kernels read score channels zero-padded to a multiple of 16 (scoreDepth % 16 != 0).  The padded tensors
        are the parameters' and gradients' own storage -- own[n] / own_grad[n] are narrow views of them, rebound here
        whenever a parameter's storage was replaced (cuda(), a checkpoint load) -- so a step copies nothing (it used to
        copy five parameters in and add five gradients back: ~20 launches a step).  The padded rows stay zero: a padded
        channel has we_j = 0, so the kernels' gradients there are 0 too.  (grads_zero: kept for the call sites.)"""
        if self._scp == self.scoreDepth or self._pad_bound():
            return
        Sc = self.scoreDepth
        mk, gk = {}, {}
        with torch.no_grad():
            for n, ax in self._PADDED.items():
                if n not in self.own:
                    continue
                shp = list(self.own[n].shape)
                shp[ax] = self._scp
                dev = self.own[n].device
                p = torch.zeros(shp, dtype=torch.float32, device=dev)
                g = torch.zeros(shp, dtype=torch.float32, device=dev)
                p.narrow(ax, 0, Sc).copy_(self.own[n])
                g.narrow(ax, 0, Sc).copy_(self.own_grad[n])
                self.own[n].data = p.narrow(ax, 0, Sc)
                self.own_grad[n].data = g.narrow(ax, 0, Sc)
                mk[n], gk[n] = p, g
        self._pad = (mk, gk)

    def _unpad_grads(self):
        pass  # (the kernels accumulate into the gradients' padded storage directly, _sync_pad)

    def _tensors(self, grads=False, kernel=False):
        o = self.own_grad if grads else self.own
        if kernel and self._scp != self.scoreDepth:
            o = dict(o)
            o.update(self._pad[1] if grads else self._pad[0])
        r = self.decoder_recurrent.gradWeight if grads else self.decoder_recurrent.weight
        lstm_w = None
        if self.decoder_lstm:  # params 10-12 unused; the LSTM's 16 at 20-35 (S2S_ATTN_NPARAMS_LSTM)
            lstm_w, r = list(r), [None] * 3
        if self.external_mlp:
            m = [None] * 4  # params 13-16 unused with an external decoder_mlp
        else:
            m = self.decoder_mlp.gradWeight if grads else self.decoder_mlp.weight
        out = [o["V"], o["Ws"], o["bs"], o["we"], o["Wy"], o["by"], o["Wc"], o["bc"], o["Wd"], o["bd"],
               r[0], r[1], r[2], m[0], m[1], m[2], m[3]]
        if "hybW" in o:
            out += [o["hybW"], o["hybb"], o["hybU"]]
        elif lstm_w is not None:
            out += [None] * 3
        if lstm_w is not None:
            out += lstm_w
        return out

    def parameters(self):
        ws, gs = [t for t in self._tensors(False) if t is not None], [t for t in self._tensors(True) if t is not None]
        if self.external_mlp:
            w2, g2 = self.decoder_mlp.parameters()
            ws, gs = ws + list(w2), gs + list(g2)
        return ws, gs

    def _ptrs(self, grads=False):
        return ptr_array([t.data_ptr() if t is not None else 0 for t in self._tensors(grads, kernel=True)])

    # dropout: injected (B, T, S+A) multipliers for the next forward (parity with an external RNG),
    # else drawn in-kernel from dropout_seed + the forward count
    dropout_mask = None
    dropout_seed = 0x5eed
    # variable-length batch: (B,) frames of h and labels per utterance (None = all L / T)
    frame_lengths = None
    label_lengths = None

    def _set_lengths(self, d, B, L, T, dev):
        self._len_keep = []
        if self.frame_lengths is not None:
            t = lengths_tensor(self.frame_lengths, B, L, dev)
            self._len_keep.append(t)
            d.frame_lengths = t.data_ptr()
        if self.label_lengths is not None:
            t = lengths_tensor(self.label_lengths, B, T, dev)
            self._len_keep.append(t)
            d.label_lengths = t.data_ptr()

    def _dims(self, h, T):
        B, L = (1, h.shape[0]) if h.dim() == 2 else (h.shape[0], h.shape[1])
        m = self.decoder_mlp
        if self.external_mlp:
            d = _lib.s2s_attn_dims(B, L, T, self.annotationDepth, self._scp, self.stateDepth, self.outputDepth,
                                   1, 1, self.penalty, 0.0)
            d.external_mlp = 1
            d.decoder_lstm = int(self.decoder_lstm)
            if self.hybridAttendFeatureMaps and self.hybridAttendFeatureMaps > 0:
                d.hybridAttendFilterSize = int(self.hybridAttendFilterSize)
                d.hybridAttendFeatureMaps = int(self.hybridAttendFeatureMaps)
            self._set_lengths(d, B, L, T, h.device)
            return d
        p = m.dropout if (m.dropout > 0 and self.train) else 0.0
        d = _lib.s2s_attn_dims(B, L, T, self.annotationDepth, self._scp, self.stateDepth, self.outputDepth,
                               m.mlpDepth, m.window, self.penalty, p)
        d.decoder_lstm = int(self.decoder_lstm)
        if self.hybridAttendFeatureMaps and self.hybridAttendFeatureMaps > 0:
            d.hybridAttendFilterSize = int(self.hybridAttendFilterSize)
            d.hybridAttendFeatureMaps = int(self.hybridAttendFeatureMaps)
        self._set_lengths(d, B, L, T, h.device)
        if p > 0:
            self._fwd_count = getattr(self, "_fwd_count", 0) + 1
            d.dropout_seed = (self.dropout_seed * 1000003 + self._fwd_count) & ((1 << 64) - 1)
            if self.dropout_mask is not None:
                msk = self.dropout_mask
                if msk.shape != (B, T, self.stateDepth + self.annotationDepth) or msk.dtype != torch.float32:
                    raise S2SArgumentError("dropout_mask must be float32 (B, T, stateDepth + annotationDepth)")
                self._mask_keep = msk.contiguous()
                d.dropout_mask = self._mask_keep.data_ptr()
        return d

    def dropout_mask_used(self):
        """(B, T, S+A) dropout multipliers of the last forward (inside the saved buffer)."""
        d = self._d
        if d.dropout <= 0:
            return None
        p = lib.s2s_attn_dropout_mask(ctypes.byref(d), dptr(self._saved))
        off = p - self._saved.data_ptr()
        n = d.B * d.T * (self.stateDepth + self.annotationDepth)
        return self._saved[off:off + 4 * n].view(torch.float32).view(d.B, d.T, -1)

    @staticmethod
    def labels_from(y, O):
        if y.dtype in (torch.int32, torch.int64):
            return y.to(torch.int32).contiguous()
        # labelmask: one-hot rows (timit/timit.lua:262)
        return y.argmax(-1).to(torch.int32).contiguous()

    def updateOutput(self, input):
        h, y = input
        if h.dim() not in (2, 3):
            raise S2SArgumentError("x must be 2d or 3d")  # Attention.lua:316
        _require_cuda_f32(h, "h")
        self._check_params(h)
        lab = self.labels_from(y, self.outputDepth)
        if lab.dim() == 1:
            lab = lab[None]
        T = lab.shape[1]
        d = self._dims(h, T)
        dev = h.device
        self._d = d
        self._sync_pad()
        self._labels = lab
        self._saved = _bytes(lib.s2s_attn_saved_bytes(ctypes.byref(d)), dev)
        scr = _bytes(lib.s2s_attn_scratch_bytes(ctypes.byref(d)), dev)
        out = None if self.external_mlp else torch.empty((d.B, T, self.outputDepth), device=dev, dtype=torch.float32)
        check(lib.s2s_attn_fwd(get_context(dev.index).handle, stream_ptr(), ctypes.byref(d), dptr(h), dptr(lab),
                               self._ptrs(False), dptr(out), dptr(self._saved), dptr(scr), scr.numel()))
        if self.external_mlp:  # decoder_mlp over all B*T rows of [s_t; c_t] (RNNAttention.lua:165)
            self._mlp_in = self.mlp_input().reshape(d.B * T, -1)
            out = self.decoder_mlp.forward(self._mlp_in).reshape(d.B, T, -1)
        self.output = out if h.dim() == 3 else out[0]
        return self.output

    def mlp_input(self):
        """(B, T, S+A) decoder_mlp input rows [s_t; c_t] of the last forward (inside the saved buffer)."""
        d = self._d
        p = lib.s2s_attn_mlp_input(ctypes.byref(d), dptr(self._saved))
        off = p - self._saved.data_ptr()
        n = d.B * d.T * (self.stateDepth + self.annotationDepth)
        return self._saved[off:off + 4 * n].view(torch.float32).view(d.B, d.T, -1)

    def updateGradInput(self, input, gradOutput, scale=1.0):
        h, _ = input
        d = self._d
        dev = h.device
        go = gradOutput.contiguous()
        if go.dim() == 2:
            go = go[None]
        dh = torch.empty((d.B, d.L, self.annotationDepth), device=dev, dtype=torch.float32)
        scr = _bytes(lib.s2s_attn_scratch_bytes(ctypes.byref(d)), dev)
        if self.external_mlp:  # d[s_t; c_t] from the decoder_mlp backward replaces dlogp
            with serial_param_grads(dev.index):  # (ahead of the decoder launch, which holds every CU)
                go = self.decoder_mlp.backward(self._mlp_in, go.reshape(d.B * d.T, -1), scale)
            go = go.reshape(d.B, d.T, -1).contiguous()
        self._sync_pad(grads_zero=True)
        check(lib.s2s_attn_bwd(get_context(dev.index).handle, stream_ptr(), ctypes.byref(d), dptr(h),
                               dptr(self._labels), self._ptrs(False), dptr(self._saved), dptr(go), dptr(dh), 0,
                               self._ptrs(True), float(scale), dptr(scr), scr.numel()))
        side_uses(dev, scr)
        self._unpad_grads()
        self.gradInput = [dh if h.dim() == 3 else dh[0], None]
        return self.gradInput

    def accGradParameters(self, input, gradOutput, scale=1.0):
        pass

    def BeamSearch(self, annotations, eos, K=5, maxseqlength=None):
        """decoder:BeamSearch(annotations, eos, K, maxseqlength) (Attention.lua:332-438) in evaluate()
        mode.  annotations (L, A) -> 1-D int tensor (the prediction, 0-based tokens, eos last when it
        finished on eos); (B, L, A) -> (tokens (B, maxseqlength + 1) padded with -1, lengths (B),
        scores (B)).  maxseqlength defaults to L (:337).  Content or hybrid attention, GRU or LSTM
        decoder_recurrent; an external decoder_mlp runs between the search's step and advance calls on
        the (B*K, S+A) hypothesis rows."""
        h = annotations
        if h.dim() not in (2, 3):
            raise S2SArgumentError("annotations must be 2d or 3d")
        _require_cuda_f32(h, "annotations")
        single = h.dim() == 2
        if single:
            h = h[None]
        h = h.contiguous()
        B, L = h.shape[0], h.shape[1]
        maxlen = int(maxseqlength or L)
        was_train, self.train = self.train, False
        d = self._dims(h, 1)
        self.train = was_train
        d.frame_lengths = d.label_lengths = None  # the utterances' whole annotation sequences are searched
        dev = h.device
        self._sync_pad()
        ws = _bytes(lib.s2s_attn_beam_workspace_bytes(ctypes.byref(d), K, maxlen), dev)
        out = torch.empty((B, maxlen + 1), dtype=torch.int32, device=dev)
        olen = torch.empty(B, dtype=torch.int32, device=dev)
        osc = torch.empty(B, dtype=torch.float32, device=dev)
        params = self._ptrs(False)
        ctx, st = get_context(dev.index).handle, stream_ptr()
        if not self.external_mlp:
            check(lib.s2s_attn_beam_search(ctx, st, ctypes.byref(d), dptr(h), params, int(eos), int(K), maxlen,
                                           dptr(out), maxlen + 1, dptr(olen), dptr(osc), dptr(ws), ws.numel()))
        else:
            R, W = B * int(K), self.stateDepth + self.annotationDepth
            p = lib.s2s_attn_beam_mlp_input(ctypes.byref(d), int(K), maxlen, dptr(ws))
            off = p - ws.data_ptr()
            rows = ws[off:off + 4 * R * W].view(torch.float32).view(R, W)
            mlp_train = getattr(self.decoder_mlp, "train", None)
            if mlp_train is not None:
                self.decoder_mlp.train = False
            done = ctypes.c_int(0)
            try:
                check(lib.s2s_attn_beam_init(ctx, st, ctypes.byref(d), dptr(h), params, int(eos), int(K), maxlen,
                                             dptr(ws), ws.numel()))
                for count in range(maxlen + 1):
                    check(lib.s2s_attn_beam_step(ctx, st, ctypes.byref(d), params, int(K), maxlen, count, dptr(ws),
                                                 ws.numel()))
                    logp = self.decoder_mlp.forward(rows).contiguous()
                    if logp.shape != (R, self.outputDepth) or logp.dtype != torch.float32:
                        raise S2SArgumentError("decoder_mlp must map (B*K, S+A) rows to (B*K, outputDepth) fp32")
                    check(lib.s2s_attn_beam_advance(ctx, st, ctypes.byref(d), int(eos), int(K), maxlen, count,
                                                    dptr(logp), dptr(ws), ws.numel()))
                    if (count & 3) == 3 or count == maxlen:
                        check(lib.s2s_attn_beam_done(ctx, st, ctypes.byref(d), int(K), maxlen, dptr(ws),
                                                     ctypes.byref(done)))
                        if done.value:
                            break
                check(lib.s2s_attn_beam_finish(ctx, st, ctypes.byref(d), int(K), maxlen, dptr(out), maxlen + 1,
                                               dptr(olen), dptr(osc), dptr(ws)))
            finally:
                if mlp_train is not None:
                    self.decoder_mlp.train = mlp_train
        if single:
            return out[0, :int(olen[0].item())]
        return out, olen, osc

    def mono_ind(self):
        """(B, T) MonotonicAlignment indicators 1[penalty_t > 0] of the last forward
        (MonotonicAlignment.lua:27-39): the discrete decision its backward (:44-77) depends on."""
        d = self._d
        p = lib.s2s_attn_mono_ind(ctypes.byref(d), dptr(self._saved))
        off = p - self._saved.data_ptr()
        n = d.B * d.T
        return self._saved[off:off + 4 * n].view(torch.float32).view(d.B, d.T)

    def maxout_argmax(self):
        """(B, T, mlpDepth) int32: which unit of each Maxout group won in the last forward (first maximum,
        Maxout.lua:14-18) -- the discrete decision its backward routes each gradient row by."""
        d = self._d
        return saved_view(self._saved, lib.s2s_attn_maxout_argmax(ctypes.byref(d), dptr(self._saved)),
                          (d.B, d.T, d.mlpDepth), torch.int32)

    def alpha(self):
        """Attention:alpha() (Attention.lua:241-243): (B, T, L) attention weights of the last forward."""
        d = self._d
        return saved_view(self._saved, lib.s2s_attn_alpha(ctypes.byref(d), dptr(self._saved)), (d.B, d.T, d.L))

    def penalty(self):
        """Attention:penalty() (Attention.lua:244-246): the output of the graph node named 'penalty', i.e.
        MonotonicAlignment's output, which is alpha itself (MonotonicAlignment.lua:40) -- (B, T, L)."""
        return self.alpha()

    def Ws(self):
        """Attention:Ws() (Attention.lua:247-249): the 'Ws' node ExpandAs(ws_t, Vh) -- the rows
        ws_t = W_s s_{t-1} + b_s broadcast over the L frames, (B, T, L, scoreDepth) (an expand view of the
        saved (B, T, scoreDepth) rows, no copy)."""
        d = self._d
        ws = saved_view(self._saved, lib.s2s_attn_ws(ctypes.byref(d), dptr(self._saved)), (d.B, d.T, d.scoreDepth))
        ws = ws[..., :self.scoreDepth]
        return ws[:, :, None, :].expand(d.B, d.T, d.L, self.scoreDepth)

    @property
    def Vh_output(self):
        """decoder.Vh.output (Attention.lua:43-47, timit/timit.lua:521): Vh = h V^T, (B, L, scoreDepth)."""
        d = self._d
        vh = saved_view(self._saved, lib.s2s_attn_vh(ctypes.byref(d), dptr(self._saved)), (d.B, d.L, d.scoreDepth))
        return vh[..., :self.scoreDepth]


def saved_view(buf, p, shape, dtype=torch.float32):
    """`dtype` (4-byte) view of `shape` at device address p inside the byte buffer `buf`."""
    if not p:
        raise S2SArgumentError("no such tensor in the saved buffer")
    off = p - buf.data_ptr()
    n = math.prod(shape)
    if off < 0 or off + 4 * n > buf.numel():
        raise S2SArgumentError("saved-buffer view out of range")
    return buf[off:off + 4 * n].view(dtype).view(*shape)


def nll_seed(logp, labels, normalize=False, label_lengths=None):
    """timit/timit.lua:262-282: per-utterance nll and dlogp = -labelmask (label_lengths: (B,) labels per
    utterance of a variable-length batch; steps past them carry no loss and dlogp = 0)."""
    B, T, O = logp.shape
    lab = labels.to(torch.int32).contiguous()
    nll = torch.empty(B, device=logp.device, dtype=torch.float32)
    dlogp = torch.empty_like(logp)
    tl = lengths_tensor(label_lengths, B, T, logp.device) if label_lengths is not None else None
    check(lib.s2s_nll_seed(get_context(logp.device.index).handle, stream_ptr(), B, T, O, dptr(logp), dptr(lab),
                           dptr(tl), int(normalize), dptr(nll), dptr(dlogp)))
    return nll, dlogp


def edit_distance(a, alen, b, blen):
    """WagnerFischer (utils.lua:3-27) for n sequence pairs on the device: a (n, la), b (n, lb) int32
    CUDA tensors with per-row lengths -> (n,) int32 distances (PER/CER numerators, timit.lua:396-410)."""
    a = a.to(torch.int32).contiguous()
    b = b.to(torch.int32).contiguous()
    alen = alen.to(torch.int32).contiguous()
    blen = blen.to(torch.int32).contiguous()
    out = torch.empty(a.shape[0], dtype=torch.int32, device=a.device)
    check(lib.s2s_edit_distance(get_context(a.device.index).handle, stream_ptr(), a.shape[0], dptr(a), dptr(alen),
                                a.shape[1], dptr(b), dptr(blen), b.shape[1], dptr(out)))
    return out
