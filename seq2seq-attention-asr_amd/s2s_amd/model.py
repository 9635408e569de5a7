"""The Chorowski TIMIT baseline autoencoder (timit/model_chorowski_baseline.lua:10-83) as one
flat-buffer training step on libs2s_hip.so (s2s_model_step).

`loadmodel(opt)` field names are kept in ModelConfig; the flat parameter/gradient buffers
play the role of `parameters, gradients = autoencoder:getParameters()` (timit/timit.lua:172).
"""
import ctypes
import dataclasses
import math

import torch

from . import _lib
from ._lib import check, lib
from .nn import _bytes, dptr, get_context, lengths_tensor, saved_view, stream_ptr


@dataclasses.dataclass
class ModelConfig:
    inputFrameSize: int = 123
    hiddenFrameSize: int = 256
    outputFrameSize: int = 256
    scoreDepth: int = 512
    stateDepth: int = 256
    outputDepth: int = 62        # opt.numPhonemes (TIMIT, incl. EOS) / opt.outputDepth (LibriSpeech chars)
    mlpDepth: int = 64
    maxoutWindow: int = 7
    penalty: float = 0.0
    numLayers: int = 3
    dropout: float = 0.0         # opt.dropout of model_chorowski_baseline_dropout.lua (0: the baseline model)

    @property
    def annotationDepth(self):
        return 2 * self.outputFrameSize

    @classmethod
    def from_opt(cls, opt: dict):
        """loadmodel(opt) defaults (timit/model_chorowski_baseline.lua:14-46)."""
        return cls(inputFrameSize=opt.get("inputFrameSize", 123), hiddenFrameSize=opt.get("hiddenFrameSize", 256),
                   outputFrameSize=opt.get("outputFrameSize", 256), scoreDepth=opt.get("scoreDepth", 512),
                   stateDepth=opt.get("stateDepth", 256),
                   outputDepth=opt.get("numPhonemes", opt.get("outputDepth", 62)),
                   mlpDepth=opt.get("mlpDepth", 64), penalty=opt.get("penalty", 0.0),
                   dropout=opt.get("dropout", 0.0))


def _mix64(a: int, b: int) -> int:
    """splitmix64 of (a, b): the default per-step dropout seed (never 0 for distinct inputs in practice)."""
    z = (int(a) * 0x9E3779B97F4A7C15 + int(b) + 0x632BE59BD9B4E019) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & 0xFFFFFFFFFFFFFFFF
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & 0xFFFFFFFFFFFFFFFF
    return z ^ (z >> 31)


def _dist_rank() -> int:
    try:
        import torch.distributed as dist
        if dist.is_available() and dist.is_initialized():
            return dist.get_rank()
    except Exception:
        pass
    import os
    return int(os.environ.get("RANK", "0"))


def param_shapes(cfg: ModelConfig):
    """Flat layout (DESIGN.md §Data layout): encoder layers x (fwd, bwd) x (Wz, Wr, Wh), then the
    decoder in s2s_attn parameter order."""
    out = []
    D = cfg.inputFrameSize
    for l in range(1, cfg.numLayers + 1):
        H = cfg.outputFrameSize if l == cfg.numLayers else cfg.hiddenFrameSize
        for d in ("f", "b"):
            for g in ("Wz", "Wr", "Wh"):
                out.append((f"enc{l}{d}.{g}", (H, H + D)))
        D = 2 * H
    A, Sc, S, O, M, k = (cfg.annotationDepth, cfg.scoreDepth, cfg.stateDepth, cfg.outputDepth, cfg.mlpDepth,
                         cfg.maxoutWindow)
    out += [("V", (Sc, A)), ("Ws", (Sc, S)), ("bs", (Sc,)), ("we", (1, Sc)), ("Wy", (S, O)), ("by", (S,)),
            ("Wc", (S, A)), ("bc", (S,)), ("Wd", (S, 2 * S)), ("bd", (S,)), ("dec.Wz", (S, 2 * S)),
            ("dec.Wr", (S, 2 * S)), ("dec.Wh", (S, 2 * S)), ("Wm", (M * k, S + A)), ("bm", (M * k,)),
            ("Wo", (O, M)), ("bo", (O,))]
    return out


def _fan_in(name, shape, cfg):
    S, Sc, A, O, M = cfg.stateDepth, cfg.scoreDepth, cfg.annotationDepth, cfg.outputDepth, cfg.mlpDepth
    table = {"V": A, "Ws": S, "bs": S, "we": Sc, "Wy": O, "by": O, "Wc": A, "bc": A, "Wd": 2 * S, "bd": 2 * S,
             "Wm": S + A, "bm": S + A, "Wo": M, "bo": M}
    return table.get(name, shape[1] if len(shape) > 1 else shape[0])


def buckets_of_shapes(shapes, num_layers):
    """grad_buckets from a param_shapes list (pure Python; pins s2s_model_bucket in the ABI tests)."""
    sizes = [math.prod(s) for _, s in shapes]
    starts = [sum(sizes[:i]) for i in range(len(sizes) + 1)]
    out = [(starts[6 * num_layers], starts[-1] - starts[6 * num_layers])]
    for l in range(num_layers - 1, -1, -1):
        out.append((starts[6 * l], starts[6 * l + 6] - starts[6 * l]))
    return out


def grad_buckets(cfg: ModelConfig):
    """[(offset, count)] slices of the flat gradient in the order the step finalises them: the
    decoder, then encoder layers numLayers .. 1 (s2s_model_bucket; host-only, no GPU call)."""
    c = cfg
    d = _lib.s2s_model_dims(1, 1, 1, c.inputFrameSize, c.hiddenFrameSize, c.outputFrameSize, c.numLayers,
                            c.scoreDepth, c.stateDepth, c.outputDepth, c.mlpDepth, c.maxoutWindow, c.penalty, 0.0)
    out = []
    nb = lib.s2s_model_bucket_count(ctypes.byref(d))
    if nb < 0:
        check(1)  # the dims are not a model the library runs (s2s_last_error says why)
    for i in range(nb):
        off, n = ctypes.c_size_t(), ctypes.c_size_t()
        check(lib.s2s_model_bucket(ctypes.byref(d), i, ctypes.byref(off), ctypes.byref(n)))
        out.append((off.value, n.value))
    return out


class ChorowskiBaseline:
    """autoencoder = decoder({encoder(x), labelmask}) with flat params/grads on one device."""

    def __init__(self, cfg: ModelConfig = None, device=None, seed: int = 1234, graph: bool = False,
                 overlap: bool = False, precision: str = "fp32"):
        self.cfg = cfg or ModelConfig()
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else device)
        shapes = param_shapes(self.cfg)
        self.shapes = shapes
        n = sum(math.prod(s) for _, s in shapes)
        g = torch.Generator().manual_seed(seed)
        flat = torch.empty(n, dtype=torch.float32)
        off = 0
        for name, shp in shapes:
            sz = math.prod(shp)
            stdv = 1.0 / math.sqrt(_fan_in(name, shp, self.cfg))
            flat[off:off + sz] = (torch.rand(sz, generator=g, dtype=torch.float64) * 2 - 1).mul_(stdv).float()
            off += sz
        self.params = flat.to(self.device)
        self.grads = torch.zeros_like(self.params)
        if graph or overlap or precision != "fp32":
            from .nn import Context
            self.ctx = Context(self.device.index, graph=graph, overlap=overlap)
            # "bf16": the step's hoisted GEMMs on bf16 MFMA, fp32 accumulation (BASELINE config 3)
            self.ctx.set_precision(precision)
        else:
            self.ctx = get_context(self.device.index)
        self.precision = precision
        self._wsbuf = None
        self._mask_buf = None
        self._outputs = {}
        self._lenbufs = {}
        self.train = True
        self._steps = 0
        # default dropout seeds: a per-step counter mixed with the init seed and the data-parallel rank,
        # so replicas draw independent nn.Dropout masks (the reference draws a fresh mask per forward)
        self.seed = int(seed)
        self.dropout_seed_base = _mix64(seed, _dist_rank())
        self._check_layout()

    def dims(self, B, L, T):
        c = self.cfg
        p = c.dropout if self.train else 0.0
        return _lib.s2s_model_dims(B, L, T, c.inputFrameSize, c.hiddenFrameSize, c.outputFrameSize, c.numLayers,
                                   c.scoreDepth, c.stateDepth, c.outputDepth, c.mlpDepth, c.maxoutWindow, c.penalty, p)

    def training(self):
        self.train = True

    def evaluate(self):
        """nn.Dropout's evaluate() mode: the decoder MLP input passes unscaled."""
        self.train = False

    def _check_layout(self):
        d = self.dims(1, 1, 1)
        assert lib.s2s_model_param_count(ctypes.byref(d)) == self.params.numel()
        off = 0
        for i, (_, shp) in enumerate(self.shapes):
            numel = ctypes.c_long()
            assert lib.s2s_model_param_offset(ctypes.byref(d), i, ctypes.byref(numel)) == off
            assert numel.value == math.prod(shp)
            off += numel.value

    def getParameters(self):
        return self.params, self.grads

    def views(self, flat=None):
        flat = self.params if flat is None else flat
        out, off = {}, 0
        for name, shp in self.shapes:
            sz = math.prod(shp)
            out[name] = flat[off:off + sz].view(shp)
            off += sz
        return out

    def workspace(self, B, L, T):
        """One workspace for every shape (grown on demand): ragged training (step_ragged) visits many
        (B, L, T) and must not keep one ~100 MB buffer per shape."""
        d = self.dims(B, L, T)
        nbytes = lib.s2s_model_workspace_bytes(ctypes.byref(d))
        if nbytes == 0:
            check(1)
        if self._wsbuf is None or self._wsbuf.numel() < nbytes:
            self._wsbuf = None
            self._wsbuf = _bytes(nbytes, self.device)
        return self._wsbuf

    def grad_buckets(self):
        return grad_buckets(self.cfg)

    def wait_bucket(self, i, stream):
        """`stream` waits until gradient bucket i of the last step(bucket_events=True) is final."""
        check(lib.s2s_stream_wait_bucket(self.ctx.handle, ctypes.c_void_p(stream.cuda_stream), i))

    def step(self, x, labels, scale=None, zero_grads=True, normalizeNLL=True, logp=None, nll=None, stream=None,
             dropout_seed=None, dropout_mask=None, bucket_events=False, frame_lengths=None, label_lengths=None):
        """One training-step gradient (timit/timit.lua:240-295): grads (+)= scale * d(sum_b nll_b)/dparams,
        scale = 1/B when B > 1 (timit.lua:292-295).  Returns (nll (B,), logp (B, T, O)); unless given, both
        are module-owned buffers overwritten by the next step of the same shape (Torch's self.output).
        With cfg.dropout > 0 (training mode) the decoder MLP input is dropped out with masks drawn
        in-kernel from dropout_seed (default: a per-step counter) or given as dropout_mask
        (B, T, S+A) multipliers.  bucket_events=True records the per-bucket "gradients final" events
        that dist.allreduce_buckets waits on.
        frame_lengths / label_lengths: (B,) frames and labels per utterance of a padded variable-length
        batch (each in [1, L] / [1, T]): the step then equals the reference's per-utterance loop over the
        unpadded utterances (timit/timit.lua:239-295); logp rows past T_b are padding.
        stream: the step runs there; it first waits for the caller's current stream (inputs and an injected
        mask written there are complete), and every host-side tensor op of the step (mask / lengths copies
        into the model-owned buffers) is issued on it too.  Outputs are ready on `stream`."""
        if stream is not None and stream != torch.cuda.current_stream(self.device):
            stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(stream):
                return self._step(x, labels, scale, zero_grads, normalizeNLL, logp, nll, stream, dropout_seed,
                                  dropout_mask, bucket_events, frame_lengths, label_lengths)
        return self._step(x, labels, scale, zero_grads, normalizeNLL, logp, nll, stream, dropout_seed, dropout_mask,
                          bucket_events, frame_lengths, label_lengths)

    def _step(self, x, labels, scale, zero_grads, normalizeNLL, logp, nll, stream, dropout_seed, dropout_mask,
              bucket_events, frame_lengths, label_lengths):
        # every torch op here runs on the step's stream (step() entered its context when it differs)
        if x.dim() == 2:
            x = x[None]
        if labels.dim() == 1:
            labels = labels[None]
        B, L, F = x.shape
        T = labels.shape[1]
        if F != self.cfg.inputFrameSize:
            raise ValueError(f"input frame size {F} != {self.cfg.inputFrameSize}")
        if not (x.is_cuda and x.dtype == torch.float32 and x.is_contiguous()):
            raise ValueError("x must be a contiguous float32 CUDA tensor")
        lab = labels.to(torch.int32).contiguous()
        if scale is None:
            scale = 1.0 / B if B > 1 else 1.0
        if logp is None or nll is None:
            # module-owned outputs reused from step to step (as Torch's self.output): stable pointers keep
            # a graph-mode context replaying one captured step; clone them to keep a step's values
            o = self._outputs.get((B, T))
            if o is None:
                o = (torch.empty((B, T, self.cfg.outputDepth), device=self.device, dtype=torch.float32),
                     torch.empty(B, device=self.device, dtype=torch.float32))
                self._outputs[(B, T)] = o
            logp = o[0] if logp is None else logp
            nll = o[1] if nll is None else nll
        ws = self.workspace(B, L, T)
        d = self.dims(B, L, T)
        self._steps += 1
        if d.dropout > 0:
            d.dropout_seed = _mix64(self.dropout_seed_base, self._steps) if dropout_seed is None else int(dropout_seed)
            if dropout_mask is not None:
                S, A = self.cfg.stateDepth, self.cfg.annotationDepth
                if dropout_mask.shape != (B, T, S + A) or dropout_mask.dtype != torch.float32:
                    raise ValueError("dropout_mask must be float32 (B, T, stateDepth + annotationDepth)")
                # copied into a model-owned buffer: its pointer (part of a captured step's key) stays the
                # same from step to step, so a graph-mode context replays instead of re-capturing
                n = dropout_mask.numel()
                if self._mask_buf is None or self._mask_buf.numel() < n:
                    self._mask_buf = torch.empty(n, device=self.device, dtype=torch.float32)
                self._mask_buf[:n].copy_(dropout_mask.reshape(-1))
                d.dropout_mask = self._mask_buf.data_ptr()
        if frame_lengths is not None or label_lengths is not None:
            fl = lengths_tensor(frame_lengths if frame_lengths is not None else [L] * B, B, L, "cpu")
            tl = lengths_tensor(label_lengths if label_lengths is not None else [T] * B, B, T, "cpu")
            # model-owned (2, B) device buffer: a stable pointer (part of a captured step's key) whose
            # contents the replayed kernels read at run time; written on the step's stream
            buf = self._lenbufs.get(B)
            if buf is None:
                buf = torch.empty((2, B), dtype=torch.int32, device=self.device)
                self._lenbufs[B] = buf
            host = torch.stack([fl, tl]).pin_memory()
            buf.copy_(host, non_blocking=True)  # on the step's stream; the caching host allocator keeps
            self._len_host = host                # the pinned source alive until the copy has run
            d.frame_lengths = buf[0].data_ptr()
            d.label_lengths = buf[1].data_ptr()
        flags = (_lib.S2S_ZERO_GRADS if zero_grads else 0) | (_lib.S2S_NORMALIZE_NLL if normalizeNLL else 0)
        if bucket_events:
            flags |= _lib.S2S_BUCKET_EVENTS
        st = ctypes.c_void_p(stream.cuda_stream) if stream is not None else stream_ptr()
        check(lib.s2s_model_step(self.ctx.handle, st, ctypes.byref(d), dptr(self.params), dptr(self.grads), dptr(x),
                                 dptr(lab), float(scale), flags, dptr(logp), dptr(nll), dptr(ws), ws.numel()))
        self._last = (B, L, T)
        return nll, logp

    def step_ragged(self, xs, labels, max_batch=None, normalizeNLL=True, stream=None):
        """The reference's minibatch over variable-length utterances (timit/timit.lua:240-295: one
        forward/backward per utterance, gradients summed, then / B) as padded, length-masked batched steps:
        utterances sorted by length, cut into batches of at most max_batch (default: all), each padded to its
        longest utterance and run with frame_lengths / label_lengths, accumulating into the same gradient
        with scale 1/B (B = all utterances) -- the per-utterance sum up to fp32 reassociation.
        xs: list of (L_i, F) float32 CUDA tensors; labels: list of (T_i,) 0-based int tensors.
        Returns nll (B,) in input order and the per-utterance logp list ((T_i, O) each)."""
        if len(xs) != len(labels) or not xs:
            raise ValueError("step_ragged needs one label sequence per utterance")
        if stream is not None and stream != torch.cuda.current_stream(self.device):
            stream.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(stream):  # padding, the steps and the output clones all on `stream`
                return self.step_ragged(xs, labels, max_batch, normalizeNLL, stream)
        B = len(xs)
        scale = 1.0 / B if B > 1 else 1.0
        nll = torch.empty(B, device=self.device, dtype=torch.float32)
        logps = [None] * B
        order = sorted(range(B), key=lambda i: (xs[i].shape[0], labels[i].shape[0]))
        nb = max_batch or B
        first = True
        for c0 in range(0, B, nb):
            idx = order[c0:c0 + nb]
            Ls = [xs[i].shape[0] for i in idx]
            Ts = [labels[i].shape[0] for i in idx]
            L, T, F = max(Ls), max(Ts), xs[idx[0]].shape[1]
            x = torch.zeros((len(idx), L, F), device=self.device, dtype=torch.float32)
            y = torch.zeros((len(idx), T), device=self.device, dtype=torch.int32)
            for j, i in enumerate(idx):
                x[j, :Ls[j]] = xs[i]
                y[j, :Ts[j]] = labels[i].to(torch.int32)
            n, lp = self.step(x, y, scale=scale, zero_grads=first, normalizeNLL=normalizeNLL, stream=stream,
                              frame_lengths=Ls, label_lengths=Ts)
            first = False
            nll[torch.tensor(idx, device=self.device)] = n
            for j, i in enumerate(idx):
                logps[i] = lp[j, :Ts[j]].clone()  # lp is the module-owned output, reused by the next batch
        return nll, logps

    # ---- the decoder's trainer-visible surface after a step (timit/timit.lua:519-521, 534-536)
    def _attn(self):
        B, L, T = self._last
        d = self.dims(B, L, T)
        ad = _lib.s2s_attn_dims()
        check(lib.s2s_model_attn_dims(ctypes.byref(d), ctypes.byref(ad)))
        p = lib.s2s_model_attn_saved(ctypes.byref(d), dptr(self._wsbuf))
        if not p:
            check(1)
        return ad, p

    def decoder_alpha(self):
        """decoder:alpha() (Attention.lua:241-243) of the last step: (B, T, L)."""
        ad, sv = self._attn()
        return saved_view(self._wsbuf, lib.s2s_attn_alpha(ctypes.byref(ad), ctypes.c_void_p(sv)), (ad.B, ad.T, ad.L))

    def decoder_penalty(self):
        """decoder:penalty() (Attention.lua:244-246): MonotonicAlignment's output, i.e. alpha."""
        return self.decoder_alpha()

    def decoder_Ws(self):
        """decoder:Ws() (Attention.lua:247-249): ws_t broadcast over L, (B, T, L, scoreDepth) expand view."""
        ad, sv = self._attn()
        ws = saved_view(self._wsbuf, lib.s2s_attn_ws(ctypes.byref(ad), ctypes.c_void_p(sv)),
                        (ad.B, ad.T, ad.scoreDepth))
        return ws[:, :, None, :].expand(ad.B, ad.T, ad.L, ad.scoreDepth)

    def decoder_Vh(self):
        """decoder.Vh.output (Attention.lua:43-47): (B, L, scoreDepth)."""
        ad, sv = self._attn()
        return saved_view(self._wsbuf, lib.s2s_attn_vh(ctypes.byref(ad), ctypes.c_void_p(sv)),
                          (ad.B, ad.L, ad.scoreDepth))

    def decoder_maxout_argmax(self):
        """(B, T, mlpDepth) int32 Maxout decisions of the last step's decoder (which unit of each group won)."""
        ad, sv = self._attn()
        return saved_view(self._wsbuf, lib.s2s_attn_maxout_argmax(ctypes.byref(ad), ctypes.c_void_p(sv)),
                          (ad.B, ad.T, ad.mlpDepth), torch.int32)

    def dropout_mask_used(self):
        """(B, T, S+A) nn.Dropout multipliers of the last step (None without dropout)."""
        ad, sv = self._attn()
        if ad.dropout <= 0:
            return None
        return saved_view(self._wsbuf, lib.s2s_attn_dropout_mask(ctypes.byref(ad), ctypes.c_void_p(sv)),
                          (ad.B, ad.T, ad.stateDepth + ad.annotationDepth))

    def encoder_output(self):
        B, L, T = self._last
        d = self.dims(B, L, T)
        ws = self._wsbuf
        p = lib.s2s_model_encoder_output(ctypes.byref(d), dptr(ws))
        off = p - ws.data_ptr()
        n = B * L * self.cfg.annotationDepth
        return ws[off:off + 4 * n].view(torch.float32).view(B, L, self.cfg.annotationDepth)
