"""Device optimizer step: timit/timit.lua:292-347 on the flat buffers --
global-norm clip, L2, optim.adadelta and TrainUtils.columnNormConstraint -- in one stream-ordered
sequence of kernels (libs2s_hip.so: s2s_optim_adadelta_step), no host round trip.

    opt = Adadelta(model, rho=0.95, eps=1e-8, colnormconstr=True)   # exp_logmel7_..._colnorm.lua
    model.step(x, labels)                                           # grads = mean over the batch
    opt.step()                                                      # x updated in place

Data parallel (one process per GPU): every rank's gradients went into the all-reduce, so a rank whose persistent
launch failed poisons every replica's sum -- all ranks must skip that update together:

    flag = opt.failure_flag()                   # 1.0 on a rank whose step failed (device, stream-ordered)
    dist.reduce_failure_flag(flag)              # MAX over the ranks
    opt.step(skip_flag=flag)                    # skipped on every rank if any rank failed
"""
import ctypes

import torch

from . import _lib
from ._lib import check, lib
from .nn import dptr, get_context, stream_ptr


def weight_matrices(cfg):
    """(offset, rows, cols) of every module weight of the flat layout (s2s_model_weight_matrices)."""
    from .model import ModelConfig  # noqa: F401
    c = cfg
    d = _lib.s2s_model_dims(1, 1, 1, c.inputFrameSize, c.hiddenFrameSize, c.outputFrameSize, c.numLayers,
                            c.scoreDepth, c.stateDepth, c.outputDepth, c.mlpDepth, c.maxoutWindow, c.penalty, 0.0)
    n = lib.s2s_model_weight_matrices(ctypes.byref(d), None)
    if n < 0:
        check(1)
    buf = (ctypes.c_long * (3 * n))()
    lib.s2s_model_weight_matrices(ctypes.byref(d), buf)
    return [tuple(buf[3 * i:3 * i + 3]) for i in range(n)]


class Adadelta:
    """optim.adadelta with the reference trainer's surroundings (timit/timit.lua:292-347):
    opt.maxnorm (gradient clip), opt.weightDecay (L2), opt.colnormconstr (max row norm 1) and the
    gradient noise table gradnoise = {eta, gamma} (timit.lua:185-189, 310-315; the configs set eta = 0,
    timit.lua's own default is 1e-3).  The noise counter t lives in self.state (checkpointed with it);
    gradnoise_seed must be equal on every data-parallel rank so the replicas stay identical.
    params / grads: flat float32 CUDA tensors (ChorowskiBaseline.getParameters()), or pass the model.
    The update runs on the model's context (or ctx): if that context's failure status is set when the update
    runs on the device (a persistent launch of the step before it timed out), the update is skipped there."""

    def __init__(self, model=None, params=None, grads=None, mats=None, rho=0.95, eps=1e-8, maxnorm=1e20,
                 weightDecay=0.0, colnormconstr=False, colnorm_max=1.0, gradnoise_eta=0.0, gradnoise_gamma=0.55,
                 gradnoise_seed=0x5EED, ctx=None):
        if model is not None:
            params, grads = model.getParameters()
            if mats is None:
                mats = weight_matrices(model.cfg)
        if not (params.is_cuda and params.dtype == torch.float32 and params.is_contiguous()
                and grads.shape == params.shape):
            raise ValueError("params / grads must be flat contiguous float32 CUDA tensors of one size")
        self.params, self.grads = params, grads
        self.n = params.numel()
        self.cfg = _lib.s2s_optim_config(rho, eps, maxnorm, weightDecay, colnorm_max if colnormconstr else 0.0,
                                         gradnoise_eta, gradnoise_gamma, gradnoise_seed)
        mats = list(mats or [])
        self._mats = (ctypes.c_long * max(1, 3 * len(mats)))(*[v for m in mats for v in m])
        self._nmats = len(mats)
        self.state = torch.zeros(lib.s2s_optim_state_bytes(self.n), dtype=torch.uint8, device=params.device)
        self.gradnorm = torch.zeros(1, dtype=torch.float32, device=params.device)
        if ctx is None:
            ctx = getattr(model, "ctx", None) or get_context(params.device.index)
        self.ctx = ctx

    def set_noise_step(self, t, stream=None):
        """gradnoise.t of a resumed run (timit/timit.lua:92, 312): the next step draws with t + 1."""
        st = ctypes.c_void_p(stream.cuda_stream) if stream is not None else stream_ptr()
        check(lib.s2s_optim_set_noise_step(self.ctx.handle, st, dptr(self.state), self.n, int(t)))

    def failure_flag(self, stream=None, out=None):
        """A one-float device tensor: 1.0 if this context's failure status is set when it runs on the stream, else
        0.0 (stream-ordered, no host sync).  Data parallel: all-reduce it across the ranks (dist.reduce_failure_flag)
        and pass it to step(skip_flag=...), so a failure on any rank skips the update on every rank."""
        st = ctypes.c_void_p(stream.cuda_stream) if stream is not None else stream_ptr()
        if out is None:
            out = torch.zeros(1, dtype=torch.float32, device=self.params.device)
        check(lib.s2s_ctx_status_flag(self.ctx.handle, st, dptr(out)))
        return out

    def step(self, stream=None, skip_flag=None):
        """One update; self.gradnorm holds ||g|| before clipping (timit.lua:297 gradnorms).  skip_flag: a one-float
        device tensor (the all-reduced failure_flag of every rank); nonzero when the update runs = skip it."""
        st = ctypes.c_void_p(stream.cuda_stream) if stream is not None else stream_ptr()
        if skip_flag is None:
            check(lib.s2s_optim_adadelta_step(self.ctx.handle, st, ctypes.byref(self.cfg), dptr(self.params),
                                              dptr(self.grads), self.n, dptr(self.state), self._mats, self._nmats,
                                              dptr(self.gradnorm)))
            return
        if not (skip_flag.is_cuda and skip_flag.dtype == torch.float32 and skip_flag.numel() >= 1):
            raise ValueError("skip_flag must be a float32 CUDA tensor")
        check(lib.s2s_optim_adadelta_step_flag(self.ctx.handle, st, ctypes.byref(self.cfg), dptr(self.params),
                                               dptr(self.grads), self.n, dptr(self.state), self._mats, self._nmats,
                                               dptr(self.gradnorm), dptr(skip_flag)))
