"""ctypes wrapper of oracle/cpu_ref.c (libs2s_cpuref.so): the C restatement of the training step.

TEST / MEASUREMENT INFRASTRUCTURE (bench.py's cpu_baseline leg, tests/test_cpu_ref.py), never the product path.
Build: make -C oracle (__graft_entry__.build() runs it)."""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(_HERE, "build", "libs2s_cpuref.so")


class _Cfg(ctypes.Structure):
    _fields_ = [("F", ctypes.c_int), ("Hh", ctypes.c_int), ("Ho", ctypes.c_int), ("nl", ctypes.c_int),
                ("Sc", ctypes.c_int), ("S", ctypes.c_int), ("O", ctypes.c_int), ("M", ctypes.c_int),
                ("k", ctypes.c_int), ("penalty", ctypes.c_float)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} missing: run make -C oracle")
        _lib = ctypes.CDLL(LIB_PATH)
        P = ctypes.c_void_p
        _lib.s2s_cpu_step.restype = ctypes.c_int
        _lib.s2s_cpu_step.argtypes = [ctypes.POINTER(_Cfg), P, P, P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P,
                                      ctypes.c_int, ctypes.c_int, P, P]
        _lib.s2s_cpu_param_count.restype = ctypes.c_long
        _lib.s2s_cpu_param_count.argtypes = [ctypes.POINTER(_Cfg)]
    return _lib


def cfg_of(c):
    """an oracle / s2s_amd ModelConfig (field names of loadmodel(opt)) -> the C struct"""
    return _Cfg(c.inputFrameSize, c.hiddenFrameSize, c.outputFrameSize, c.numLayers, c.scoreDepth, c.stateDepth,
                c.outputDepth, c.mlpDepth, c.maxoutWindow, float(c.penalty))


def training_step(x, labels, flat_params, cfg, normalizeNLL=True, dropout_mask=None, threads=0):
    """oracle.training_step's contract on the C restatement: x (B, L, F), labels (B, T) 0-based, flat fp32 params
    (model.param_shapes order).  Returns (nll per utterance (B,), flat gradient (1/B if B > 1) * sum)."""
    L_ = lib()
    c = cfg_of(cfg)
    x = np.ascontiguousarray(x, np.float32)
    lab = np.ascontiguousarray(labels, np.int32)
    W = np.ascontiguousarray(flat_params, np.float32)
    B, L, F = x.shape
    T = lab.shape[1]
    n = L_.s2s_cpu_param_count(ctypes.byref(c))
    if W.size != n:
        raise ValueError(f"{W.size} parameters, the layout has {n}")
    m = None if dropout_mask is None else np.ascontiguousarray(dropout_mask, np.float32)
    g = np.zeros(n, np.float32)
    nll = np.zeros(B, np.float32)
    rc = L_.s2s_cpu_step(ctypes.byref(c), W.ctypes.data, x.ctypes.data, lab.ctypes.data, B, L, T,
                         None if m is None else m.ctypes.data, int(normalizeNLL), int(threads), g.ctypes.data,
                         nll.ctypes.data)
    if rc != 0:
        raise MemoryError("s2s_cpu_step failed")
    return nll, g
