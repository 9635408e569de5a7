"""Diagnostic: the library's MFMA GEMM on the config-5 VGG shapes, fp32 vs bf16 operands (s2s_debug_gemm),
TFLOP/s from HIP events.  Run on a GPU box:  python tools/gemm_bf16_bench.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
import torch  # noqa: E402

from s2s_amd import _lib  # noqa: E402

fn = _lib.lib.s2s_debug_gemm
fn.restype = ctypes.c_int
fn.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_float, ctypes.c_void_p,
               ctypes.c_long, ctypes.c_void_p, ctypes.c_long, ctypes.c_float, ctypes.c_void_p, ctypes.c_long,
               ctypes.c_int, ctypes.c_void_p, ctypes.c_size_t]
ws = torch.empty(8 << 20, device="cuda")
# (name, tA, tB, M, N, K): 1x1 layer fwd (NT), dX (NN), dW (TN); a square reference shape
SHAPES = [("1x1 fwd", 0, 1, 8128, 2048, 2048), ("1x1 dX", 0, 0, 8128, 2048, 2048),
          ("1x1 dW", 1, 0, 2048, 2048, 8128), ("square", 0, 1, 4096, 4096, 4096)]
for name, tA, tB, M, N, K in SHAPES:
    A = torch.randn((K, M) if tA else (M, K), device="cuda")
    B = torch.randn((N, K) if tB else (K, N), device="cuda")
    C = torch.empty(M, N, device="cuda")
    out = {"shape": name, "M": M, "N": N, "K": K}
    for bf16 in (0, 1):
        for _ in range(2):
            fn(tA, tB, M, N, K, 1.0, A.data_ptr(), A.shape[1], B.data_ptr(), B.shape[1], 0.0, C.data_ptr(), N, bf16,
               ws.data_ptr(), ws.numel())
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(torch.cuda.default_stream())
        for _ in range(10):
            fn(tA, tB, M, N, K, 1.0, A.data_ptr(), A.shape[1], B.data_ptr(), B.shape[1], 0.0, C.data_ptr(), N, bf16,
               ws.data_ptr(), ws.numel())
        e1.record(torch.cuda.default_stream())
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 100.0
        out["bf16" if bf16 else "fp32"] = {"us": round(us, 1), "tflops": round(2.0 * M * N * K / us / 1e6, 1)}
    print(json.dumps(out), flush=True)
