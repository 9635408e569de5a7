"""Throughput of the big-tile bf16 GEMM (gemm_bf16.hip) on the config-5 shapes and on square problems.
Run on a GPU box:  python tools/gemm_big_bench.py
(The round-4 A/B against hipBLASLt, before it left the library: profiles/r04/gemm_big.txt.)
Prints, per shape: the direct kernel (staging passes included) and the VGG 1x1 layer (TemporalConvolution(Din, Dout,
1) + ReLU, model_vgg.lua:45-52) forward + backward (3 GEMMs) through the module path, in TFLOP/s."""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "seq2seq-attention-asr_amd"), os.path.join(ROOT, "tests")]
import s2s_amd  # noqa: E402
from s2s_amd import _lib, frontend as fe  # noqa: E402
from test_gpu_bf16 import _big_run  # noqa: E402


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e-3


def direct(M, N, K, tA, tB):
    g = torch.Generator(device="cuda").manual_seed(1)
    A = torch.rand((K, M) if tA else (M, K), device="cuda", generator=g) * 2 - 1
    B = torch.rand((N, K) if tB else (K, N), device="cuda", generator=g) * 2 - 1
    C = torch.empty(M, N, device="cuda")
    ctx = s2s_amd.nn.get_context(0)
    fn = _big_run(_lib)
    done = ctypes.c_int(0)

    def run():
        fn(ctx.handle, s2s_amd.nn.stream_ptr(), tA, tB, M, N, K, 1.0, A.data_ptr(), A.shape[1], B.data_ptr(),
           B.shape[1], 0.0, C.data_ptr(), N, None, 0, ctypes.byref(done))
    t = timed(run)
    return 2.0 * M * N * K / t / 1e12


def layer(B, L, Din, Dout):
    m = fe.TemporalConvolution(Din, Dout, 1, relu=True).cuda()
    x = torch.randn(B, L, Din, device="cuda")
    dy = torch.randn(B, L, Dout, device="cuda")

    def run():
        with s2s_amd.precision("bf16-all"):
            m.forward(x)
            m.backward(x, dy, 1.0)
    t = timed(run)
    return 3 * 2.0 * B * L * Din * Dout / t / 1e12, t * 1e6


# the big bf16 products of one config-5 step (S2S_GEMM_TRACE=1 python bench.py --config librispeech_vgg_b16)
STEP_SHAPES = [(8128, 2048, 2048, 0, 1, 2), (8128, 2048, 2048, 0, 0, 2), (2048, 2048, 8128, 1, 0, 2),
               (8128, 896, 2048, 0, 0, 1), (8128, 512, 512, 0, 1, 1), (8128, 512, 512, 0, 0, 1),
               (8128, 512, 2048, 0, 1, 1), (8128, 2048, 896, 0, 1, 1), (8128, 2048, 512, 0, 0, 1),
               (512, 512, 8128, 1, 0, 1), (512, 2048, 8128, 1, 0, 1), (448, 768, 3200, 1, 0, 1),
               (3200, 768, 448, 0, 0, 1), (3200, 768, 256, 0, 0, 1), (3200, 448, 768, 0, 1, 1),
               (3200, 256, 768, 0, 0, 1), (2048, 896, 8128, 1, 0, 1)]

if __name__ == "__main__":
    tag = "in-house"
    total = 0.0
    for M, N, K, tA, tB, n in STEP_SHAPES:
        tf = direct(M, N, K, tA, tB)
        us = 2.0 * M * N * K / (tf * 1e12) * 1e6
        total += n * us
        print(f"{tag:9s} M={M:5d} N={N:5d} K={K:5d} tA={tA} tB={tB} x{n}: {tf:7.1f} TFLOP/s {us:7.1f} us", flush=True)
    print(f"{tag} step total {total:.1f} us", flush=True)
    for M, N, K, tA, tB in ((4096, 4096, 4096, 0, 1), (8192, 8192, 8192, 0, 1)):
        print(f"in-house  M={M:5d} N={N:5d} K={K:5d}: {direct(M, N, K, tA, tB):7.1f} TFLOP/s", flush=True)
