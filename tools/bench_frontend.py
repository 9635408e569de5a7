"""Front-end encoders on one MI355X: forward + backward throughput and achieved
fp32 MFMA rate.  One JSON line per encoder:
  * VGGEncoder at BASELINE config 5's shape (librispeech/model_vgg.lua: input (B, 3, L=1024, 40),
    1x1 layers 2048 wide, output 512), synthetic N(0,1) input, random-init weights;
  * ConvBiLSTMEncoder (timit/timit.lua:108-125: 3 x conv(k=3, 256) + pool, BiLSTM 2 x 128) at
    config 2's B=32, L=128 (+ a 4x longer L=512 case), D=123.
frames/s counts input frames (B*L) per fwd+bwd; flops are the algorithmic contraction flops
(2*M*N*K per GEMM-shaped product, fwd + dX + dW).
Usage (GPU box): python tools/bench_frontend.py [--steps 10]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "seq2seq-attention-asr_amd")]

import torch  # noqa: E402

PEAK_F32 = 157.3  # TFLOP/s, dense fp32 MFMA (MI355X)


def vgg_flops(B, L, F, hidden, out):
    fl, H, W = 0.0, L, F
    first = True
    for (ci, co), pool in zip(((3, 64), (64, 64), (64, 128), (128, 128)), (None, (1, 2), None, (2, 2))):
        H, W = H - 2, W - 2
        f = 2.0 * B * co * ci * 9 * H * W
        fl += f * (2 if first else 3)  # fwd + dW (+ dX except the first layer)
        first = False
        if pool:
            H, W = H // pool[0], W // pool[1]
    din = 128 * W
    for do in (hidden, hidden, hidden, out):
        fl += 3 * 2.0 * B * H * din * do
        din = do
    return fl


def conv_lstm_flops(B, L, D, Hc=256, Ho=128):
    fl, Lc, din = 0.0, L, D
    for l in range(3):
        Lc = Lc - 2
        fl += (2 if l == 0 else 3) * 2.0 * B * Lc * 3 * din * Hc
        Lc //= 2
        din = Hc
    fl += 3 * 2 * 2.0 * B * Lc * 4 * Ho * (Hc + Ho)  # two directions, 4 gates, x and h products
    return fl, Lc


def time_encoder(enc, x, dy, steps, warmup):
    for _ in range(warmup):
        enc.forward(x)
        enc.backward(x, dy)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(steps):
        enc.forward(x)
        enc.backward(x, dy)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    args = ap.parse_args()
    import s2s_amd
    torch.manual_seed(0)
    out = []
    B, L, F = 16, 1024, 40
    enc = s2s_amd.VGGEncoder(F, outputFrameSize=512, hidden=2048).cuda()
    x = torch.randn(B, 3, L, F, device="cuda")
    y = enc.forward(x)
    dy = torch.randn_like(y)
    ms = time_encoder(enc, x, dy, args.steps, args.warmup)
    fl = vgg_flops(B, L, F, 2048, 512)
    out.append({"encoder": "VGGEncoder (librispeech/model_vgg.lua)", "shape": f"B={B} x (3, L={L}, F={F})",
                "ms_per_fwd_bwd": round(ms, 3), "frames_per_s": round(B * L / ms * 1e3, 1),
                "tflops": round(fl / ms / 1e9, 2), "frac_fp32_mfma_peak": round(fl / ms / 1e9 / PEAK_F32, 4),
                "dtype": "fp32", "data": "synthetic"})
    # the whole librispeech/model_vgg.lua training step (config 5 shape): VGG encoder + GRU attention
    # decoder over L' = 508 frames, T = 200 char targets (O = 29), two-Maxout decoder_mlp, loss seed
    B, L, F, T = 16, 1024, 40, 200
    model = s2s_amd.VGGAttentionModel(F, outputFrameSize=512, hidden=2048, outputDepth=29).cuda()
    x = torch.randn(B, 3, L, F, device="cuda")
    lab = torch.randint(0, 28, (B, T), device="cuda", dtype=torch.int32)
    lab[:, -1] = 28
    for _ in range(args.warmup):
        model.step(x, lab)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.steps):
        model.step(x, lab)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    out.append({"model": "VGGAttentionModel (librispeech/model_vgg.lua, BASELINE config 5 shape)",
                "shape": f"B={B} x (3, L={L}, F={F}), T={T}, O=29", "ms_per_step": round(ms, 3),
                "frames_per_s": round(B * L / ms * 1e3, 1), "dtype": "fp32", "data": "synthetic",
                "what": "encoder + decoder forward, nll seed, backward (no optimizer)"})
    # the whole timit/timit.lua:106-145 conv + BiLSTM model step at its own sizes (D = 123, LSTM(400) decoder,
    # scoreDepth 150 -> 160 padded, hybrid attention kW = 5 / 16 maps, O = 62), B = 32, L = 512 -> L' = 62, T = 40
    B, L, D, T = 32, 512, 123, 40
    model = s2s_amd.ConvBiLSTMAttentionModel(D).cuda()
    x = torch.randn(B, L, D, device="cuda")
    lab = torch.randint(0, 61, (B, T), device="cuda", dtype=torch.int32)
    for _ in range(args.warmup):
        model.step(x, lab)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(args.steps):
        model.step(x, lab)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / args.steps
    out.append({"model": "ConvBiLSTMAttentionModel (timit/timit.lua:106-145)",
                "shape": f"B={B} x (L={L}, D={D}), T={T}, O=62", "ms_per_step": round(ms, 3),
                "frames_per_s": round(B * L / ms * 1e3, 1), "dtype": "fp32", "data": "synthetic",
                "what": "encoder + LSTM/hybrid-attention decoder forward, nll seed, backward (per-step decoder launches)"})
    for B, L in ((32, 128), (32, 512)):
        D = 123
        enc = s2s_amd.ConvBiLSTMEncoder(D).cuda()
        x = torch.randn(B, L, D, device="cuda")
        y = enc.forward(x)
        dy = torch.randn_like(y)
        ms = time_encoder(enc, x, dy, args.steps, args.warmup)
        fl, Lc = conv_lstm_flops(B, L, D)
        out.append({"encoder": "ConvBiLSTMEncoder (timit/timit.lua:108-125)", "shape": f"B={B} x (L={L}, D={D}) -> L'={Lc}",
                    "ms_per_fwd_bwd": round(ms, 3), "frames_per_s": round(B * L / ms * 1e3, 1),
                    "tflops": round(fl / ms / 1e9, 2), "frac_fp32_mfma_peak": round(fl / ms / 1e9 / PEAK_F32, 4),
                    "dtype": "fp32", "data": "synthetic"})
    for o in out:
        print(json.dumps(o))


if __name__ == "__main__":
    t0 = time.time()
    main()
