"""Diagnostic: capture a module-level training step (ConvBiLSTMAttentionModel / VGGAttentionModel) in a
torch.cuda.CUDAGraph and compare replay time and gradients with eager execution."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "seq2seq-attention-asr_amd")]
import torch  # noqa: E402

import s2s_amd  # noqa: E402


def run(name, model, x, lab, steps=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            model.zeroGradParameters()
            model.step(x, lab)
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    ref = [g.clone() for g in model.parameters()[1]]
    t0 = time.time()
    for _ in range(steps):
        model.zeroGradParameters()
        model.step(x, lab)
    torch.cuda.synchronize()
    eager = (time.time() - t0) / steps * 1e3
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        model.zeroGradParameters()
        model.step(x, lab)
    g.replay()
    torch.cuda.synchronize()
    same = all(torch.equal(a, b) for a, b in zip(ref, model.parameters()[1]))
    t0 = time.time()
    for _ in range(steps):
        g.replay()
    torch.cuda.synchronize()
    graph = (time.time() - t0) / steps * 1e3
    print(f"{name}: eager {eager:.3f} ms, graph replay {graph:.3f} ms, grads bitwise equal: {same}", flush=True)


torch.manual_seed(0)
m = s2s_amd.ConvBiLSTMAttentionModel(123).cuda()
x = torch.randn(32, 512, 123, device="cuda")
lab = torch.randint(0, 61, (32, 40), device="cuda", dtype=torch.int32)
run("conv+BiLSTM model B=32 L=512 T=40", m, x, lab)
m = s2s_amd.VGGAttentionModel(40, outputFrameSize=512, hidden=2048, outputDepth=29).cuda()
x = torch.randn(16, 3, 1024, 40, device="cuda")
lab = torch.randint(0, 28, (16, 200), device="cuda", dtype=torch.int32)
run("VGG model B=16 L=1024 T=200", m, x, lab, steps=5)
