"""A/B a library debug knob on the config-5 VGG training step (VGGAttentionModel.graph_step, as bench.py runs it):
one model per arm, each captured with its knob value set, then timed alternately in one process.
python tools/ab_vgg.py s2s_debug_sconv_wgrad_implicit 1 0 [rounds] [precision]"""
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
import s2s_amd  # noqa: E402
from s2s_amd import _lib  # noqa: E402


def main():
    name, a, b = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 3
    prec = sys.argv[5] if len(sys.argv) > 5 else "bf16-all"
    fn = getattr(_lib.lib, name)
    fn.argtypes = [ctypes.c_int]
    B, L, T, F, O = 16, 1024, 200, 40, 29
    g = torch.Generator().manual_seed(1234)
    x = torch.randn((B, 3, L, F), generator=g).cuda()
    labels = torch.randint(0, O - 1, (B, T), generator=g).to(torch.int32).cuda()
    models = {}
    for v in (a, b):
        fn(v)  # read while the step is captured
        m = s2s_amd.VGGAttentionModel(F, outputFrameSize=512, hidden=2048, outputDepth=O,
                                      generator=torch.Generator().manual_seed(1234), precision=prec).cuda()
        m.graph_step(x, labels)
        models[v] = m
    torch.cuda.synchronize()
    same = all(torch.equal(p, q) for p, q in zip(models[a].parameters()[1], models[b].parameters()[1]))
    res = {a: [], b: []}
    for _ in range(rounds):
        for v in (a, b):
            for _ in range(2):
                models[v].graph_step(x, labels)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                models[v].graph_step(x, labels)
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t0) / 10 * 1e3)
    for v in (a, b):
        xs = sorted(res[v])
        print(f"{name}={v}: median {xs[len(xs) // 2]:.3f} ms/step  all {' '.join(f'{t:.3f}' for t in res[v])}")
    rel = max(((p - q).norm() / q.norm().clamp_min(1e-30)).item()
              for p, q in zip(models[a].parameters()[1], models[b].parameters()[1]))
    print(f"grads bitwise equal across arms: {same}; max rel L2 difference {rel:.2e}")


if __name__ == "__main__":
    main()
