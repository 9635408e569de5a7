"""A/B a library debug knob on the config-2 training step under hipGraph replay (as bench.py runs it):
one model per arm, each captured with its knob value set, then timed alternately in one process.
python tools/ab_graph_knob.py s2s_debug_side_xcd_skip 1 0 [rounds] [B L T]"""
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
    rounds = int(sys.argv[4]) if len(sys.argv) > 4 else 5
    B, L, T = (int(v) for v in sys.argv[5:8]) if len(sys.argv) > 7 else (32, 128, 40)
    fn = getattr(_lib.lib, name)
    fn.argtypes = [ctypes.c_int]
    cfg = s2s_amd.ModelConfig()
    x = torch.randn(B, L, cfg.inputFrameSize, device="cuda")
    lab = torch.randint(0, cfg.outputDepth, (B, T), device="cuda", dtype=torch.int32)
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    models = {}
    for v in (a, b):
        fn(v)  # a knob is read while the step is recorded: each arm's graph is captured under its value
        m = s2s_amd.ChorowskiBaseline(cfg, graph=True, overlap=True)
        if models:
            m.params.copy_(next(iter(models.values())).params)
        with torch.cuda.stream(st):
            m.step(x, lab, stream=st)
        st.synchronize()
        models[v] = m
    res = {a: [], b: []}
    for _ in range(rounds):
        for v in (a, b):
            m = models[v]
            with torch.cuda.stream(st):
                for _ in range(3):
                    m.step(x, lab, stream=st)
                st.synchronize()
                t0 = time.perf_counter()
                for _ in range(30):
                    m.step(x, lab, stream=st)
                st.synchronize()
            res[v].append((time.perf_counter() - t0) / 30 * 1e3)
    g = {v: models[v].grads.clone() for v in (a, b)}
    for v in (a, b):
        xs = sorted(res[v])
        print(f"{name}={v}: median {xs[len(xs) // 2]:.3f} ms/step  all {' '.join(f'{t:.3f}' for t in res[v])}")
    print("grads bitwise equal across arms:", bool(torch.equal(g[a], g[b])))


if __name__ == "__main__":
    main()
