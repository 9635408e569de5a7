"""Conv + BiLSTM model step (timit/timit.lua:106-145) eager vs captured graph (ConvBiLSTMAttentionModel.graph_step),
alternating in one process.  python tools/ab_convlstm.py [B L T]"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
import s2s_amd  # noqa: E402


def main():
    B, L, T = (int(v) for v in sys.argv[1:4]) if len(sys.argv) > 3 else (32, 512, 40)
    g = torch.Generator().manual_seed(3)
    x = torch.randn((B, L, 123), generator=g).cuda()
    labels = torch.randint(0, 61, (B, T), generator=g).to(torch.int32).cuda()
    m_e = s2s_amd.ConvBiLSTMAttentionModel(generator=torch.Generator().manual_seed(1)).cuda()
    m_g = s2s_amd.ConvBiLSTMAttentionModel(generator=torch.Generator().manual_seed(1)).cuda()

    def eager():
        m_e.zeroGradParameters()
        m_e.step(x, labels)

    def graph():
        m_g.graph_step(x, labels)

    modes = (("eager", eager), ("graph", graph))
    if os.environ.get("AB_ONLY"):  # one mode (profiling): AB_ONLY=eager|graph
        modes = tuple(m for m in modes if m[0] == os.environ["AB_ONLY"])
    res = {name: [] for name, _ in modes}
    for _ in range(3 if len(modes) > 1 else 1):
        for name, fn in modes:
            for _ in range(2):
                fn()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(10):
                fn()
            torch.cuda.synchronize()
            res[name].append((time.perf_counter() - t0) / 10 * 1e3)
    for name, v in res.items():
        xs = sorted(v)
        print(f"conv+BiLSTM B={B} L={L} T={T} {name}: median {xs[len(xs) // 2]:.3f} ms/step "
              f"({B * L / xs[len(xs) // 2] * 1e3:,.0f} frames/s)  all {' '.join(f'{t:.3f}' for t in v)}")


if __name__ == "__main__":
    main()
