"""Diagnostic: the mixed-length config-2-dims step (tests/test_gpu_ragged.py) under library debug knobs,
printing the worst gradient error per encoder layer for each arm.
python tools/ragged_knob_check.py"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "seq2seq-attention-asr_amd"))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import s2s_amd  # noqa: E402
from s2s_amd import _lib  # noqa: E402
from oracle import s2s_oracle as orc  # noqa: E402
from test_gpu_ragged import _ragged_batch  # noqa: E402


def knob(name, v):
    fn = getattr(_lib.lib, name)
    fn.argtypes = [ctypes.c_int]
    fn(v)


def run(tag, graph, B, L, T, seed, full=False):
    cfg_o = orc.ModelConfig()
    model = s2s_amd.ChorowskiBaseline(s2s_amd.ModelConfig(), graph=graph, overlap=graph)
    x, labels, flen, tlen = _ragged_batch(cfg_o, B, L, T, seed)
    if full:
        flen[:] = L
        tlen[:] = T
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        nll, logp = model.step(torch.tensor(x, dtype=torch.float32, device="cuda"), torch.tensor(labels, dtype=torch.int32, device="cuda"),
                               stream=st, frame_lengths=flen, label_lengths=tlen)
    st.synchronize()
    P = orc.unflatten(model.params.cpu().double().numpy(), cfg_o)
    _, G, _, _ = orc.training_step_ragged(x, labels, flen, tlen, P, cfg_o)
    Gg = orc.unflatten(model.grads.cpu().double().numpy(), cfg_o)
    worst = {}
    for k in G:
        e = np.abs(Gg[k] - G[k]).max() / max(np.abs(G[k]).max(), 1e-30)
        grp = k[:4] if k.startswith("enc") else "dec"
        worst[grp] = max(worst.get(grp, 0.0), e)
    print(tag, " ".join(f"{g}={v:.2e}" for g, v in sorted(worst.items())), flush=True)


def main():
    for fd in (1, 0):
        knob("s2s_debug_gru_fused_dy", fd)
        for fx in (1, 0):
            knob("s2s_debug_gru_fused_xproj", fx)
            run(f"fused_dy={fd} fused_x={fx} eager ragged B12", False, 12, 96, 30, 3)
    knob("s2s_debug_gru_fused_dy", 1)
    knob("s2s_debug_gru_fused_xproj", 1)
    run("default eager full B12", False, 12, 96, 30, 3, full=True)
    run("default graph ragged B12", True, 12, 96, 30, 3)
    run("default eager ragged B16", False, 16, 96, 30, 3)
    run("default eager ragged B32", False, 32, 64, 20, 3)


if __name__ == "__main__":
    main()
