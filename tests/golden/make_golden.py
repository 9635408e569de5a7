"""Generates the committed golden fixtures from the CPU oracle (oracle/s2s_oracle.py).

The reference (Torch7/Lua) cannot run here, so these vectors are the
oracle's outputs after it was pinned by tests/test_oracle.py (notebook known answers,
autograd, finite differences).  Run:  python tests/golden/make_golden.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import s2s_oracle as orc  # noqa: E402


def cfg_fields(cfg):
    return {"cfg_" + k: np.array(getattr(cfg, k)) for k in
            ("inputFrameSize", "hiddenFrameSize", "outputFrameSize", "scoreDepth", "stateDepth",
             "outputDepth", "mlpDepth", "maxoutWindow", "penalty", "numLayers")}


def tiny():
    # notebook-sized dims (Attention.ipynb cell 42: D=5-ish, H=4, L=10, T=9, O=2..7)
    cfg = orc.ModelConfig(inputFrameSize=5, hiddenFrameSize=4, outputFrameSize=4, scoreDepth=5,
                          stateDepth=4, outputDepth=7, mlpDepth=3, maxoutWindow=2, penalty=0.0, numLayers=3)
    P = orc.init_params(cfg, seed=1234)
    x, labels = orc.synthetic_batch(cfg, 4, 10, 9, seed=1234, pad=1, eos=3)
    nll, G, logp, enc = orc.training_step(x, labels, P, cfg)
    np.savez_compressed(os.path.join(HERE, "tiny_step.npz"), x=x, labels=labels, params=orc.flatten(P, cfg),
                        logp=logp, enc=enc, grads=orc.flatten(G, cfg), nll=np.array(nll), **cfg_fields(cfg))


def chorowski():
    # Chorowski-shaped case: L=32, T=10, F=123, B=2; params from seed 1234
    cfg = orc.ModelConfig()
    P = orc.init_params(cfg, seed=1234)
    x, labels = orc.synthetic_batch(cfg, 2, 32, 10, seed=1234, pad=10, eos=23)
    nll, G, logp, enc = orc.training_step(x, labels, P, cfg)
    flatG = orc.flatten(G, cfg)
    rng = np.random.default_rng(99)
    idx = np.sort(rng.choice(flatG.size, 4096, replace=False))
    norms = np.array([np.linalg.norm(G[n]) for n, _ in orc.param_shapes(cfg)])
    np.savez_compressed(os.path.join(HERE, "chorowski_L32_T10.npz"), labels=labels, logp=logp, enc=enc,
                        grad_idx=idx, grad_vals=flatG[idx], grad_norms=norms, nll=np.array(nll),
                        seed=np.array(1234), **cfg_fields(cfg))


if __name__ == "__main__":
    tiny()
    chorowski()
    for f in sorted(os.listdir(HERE)):
        print(f, os.path.getsize(os.path.join(HERE, f)))
