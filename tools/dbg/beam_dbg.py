"""Debug: first maxseqlength at which the device beam search departs from the oracle (LSTM + hybrid)."""
import sys, os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", ".."))
import numpy as np
import torch
from test_frontend import _lstm_dec_case, _load_lstm_attention
from oracle import s2s_oracle as orc
import s2s_amd
from s2s_amd import frontend as fe

for hyb in ((5, 16), (0, 0)):
    rng = np.random.default_rng(4 * 10 + 10)
    B, L, S, A, Sc, O, eos = 5, 24, 32, 64, 48, 11, 2
    cfg, P = _lstm_dec_case(rng, S, A, Sc, O, hyb, "maxout")
    att, _ = _load_lstm_attention(s2s_amd, fe, P, cfg, s2s_amd.MaxoutMLP(S + A, 4, 3, O))
    h = rng.standard_normal((B, L, A)) * 1.5
    for K in (1, 2, 4):
        for m in range(1, 11):
            toks, lens, sc = att.BeamSearch(torch.tensor(h, dtype=torch.float32, device="cuda"), eos, K, m)
            g = [int(t) for t in toks[0, :lens[0]].cpu()]
            r = orc.beam_search(h[0], P, cfg, eos, K, m)
            print(hyb, K, m, g == r[0], g, float(sc[0]), r[0], r[1], flush=True)
