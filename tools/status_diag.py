"""Diagnostic: failure status after each config-2 model step (eager / graph, overlap), to localise a reported
hand-off failure.  python tools/status_diag.py"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "seq2seq-attention-asr_amd"))
import torch  # noqa: E402

import ctypes  # noqa: E402

import s2s_amd  # noqa: E402
from s2s_amd import _lib  # noqa: E402

_lib.lib.s2s_debug_status_words.argtypes = [ctypes.c_void_p, ctypes.c_void_p]


def words(ctx):
    w = (ctypes.c_uint * 16)()
    _lib.lib.s2s_debug_status_words(ctx.handle, w)
    return list(w)

cfg = s2s_amd.ModelConfig()
g = torch.Generator().manual_seed(1)
x = torch.randn(32, 128, 123, generator=g).cuda()
lab = torch.randint(0, 61, (32, 40), generator=g).to(torch.int32).cuda()
for knob in (1, 0):
  _lib.lib.s2s_debug_sync_handover(knob)
  for graph in (False, True):
      m = s2s_amd.ChorowskiBaseline(cfg, graph=graph, overlap=True)
      st = torch.cuda.Stream()
      out = []
      with torch.cuda.stream(st):
          for i in range(6):
              m.step(x, lab, stream=st)
              st.synchronize()
              out.append(words(m.ctx)[:8])
              m.ctx.status(st, clear=True)
      print(f"handover={knob} graph={graph} status words per step: {out}", flush=True)
