import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "seq2seq-attention-asr_amd")
for p in (ROOT, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


# The benched hot path's parity files run first (the driver runs `pytest -x`: a failure in a next-row test
# must not keep the config-2 kernels -- persistent BiGRU, XCD-local decoder -- from being checked).
_FIRST = ("test_gpu_parity.py", "test_gpu_graph.py", "test_gpu_status.py", "test_gpu_fullsize.py",
          "test_gpu_ragged.py", "test_gpu_bf16.py")


def pytest_collection_modifyitems(session, config, items):
    def rank(item):
        name = os.path.basename(str(item.fspath))
        return _FIRST.index(name) if name in _FIRST else len(_FIRST)

    items.sort(key=rank)  # stable: the order inside each file is kept
