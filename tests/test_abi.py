"""CPU-side checks of the drop-in boundary: libs2s_hip.so loads, exports every symbol
include/s2s_hip.h declares, and the host layout agrees with the oracle's.  No compute calls."""
import ctypes
import math
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    hdr = open(os.path.join(ROOT, "include", "s2s_hip.h")).read()
    return set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(s2s_\w+)\(", hdr, re.M))


def test_library_exports_every_declared_symbol():
    from s2s_amd import _lib
    syms = header_symbols()
    assert len(syms) >= 20
    for s in syms:
        assert hasattr(_lib.lib, s), s
    assert {n for n, _, _ in _lib.SIGNATURES} == syms


def test_library_is_gfx950_code_object():
    from s2s_amd import _lib
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_param_layout_matches_oracle():
    from s2s_amd import _lib, model
    from oracle import s2s_oracle as orc
    for kw in ({}, dict(inputFrameSize=80, outputDepth=29), dict(numLayers=2, hiddenFrameSize=128)):
        cfg = model.ModelConfig(**kw)
        ocfg = orc.ModelConfig(**kw)
        assert [(n, s) for n, s in model.param_shapes(cfg)] == [(n, s) for n, s in orc.param_shapes(ocfg)]
        d = _lib.s2s_model_dims(2, 8, 3, cfg.inputFrameSize, cfg.hiddenFrameSize, cfg.outputFrameSize,
                                cfg.numLayers, cfg.scoreDepth, cfg.stateDepth, cfg.outputDepth, cfg.mlpDepth,
                                cfg.maxoutWindow, cfg.penalty)
        assert _lib.lib.s2s_model_param_count(ctypes.byref(d)) == sum(math.prod(s) for _, s in model.param_shapes(cfg))
        assert _lib.lib.s2s_model_param_offset(ctypes.byref(d), 10 ** 6, None) == -1


def test_grad_buckets_cover_the_flat_layout():
    """s2s_model_bucket (S2S_BUCKET_EVENTS order: decoder, then encoder layers top-down) agrees with
    the Python layout and tiles the flat gradient exactly once."""
    from s2s_amd import model
    for kw in ({}, dict(numLayers=2, hiddenFrameSize=128), dict(numLayers=4)):
        cfg = model.ModelConfig(**kw)
        shapes = model.param_shapes(cfg)
        got = model.grad_buckets(cfg)
        assert got == model.buckets_of_shapes(shapes, cfg.numLayers)
        assert len(got) == cfg.numLayers + 1
        cover = sorted(got)
        assert cover[0][0] == 0 and cover[-1][0] + cover[-1][1] == sum(math.prod(s) for _, s in shapes)
        assert all(o + n == o2 for (o, n), (o2, _) in zip(cover, cover[1:]))


def test_weight_matrices_are_the_2d_params():
    """s2s_model_weight_matrices (the column-norm constraint's targets) = every 2-D parameter of the
    flat layout, at its offset, rows x cols = its (out, in) shape."""
    from s2s_amd import model, optim
    for kw in ({}, dict(numLayers=2, hiddenFrameSize=128)):
        cfg = model.ModelConfig(**kw)
        want, off = [], 0
        for _, shp in model.param_shapes(cfg):
            if len(shp) == 2:
                want.append((off, shp[0], shp[1]))
            off += math.prod(shp)
        assert optim.weight_matrices(cfg) == want


def test_chorowski_param_count():
    """4,356,735 incl. the two zero TCZB biases (512 + 1) the flat layout omits."""
    from s2s_amd import model
    n = sum(math.prod(s) for _, s in model.param_shapes(model.ModelConfig()))
    assert n + 513 == 4356735


def test_errors_are_reported_not_aborted():
    from s2s_amd import _lib
    d = _lib.s2s_model_dims(0, 8, 3, 123, 256, 256, 3, 512, 256, 62, 64, 7, 0.0)
    assert _lib.lib.s2s_model_workspace_bytes(ctypes.byref(d)) == 0
    rc = _lib.lib.s2s_model_step(None, None, ctypes.byref(d), None, None, None, None, 1.0, 0, None, None, None, 0)
    assert rc != 0
    assert b"context" in _lib.lib.s2s_last_error() or b"null" in _lib.lib.s2s_last_error()


def test_unsupported_configs_raise():
    import s2s_amd
    # hybrid attention needs a filter of 1..8 taps (kMaxHybK); the baseline (0 maps) any value
    with pytest.raises(s2s_amd.nn.S2SArgumentError):
        s2s_amd.Attention(s2s_amd.GRU(16, 16), s2s_amd.MaxoutMLP(48, 4, 7, 10), 32, 0, 16, 16, 32, 10, True, 0)
    with pytest.raises(s2s_amd.nn.S2SArgumentError):
        s2s_amd.Attention(s2s_amd.GRU(16, 16), s2s_amd.MaxoutMLP(48, 4, 7, 10), 32, 9, 16, 16, 32, 10, True, 0)
    att = s2s_amd.Attention(s2s_amd.GRU(16, 16), s2s_amd.MaxoutMLP(48, 4, 7, 10), 32, 5, 16, 16, 32, 10, True, 0)
    assert [tuple(t.shape) for t in att.parameters()[0][17:]] == [(16, 5), (16,), (32, 16)]
    with pytest.raises(s2s_amd.nn.S2SArgumentError):
        s2s_amd.RNN(s2s_amd.GRU(5, 10))
