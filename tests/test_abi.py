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


def test_lua_shim_cdef_is_current_and_complete():
    """lua/s2s_ffi.lua's ffi.cdef is generated from include/s2s_hip.h (tools/gen_lua_cdef.py): it must be
    current, declare every function of the header, and carry every #define as a module constant."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_lua_cdef", os.path.join(ROOT, "tools", "gen_lua_cdef.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    shim = open(gen.SHIM).read()
    assert gen.render(shim) == shim, "stale: run python tools/gen_lua_cdef.py"
    cdef = shim[shim.index(gen.BEGIN_CDEF):shim.index(gen.END_CDEF)]
    for name in header_symbols():
        assert re.search(r"\b%s\(" % name, cdef), name
    for k, v in gen.constants():
        assert f"M.{k} = {v}" in shim
    # the Lua wrappers for the module methods the shim replaces (RNN / Attention update* + the model step)
    for fn in ("gru_forward", "gru_backward", "attention_forward", "attention_backward", "attention_views",
               "model_step", "beam_search", "adadelta_step", "ctx_status"):
        assert f"function M.{fn}(" in shim, fn


def _gen():
    import importlib.util
    spec = importlib.util.spec_from_file_location("gen_lua_cdef", os.path.join(ROOT, "tools", "gen_lua_cdef.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    return gen


def test_integration_snippet_cdef_matches_header():
    """INTEGRATION.md's LuaJIT snippet declares its functions exactly as include/s2s_hip.h does (generated by
    tools/gen_lua_cdef.py; round 2's hand-written copy had lost the `lengths` argument of s2s_gru_fwd/bwd),
    and its example calls pass as many arguments as those declarations take."""
    gen = _gen()
    doc = open(gen.INTEGRATION).read()
    assert gen.render_integration(doc) == doc, "stale: run python tools/gen_lua_cdef.py"
    block = doc[doc.index(gen.BEGIN_SNIP):doc.index(gen.END_SNIP)]
    decls = set(gen.declarations())
    funcs = [d for d in block.splitlines() if "(" in d and d.endswith(";")]
    assert len(funcs) == len(gen.SNIPPET_FUNCS)
    for d in funcs:
        assert d in decls, d
    # every C.s2s_*( call in the snippet passes the declared number of arguments
    nargs = {}
    for d in funcs:
        name = re.search(r"(s2s_\w+)\(", d).group(1)
        inner = d[d.index("(") + 1:d.rindex(")")]
        nargs[name] = 0 if inner.strip() in ("", "void") else inner.count(",") + 1
    snippet = doc[doc.index("```lua"):doc.index("```", doc.index("```lua") + 6)]
    calls = 0
    for m in re.finditer(r"C\.(s2s_\w+)\(", snippet):
        depth, i, commas = 1, m.end(), 0
        while depth:
            ch = snippet[i]
            depth += ch in "({"
            depth -= ch in ")}"
            commas += ch == "," and depth == 1
            i += 1
        inner = snippet[m.end():i - 1].strip()
        n = 0 if not inner else commas + 1
        assert n == nargs[m.group(1)], (m.group(1), n, nargs[m.group(1)])
        calls += 1
    assert calls >= 3


def test_ctypes_structs_match_header_typedefs():
    """The ctypes mirrors of s2s_attn_dims / s2s_model_dims / s2s_optim_config list the header's fields in
    order (a silent layout drift would pass garbage lengths / seeds to the kernels)."""
    from s2s_amd import _lib
    hdr = open(os.path.join(ROOT, "include", "s2s_hip.h")).read()
    hdr = re.sub(r"/\*.*?\*/", " ", hdr, flags=re.S)
    for name, cls in (("s2s_attn_dims", _lib.s2s_attn_dims), ("s2s_model_dims", _lib.s2s_model_dims),
                      ("s2s_optim_config", _lib.s2s_optim_config)):
        body = re.search(r"typedef struct \{([^{}]*)\}\s*%s;" % name, hdr).group(1)
        fields = []
        for decl in body.split(";"):
            decl = decl.strip()
            if not decl:
                continue
            names = decl.split(",")
            first = re.findall(r"(\w+)\s*$", names[0].strip())[0]
            fields.append(first)
            fields += [n.strip() for n in names[1:]]
        assert [f for f, _ in cls._fields_] == fields, name


@pytest.mark.gpu
def test_rccl_c_abi_single_rank_allreduce_is_identity():
    """s2s_comm_unique_id / s2s_comm_init / s2s_allreduce_sum (the Lua host's collective, no torch) on one
    rank: the sum over one rank is the identity."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import s2s_amd
    from s2s_amd import _lib
    ctx = s2s_amd.Context(0)
    uid = ctypes.create_string_buffer(_lib.S2S_UNIQUE_ID_BYTES)
    _lib.check(_lib.lib.s2s_comm_unique_id(uid))
    _lib.check(_lib.lib.s2s_comm_init(ctx.handle, uid, 1, 0))
    x = torch.randn(4_356_222, device="cuda")
    ref = x.clone()
    st = torch.cuda.current_stream()
    _lib.check(_lib.lib.s2s_allreduce_sum(ctx.handle, ctypes.c_void_p(st.cuda_stream), ctypes.c_void_p(x.data_ptr()),
                                          x.numel()))
    torch.cuda.synchronize()
    assert torch.equal(x, ref)
    # a null context is an error status, not an abort
    assert _lib.lib.s2s_allreduce_sum(None, None, None, 0) != 0
    assert "null context" in _lib.lib.s2s_last_error().decode()
