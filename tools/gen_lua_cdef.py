"""Regenerate the ffi.cdef block and the constant table of lua/s2s_ffi.lua, and the cdef block of
INTEGRATION.md's LuaJIT snippet, from include/s2s_hip.h.

The header is the single source of the C ABI; the LuaJIT shim's cdef is the header's declarations with
comments, preprocessor lines and the extern "C" wrapper removed (LuaJIT's ffi.cdef parses plain C
declarations, not #define), and the #define constants become fields of the module table.
INTEGRATION.md's snippet declares the subset of the header a maintainer's nn.RNN binding needs (SNIPPET_FUNCS),
generated the same way.  tests/test_abi.py checks both committed files against this generator.

  python tools/gen_lua_cdef.py          # rewrite the generated sections in place
  python tools/gen_lua_cdef.py --check  # exit 1 if they are stale
"""
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "s2s_hip.h")
SHIM = os.path.join(ROOT, "seq2seq-attention-asr_amd", "lua", "s2s_ffi.lua")
BEGIN_CDEF, END_CDEF = "-- BEGIN GENERATED CDEF (tools/gen_lua_cdef.py)", "-- END GENERATED CDEF"
BEGIN_CONST, END_CONST = "-- BEGIN GENERATED CONSTANTS (tools/gen_lua_cdef.py)", "-- END GENERATED CONSTANTS"
INTEGRATION = os.path.join(ROOT, "INTEGRATION.md")
BEGIN_SNIP, END_SNIP = "-- BEGIN GENERATED SUBSET (tools/gen_lua_cdef.py)", "-- END GENERATED SUBSET"
SNIPPET_FUNCS = ("s2s_last_error", "s2s_ctx_create", "s2s_ctx_status", "s2s_gru_saved_bytes", "s2s_gru_scratch_bytes",
                 "s2s_gru_fwd", "s2s_gru_bwd")


def header_text():
    return open(HEADER).read()


def declarations(text=None):
    """The header's C declarations, one per line, comments / preprocessor / extern "C" removed."""
    text = header_text() if text is None else text
    text = re.sub(r"/\*.*?\*/", " ", text, flags=re.S)
    text = re.sub(r"//[^\n]*", " ", text)
    lines = []
    for ln in text.splitlines():
        s = ln.strip()
        if not s or s.startswith("#") or s in ('extern "C" {', "}"):
            continue
        lines.append(s)
    decls, cur = [], ""
    depth = 0
    for s in lines:
        cur = (cur + " " + s).strip()
        depth += s.count("{") - s.count("}")
        if depth == 0 and cur.endswith(";"):
            decls.append(re.sub(r"\s+", " ", cur))
            cur = ""
    return decls


def constants(text=None):
    text = header_text() if text is None else text
    return re.findall(r"^#define\s+(S2S_[A-Z0-9_]+)\s+(\d+)\s*$", text, flags=re.M)


def functions(text=None):
    """Names of the functions the header declares."""
    out = []
    for d in declarations(text):
        if d.startswith("typedef"):
            continue
        m = re.search(r"([A-Za-z_][A-Za-z0-9_]*)\s*\(", d)
        if m:
            out.append(m.group(1))
    return out


def cdef_block():
    body = "\n".join(declarations())
    return f"{BEGIN_CDEF}\nffi.cdef[[\n{body}\n]]\n{END_CDEF}"


def const_block():
    body = "\n".join(f"M.{k} = {v}" for k, v in constants())
    return f"{BEGIN_CONST}\n{body}\n{END_CONST}"


def snippet_block():
    keep = []
    for d in declarations():
        if d.startswith("typedef"):
            if "{" not in d:  # the opaque context and stream types; the dims structs are not needed here
                keep.append(d)
            continue
        m = re.search(r"([A-Za-z_][A-Za-z0-9_]*)\s*\(", d)
        if m and m.group(1) in SNIPPET_FUNCS:
            keep.append(d)
    body = "\n".join(keep)
    return f"{BEGIN_SNIP}\nffi.cdef[[\n{body}\n]]\n{END_SNIP}"


def render_integration(doc):
    i, j = doc.index(BEGIN_SNIP), doc.index(END_SNIP) + len(END_SNIP)
    return doc[:i] + snippet_block() + doc[j:]


def render(shim):
    for (b, e), block in (((BEGIN_CDEF, END_CDEF), cdef_block()), ((BEGIN_CONST, END_CONST), const_block())):
        i, j = shim.index(b), shim.index(e) + len(e)
        shim = shim[:i] + block + shim[j:]
    return shim


def main():
    rc = 0
    for path, fn in ((SHIM, render), (INTEGRATION, render_integration)):
        old = open(path).read()
        new = fn(old)
        if "--check" in sys.argv:
            if new != old:
                print(f"{os.path.relpath(path, ROOT)} is stale: run python tools/gen_lua_cdef.py")
                rc = 1
        elif new != old:
            open(path, "w").write(new)
    return rc


if __name__ == "__main__":
    sys.exit(main())
