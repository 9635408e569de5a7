"""Regenerate the ffi.cdef block and the constant table of lua/s2s_ffi.lua from include/s2s_hip.h.

The header is the single source of the C ABI; the LuaJIT shim's cdef is the header's declarations with
comments, preprocessor lines and the extern "C" wrapper removed (LuaJIT's ffi.cdef parses plain C
declarations, not #define), and the #define constants become fields of the module table.
tests/test_abi.py checks the committed shim against this generator.

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


def render(shim):
    for (b, e), block in (((BEGIN_CDEF, END_CDEF), cdef_block()), ((BEGIN_CONST, END_CONST), const_block())):
        i, j = shim.index(b), shim.index(e) + len(e)
        shim = shim[:i] + block + shim[j:]
    return shim


def main():
    shim = open(SHIM).read()
    new = render(shim)
    if "--check" in sys.argv:
        if new != shim:
            print("lua/s2s_ffi.lua is stale: run python tools/gen_lua_cdef.py")
            return 1
        return 0
    if new != shim:
        open(SHIM, "w").write(new)
    return 0


if __name__ == "__main__":
    sys.exit(main())
