"""The C-ABI library builds, loads without a GPU and exports every entry point
declared in include/*.h; packed struct sizes agree between host and library."""
import ctypes as C
import glob
import os
import re

from acs_mi355x import build, layout, native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(acs_\w+)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return names


def test_library_exports_every_declared_symbol():
    build.build_product()
    lib = native.load()
    decl = declared_functions()
    assert {"acs_compile", "acs_is_allowed", "acs_what_is_allowed", "acs_free", "acs_last_error"} <= decl
    for name in decl:
        assert hasattr(lib, name), name
    assert set(native.EXPORTS) == decl


def test_layout_sizes_match_host_dtypes():
    lib = native.load()
    out = (C.c_uint32 * 5)()
    assert lib.acs_layout_sizes(out, 5) == 5
    names = ["NodeRec", "RuleResAttr", "ReqHdr", "ReqRes", "Decision"]
    assert dict(zip(names, list(out))) == layout.SIZES


def test_blob_roundtrip_rejects_garbage():
    lib = native.load()
    assert not lib.acs_compile(b"\0" * 64, 64, 0)
    assert b"magic" in lib.acs_last_error()
