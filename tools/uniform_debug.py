#!/usr/bin/env python3
"""Debug: run the golden vectors + random cases through one build of the library and
report mismatches against the CPU build of the core, plus the non-uniform table-load
counters of an ACS_CHECK_UNIFORM build.  usage: uniform_debug.py <lib.so>"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "access-control-srv_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

from acs_mi355x import compiler, encoder, native, store  # noqa: E402
import host_core  # noqa: E402
import randgen  # noqa: E402
from kat_utils import load_kats, load_fixture, urns_for  # noqa: E402
from oracle.acs_oracle import DEFAULT_CAS  # noqa: E402


def main():
    lib = native.load(sys.argv[1])
    dbg = getattr(lib, "acs_debug_read", None)
    buf = (C.c_ulonglong * 4)()
    if dbg:
        dbg.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
        dbg(buf, 4)
    bad = []
    cases = []
    by_fx = {}
    for v in load_kats():
        if v["op"] == "isAllowed":
            by_fx.setdefault((v["fixture"], v["urns"]), []).append(v)
    for (fx, _), vecs in by_fx.items():
        cases.append((f"kat:{fx}", urns_for(vecs[0]), load_fixture(fx), [v["request"] for v in vecs]))
    for seed in range(int(os.environ.get("SEEDS", "150"))):
        urns, doc, reqs = randgen.rand_case(seed)
        cases.append((f"rand:{seed}", urns, doc, reqs))
    n = 0
    for name, urns, doc, reqs in cases:
        cs = compiler.compile_store(store.populate(doc), urns, DEFAULT_CAS)
        b = encoder.Encoder(cs).encode(reqs)
        t = native.Tables(compiler.store_blob(cs), 0)
        got = t.is_allowed(b)
        t.close()
        want = host_core.is_allowed(cs, b)
        n += len(reqs)
        for i in np.flatnonzero(got.view(np.uint64) != want.view(np.uint64)):
            bad.append((name, int(i), tuple(int(x) for x in got[i].tolist()), tuple(int(x) for x in want[i].tolist())))
    res = {"lib": os.path.basename(sys.argv[1]), "requests": n, "mismatches": len(bad), "first": bad[:8]}
    if dbg:
        dbg(buf, 4)
        res["nonuniform_loads"] = {"total": buf[0], "node64": buf[1], "rres16": buf[2], "pair8": buf[3]}
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
