#!/usr/bin/env python3
"""whatIsAllowed through host buffers (acs_what_is_allowed): c4-shaped batch (c3 store, 1-2 role
associations), wall time per call and the device-to-host bytes the call moves — rows, log lengths,
records and the packed logs (obl_n entries of 8 B each) — against the full 128-entry log slots.

usage: python tools/wia_host_rate.py [requests]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "access-control-srv_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

from acs_mi355x import compiler, native, store, synth, layout as L  # noqa: E402
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    cs = compiler.compile_store(store.populate(synth.c3_store()), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, n, "c3", second_role=0.5)
    t = native.Tables(compiler.store_blob(cs), 0)
    t.what_is_allowed(sb.batch, compact=True)  # warm
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        bits, obl, obl_n, out = t.what_is_allowed(sb.batch, compact=True)
        times.append(time.perf_counter() - t0)
    words = t.words
    entries = int(np.minimum(obl_n, L.OBL_MAX).sum())
    d2h = n * (4 * words + 4 + 8) + 8 * entries
    full = n * (4 * words + 4 + 8 + 8 * L.OBL_MAX)
    print(json.dumps({"requests": n, "ms": 1e3 * min(times), "words_per_request": words,
                      "obligation_entries_mean": entries / n, "d2h_bytes_per_request": d2h / n,
                      "bound_bytes_per_request": 4 * words + 8 * entries / n + 12,
                      "full_slots_bytes_per_request": full / n}))
    t.close()


if __name__ == "__main__":
    main()
