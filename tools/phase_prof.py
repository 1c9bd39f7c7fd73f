#!/usr/bin/env python3
"""Where K1's time goes: per-phase lane-cycles from the -DACS_PHASE_PROF build.

usage: python tools/phase_prof.py [c2|c3|c5] [requests] [second_role]
Prints, per phase, the share of lane-cycles inside is_allowed_t (set targets, the
exact-policy scan, multi-entity check, policy targets, rule targets, HR, ACL; the
rest is iteration / bookkeeping) and the kernel time of the profiling build.
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "access-control-srv_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from acs_mi355x import build, compiler, native, store, synth  # noqa: E402
from acs_mi355x.device import DeviceBatch, is_allowed_device  # noqa: E402
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS  # noqa: E402

PHASES = ["total", "set_target", "pol_exact_scan", "multi_entity", "pol_target", "rule_target", "rule_hr", "rule_acl"]


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "c2"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    second = float(sys.argv[3]) if len(sys.argv) > 3 else 0.0
    lib_path = build.build_prof()
    lib = native.load(lib_path)
    lib.acs_phase_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    mk = {"c2": synth.c2_store, "c3": synth.c3_store, "c5": synth.c5_store}[kind]
    cs = compiler.compile_store(store.populate(mk()), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, n, "c2" if kind == "c2" else "c3", second_role=second)
    t = native.Tables(compiler.store_blob(cs), 0)
    t.set_timing(True)
    db = DeviceBatch(sb.batch, 0, compact=True)
    out = torch.empty((n, 8), dtype=torch.uint8, device="cuda")
    is_allowed_device(t, db, out)
    torch.cuda.synchronize()
    acc = (C.c_ulonglong * 16)()
    lib.acs_phase_read(acc, 16)  # reset after warmup
    steps = 3
    for _ in range(steps):
        is_allowed_device(t, db, out)
    torch.cuda.synchronize()
    lib.acs_phase_read(acc, 16)
    v = np.array(acc[:len(PHASES)], np.float64)
    tot = v[0]
    res = {"config": kind, "requests": n, "second_role": second, "kernel_ms": float(np.mean(t.kernel_times(steps))),
           "lane_cycles_per_request": tot / (n * steps),
           "share": {p: float(v[k] / tot) for k, p in enumerate(PHASES) if k}}
    res["share"]["iteration_other"] = 1.0 - sum(res["share"].values())
    print(json.dumps(res, indent=1))
    t.close()


if __name__ == "__main__":
    main()
