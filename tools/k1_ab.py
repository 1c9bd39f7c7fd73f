#!/usr/bin/env python3
"""Same-process A/B of library builds on one resident batch: K1 (isAllowed) or K2
(whatIsAllowed) launch times, alternating builds launch by launch (ABAB...), records compared
bit for bit across builds.

usage: python tools/k1_ab.py <c3|c3r1|c2|c3adv|c4|c5> <requests> <lib> [<lib> ...]
  lib: a path, or a name under access-control-srv_amd/lib/variants (``product``: the product
  library).  Prints one JSON object: per build the mean / min kernel ms over the timed launches.
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "access-control-srv_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from acs_mi355x import build, compiler, native  # noqa: E402
from acs_mi355x.device import DeviceBatch, is_allowed_device, what_is_allowed_device  # noqa: E402


def lib_path(name):
    if name == "product":
        return build.LIB
    if os.path.sep in name or name.endswith(".so"):
        return name
    return os.path.join(build.PKG, "lib", "variants", name + ".so")


def main():
    kind, n = sys.argv[1], int(sys.argv[2])
    names = sys.argv[3:]
    reps = int(os.environ.get("AB_REPS", "10"))
    import op_count
    what = kind == "c4"
    cs, sb = op_count.batch_for("c3" if what else kind, n)
    blob = compiler.store_blob(cs)
    db = DeviceBatch(sb.batch, 0, compact=True)
    tabs = []
    for nm in names:
        t = native.Tables(blob, 0, lib=native.load(lib_path(nm)))
        t.set_timing(True)
        tabs.append(t)
    stream = torch.cuda.current_stream()
    outs = [None] * len(tabs)

    def run(k):
        if what:
            outs[k] = what_is_allowed_device(tabs[k], db, outs[k], stream)
        else:
            outs[k] = is_allowed_device(tabs[k], db, outs[k], stream)

    for k in range(len(tabs)):  # warm
        run(k)
        run(k)
    torch.cuda.synchronize()
    times = [[] for _ in tabs]
    for _ in range(reps):
        for k in range(len(tabs)):
            run(k)
            torch.cuda.synchronize()
            times[k].append(float(tabs[k].kernel_times(1)[0]))
    # whatIsAllowed: bitsets, log lengths and records (log entries past a count are unspecified)
    pick = (lambda o: [o[0], o[2], o[3]]) if what else (lambda o: [o])
    ref = [x.cpu().numpy() for x in pick(outs[0])]
    same = []
    for k in range(len(tabs)):
        got = [x.cpu().numpy() for x in pick(outs[k])]
        same.append(all(np.array_equal(a, b) for a, b in zip(got, ref)))
    res = {"config": kind, "requests": n, "kernel": "K2" if what else "K1", "reps": reps,
           "builds": {nm: {"mean_ms": float(np.mean(t)), "min_ms": float(np.min(t)), "identical_to_first": s}
                      for nm, t, s in zip(names, times, same)}}
    print(json.dumps(res))
    for t in tabs:
        t.close()


if __name__ == "__main__":
    main()
