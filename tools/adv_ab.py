#!/usr/bin/env python3
"""Where c3adv's K1 time comes from: 1M requests through the native codec against the c3 and
c3-adverse stores, with and without ACL-bearing context resources (10 %), K1 mean over 20
launches each.  usage: python tools/adv_ab.py [requests]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "access-control-srv_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from acs_mi355x import compiler, native, store, synth  # noqa: E402
from acs_mi355x.device import DeviceBatch, decisions_from_tensor, is_allowed_device  # noqa: E402
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS  # noqa: E402


def run(kind, acl, n, second):
    cs = compiler.compile_store(store.populate(bench.make_store(kind)), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, n, "c3", seed=0xACC1000, second_role=second, acl=acl, classes=False)
    b = bench.codec_batch(cs, sb)
    t = native.Tables(compiler.store_blob(cs), 0)
    t.set_timing(True)
    db = DeviceBatch(b, 0, compact=True)
    out = torch.empty((n, 8), dtype=torch.uint8, device="cuda")
    for _ in range(3):
        is_allowed_device(t, db, out)
    torch.cuda.synchronize()
    steps = 20
    for _ in range(steps):
        is_allowed_device(t, db, out)
    torch.cuda.synchronize()
    ms = float(np.mean(t.kernel_times(steps)))
    dec = decisions_from_tensor(out)
    flags = dec["flags"]
    res = {"store": kind, "acl": acl, "second_role": second, "requests": n, "classes": int(b.cand.shape[0]),
           "perm_lanes": int(b.perm.size), "kernel_ms": ms,
           "host_cond": float(((flags & 0x02) != 0).mean()), "err": float(((flags & 0x01) != 0).mean())}
    t.close()
    return res


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    for kind, acl, second in (("c3", 0.0, 0.5), ("c3", 0.1, 0.5), ("c3adv", 0.0, 0.5), ("c3adv", 0.1, 0.5),
                              ("c3adv", 0.1, 0.0)):
        print(json.dumps(run(kind, acl, n, second)), flush=True)


if __name__ == "__main__":
    main()
