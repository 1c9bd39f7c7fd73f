#!/usr/bin/env python3
"""Where c3adv's K1 time comes from: 1M requests through the native codec against the c3 and
c3-adverse stores, with and without ACL-bearing context resources (10 %), K1 mean over 20
launches each; then lane orders for the c3adv batch (the codec's padded class runs, unpadded,
and requests that evaluate verifyACL grouped after the rest).  usage: python tools/adv_ab.py
[requests]"""
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


def order(b, acl_major, pad):
    """A coherence order of codec batch b: [acl-eval? | class + 1 | second class], stable; pad:
    each run of equal (acl-eval, class) starts on a 64-lane boundary (holes 0xFFFFFFFF)."""
    flags = b.lines["h"]["flags"].astype(np.int64)
    cls = flags >> 16
    rows = b.cand.shape[0]
    bucket = np.where(cls < rows, cls + 1, 0)
    acl = (((flags >> 11) & 3) == 0).astype(np.int64) if acl_major else np.zeros_like(cls)
    key = (acl << 40) | (bucket << 17) | b.lines["cls2"].astype(np.int64)
    idx = np.argsort(key, kind="stable")
    if not pad:
        return idx.astype(np.uint32)
    run_key = (acl << 20 | bucket)[idx]
    starts = np.flatnonzero(np.concatenate([[True], run_key[1:] != run_key[:-1]]))
    parts = []
    for a, e in zip(starts, np.concatenate([starts[1:], [len(idx)]])):
        parts.append(idx[a:e].astype(np.uint32))
        if (e - a) % 64:
            parts.append(np.full(64 - (e - a) % 64, 0xFFFFFFFF, np.uint32))
    return np.concatenate(parts)


def run(kind, acl, n, second, perms=False):
    cs = compiler.compile_store(store.populate(bench.make_store(kind)), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, n, "c3", seed=0xACC1000, second_role=second, acl=acl, classes=False)
    b = bench.codec_batch(cs, sb)
    if perms:
        res = []
        codec_perm = np.array(b.perm)
        for name, p in (("codec", codec_perm), ("class_nopad", order(b, False, False)),
                        ("acl_last_pad", order(b, True, True)), ("acl_last_nopad", order(b, True, False))):
            b.perm = p
            res.append(dict(run_batch(cs, b, n), order=name, perm_lanes=int(p.size)))
        return res
    return dict(run_batch(cs, b, n), store=kind, acl=acl, second_role=second, classes=int(b.cand.shape[0]),
                perm_lanes=int(b.perm.size))


def run_batch(cs, b, n):
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
    res = {"requests": n, "kernel_ms": ms, "host_cond": float(((flags & 0x02) != 0).mean()),
           "err": float(((flags & 0x01) != 0).mean()), "dec_sum": int(np.ascontiguousarray(dec).view(np.uint64).sum())}
    t.close()
    return res


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    if len(sys.argv) > 2 and sys.argv[2] == "orders":
        for kind, acl in (("c3adv", 0.1), ("c3", 0.0)):
            for r in run(kind, acl, n, 0.5, perms=True):
                print(json.dumps(dict(r, store=kind, acl=acl)), flush=True)
        return
    for kind, acl, second in (("c3", 0.0, 0.5), ("c3", 0.1, 0.5), ("c3adv", 0.0, 0.5), ("c3adv", 0.1, 0.5),
                              ("c3adv", 0.1, 0.0)):
        print(json.dumps(run(kind, acl, n, second)), flush=True)


if __name__ == "__main__":
    main()
