#!/usr/bin/env python3
"""SIMD efficiency of a lane order (test infrastructure, CPU only): the CPU build of the
evaluator core counting, per request, the table bytes its evaluation reads
(-DACS_HOST_WORK), then per 64-lane wave of an order: sum(work) / (64 x max(work)) — the share of
a wave's lane-time that does work when every lane runs as long as the wave's longest.
This ignores the union of the wave's candidate rows: grouping c3adv's ACL requests after the
rest raised this figure 0.22 -> 0.70 but made K1 slower on the GPU (3.3 -> 4.7 ms, the ACL waves
mixing many classes; profiles/r04_h), so it ranks orders only among class-coherent ones.
usage: python tools/lane_work.py <c3|c3adv|c4> [requests] [second_role]"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "access-control-srv_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402

import bench  # noqa: E402
from acs_mi355x import build, compiler, native, store, synth  # noqa: E402
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS  # noqa: E402

LIB = os.path.join(ROOT, "tests", "native", "libacs_core_host_work.so")


def lib():
    src = os.path.join(ROOT, "tests", "native", "core_host.hip")
    if build._stale(LIB, [src] + build._HEADERS):
        build._hipcc(src, LIB, ("-DACS_HOST_WORK",))
    L = C.CDLL(LIB)
    vp = C.c_void_p
    L.acs_host_is_allowed_work.argtypes = [vp, C.c_size_t, vp, vp, vp]
    L.acs_host_what_is_allowed_work.argtypes = [vp, C.c_size_t, vp, vp]
    return L


def wave_stats(work, perm):
    p = perm[perm != 0xFFFFFFFF] if perm is not None else np.arange(len(work))
    lanes = np.full(((len(perm) + 63) // 64) * 64, -1, np.int64) if perm is not None else None
    if perm is not None:
        lanes[:len(perm)] = np.where(perm == 0xFFFFFFFF, -1, perm.astype(np.int64))
    else:
        lanes = np.full(((len(work) + 63) // 64) * 64, -1, np.int64)
        lanes[:len(work)] = np.arange(len(work))
    w = np.where(lanes >= 0, work[np.maximum(lanes, 0)], 0).reshape(-1, 64)
    mx = w.max(axis=1)
    return {"waves": int(w.shape[0]), "work": float(work.sum()), "lane_time": float(64 * mx.sum()),
            "efficiency": float(work.sum() / max(1, 64 * mx.sum()))}


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "c3"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 200_000
    second = float(sys.argv[3]) if len(sys.argv) > 3 else 0.5
    L = lib()
    store_kind = "c3" if kind == "c4" else kind
    cs = compiler.compile_store(store.populate(bench.make_store(store_kind if kind != "c4" else "c4")),
                                FULL_URNS, DEFAULT_CAS)
    acl = 0.1 if kind == "c3adv" else 0.0
    sb = synth.requests(cs, n, "c3", seed=0xACC1000, second_role=second, acl=acl, classes=False)
    b = bench.codec_batch(cs, sb)
    blob = compiler.store_blob(cs)
    s = native.host_struct(b, True)
    work = np.zeros(n, np.uint64)
    if kind == "c4":
        assert L.acs_host_what_is_allowed_work(blob, len(blob), C.addressof(s), work.ctypes.data) == 0
    else:
        out = np.zeros(n * 8, np.uint8)
        assert L.acs_host_is_allowed_work(blob, len(blob), C.addressof(s), out.ctypes.data, work.ctypes.data) == 0
    work = work.astype(np.float64)
    flags = b.lines["h"]["flags"].astype(np.int64)
    acl_eval = ((flags >> 11) & 3) == 0
    res = {"config": kind, "requests": n, "second_role": second, "classes": int(b.cand.shape[0]),
           "mean_work": float(work.mean()), "p50": float(np.percentile(work, 50)), "p99": float(np.percentile(work, 99)),
           "acl_eval_share": float(acl_eval.mean()),
           "mean_work_acl": float(work[acl_eval].mean()) if acl_eval.any() else 0.0,
           "orders": {}}
    st = (flags >> 11) & 3  # verifyACL state (acs_layout.h AclState): share, mean work
    res["acl_states"] = {name: [float((st == v).mean()), float(work[st == v].mean()) if (st == v).any() else 0.0]
                         for v, name in enumerate(("continue", "ret_true", "ret_false", "none"))}
    perm = np.array(b.perm)
    pl = np.full(((len(perm) + 63) // 64) * 64, -1, np.int64)
    pl[:len(perm)] = np.where(perm == 0xFFFFFFFF, -1, perm.astype(np.int64))
    pl = pl.reshape(-1, 64)
    wmax = np.where(pl >= 0, work[np.maximum(pl, 0)], 0).max(axis=1)
    has = (np.where(pl >= 0, acl_eval[np.maximum(pl, 0)], False)).any(axis=1)
    res["codec_waves_with_acl_eval"] = [float(has.mean()), float(wmax[has].sum() / max(1, wmax.sum()))]
    res["orders"]["codec"] = wave_stats(work, np.array(b.perm))
    cls = flags >> 16
    cls2 = b.lines["cls2"].astype(np.int64)
    rows = b.cand.shape[0]
    bucket = np.where(cls < rows, cls + 1, 0)
    key = (bucket << 17) | cls2
    res["orders"]["class"] = wave_stats(work, np.argsort(key, kind="stable").astype(np.uint32))
    res["orders"]["acl_then_class"] = wave_stats(
        work, np.argsort((acl_eval.astype(np.int64) << 40) | key, kind="stable").astype(np.uint32))
    # class-level expected work known (upper bound of any per-class ordering)
    cmean = np.bincount(key.astype(np.int64) % 1000003, weights=work, minlength=1000003) / np.maximum(
        1, np.bincount(key.astype(np.int64) % 1000003, minlength=1000003))
    ew = cmean[key % 1000003]
    res["orders"]["by_class_mean_work"] = wave_stats(work, np.lexsort((key, ew)).astype(np.uint32))
    res["orders"]["acl_then_class_mean"] = wave_stats(work, np.lexsort((key, ew, acl_eval)).astype(np.uint32))
    res["orders"]["sorted_by_work"] = wave_stats(work, np.argsort(work, kind="stable").astype(np.uint32))
    res["orders"]["request_order"] = wave_stats(work, None)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
