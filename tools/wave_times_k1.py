#!/usr/bin/env python3
"""What bounds K1 on a small batch: per-wave durations from the -DACS_WAVE_TIMES build
(lib/variants/wavetimes.so: each wave's first start / last end on the 100 MHz wall clock, its
smallest class, its live lanes) next to what each wave holds — its requests' table bytes by the
host core's count (-DACS_HOST_WORK), how many of its lanes are composed (two class rows), how many
distinct classes, and its lanes' decisions.

usage: python tools/wave_times_k1.py [requests] [second_role]  -> one JSON object
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "access-control-srv_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from acs_mi355x import build, compiler, native, store, synth  # noqa: E402
from acs_mi355x.device import DeviceBatch, is_allowed_device, decisions_from_tensor  # noqa: E402
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS  # noqa: E402

WT_MAX = 1 << 16


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 131072
    second = float(sys.argv[2]) if len(sys.argv) > 2 else 0.5
    lib = native.load(os.environ.get("ACS_WT_LIB") or build.build_variant("wavetimes", ["ACS_WAVE_TIMES=1"]))
    U64, U32 = C.POINTER(C.c_ulonglong), C.POINTER(C.c_uint)
    lib.acs_wave_times_read.argtypes = [U64, U64, U32, U32, C.c_int]
    cs = compiler.compile_store(store.populate(synth.c3_store()), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, n, "c3", seed=0xACC1000, second_role=second)
    b = sb.batch
    t = native.Tables(compiler.store_blob(cs), 0, lib=lib)
    t.set_timing(True)
    db = DeviceBatch(b, 0, compact=True)
    out = torch.empty((n, 8), dtype=torch.uint8, device="cuda")
    a = np.zeros(WT_MAX, np.uint64)
    e = np.zeros(WT_MAX, np.uint64)
    cls = np.zeros(WT_MAX, np.uint32)
    lanes = np.zeros(WT_MAX, np.uint32)

    def read():
        lib.acs_wave_times_read(a.ctypes.data_as(U64), e.ctypes.data_as(U64), cls.ctypes.data_as(U32),
                                lanes.ctypes.data_as(U32), WT_MAX)

    is_allowed_device(t, db, out)
    torch.cuda.synchronize()
    read()  # reset
    spans = []
    for _ in range(3):
        is_allowed_device(t, db, out)
        torch.cuda.synchronize()
        spans.append(float(t.kernel_times(1)[0]))
    is_allowed_device(t, db, out)
    torch.cuda.synchronize()
    kern_ms = float(t.kernel_times(1)[0])
    read()
    dec = decisions_from_tensor(out)
    live = (lanes > 0) & (e > 0) & (e >= a)
    w_idx = np.flatnonzero(live)
    dur_us = (e[live] - a[live]).astype(np.float64) / 100.0  # 100 MHz ticks -> us
    start_us = (a[live] - a[live].min()).astype(np.float64) / 100.0
    perm = b.perm if getattr(b, "perm", None) is not None else np.arange(n, dtype=np.uint32)
    lanes_of = np.full(((len(perm) + 63) // 64) * 64, 0xFFFFFFFF, np.uint32)
    lanes_of[:len(perm)] = perm
    lanes_of = lanes_of.reshape(-1, 64)
    # host core's per-request table bytes
    import lane_work
    L = lane_work.lib()
    blob = compiler.store_blob(cs)
    work = np.zeros(n, np.uint64)
    hd = np.zeros(n, np.uint64)
    s = native.batch_struct(b)
    assert L.acs_host_is_allowed_work(blob, len(blob), C.byref(s), hd.ctypes.data, work.ctypes.data) == 0
    cls2 = b.lines["cls2"]
    pcol = b.lines["h"]["flags"] >> np.uint32(16)

    def wave_info(w):
        req = lanes_of[w]
        req = req[req != 0xFFFFFFFF]
        wk = work[req].astype(np.float64)
        return {"lanes": int(len(req)), "composed": int((cls2[req] != 0).sum()),
                "classes": int(len(np.unique(pcol[req]))),
                "pairs": int(len(np.unique(pcol[req].astype(np.uint64) << 32 | cls2[req]))),
                "work_max": float(wk.max()) if len(wk) else 0.0, "work_mean": float(wk.mean()) if len(wk) else 0.0,
                "decisions": np.bincount(dec["decision"][req], minlength=7)[[2, 3, 5]].tolist()}

    order = np.argsort(-dur_us)
    info = [wave_info(int(w)) for w in w_idx]
    wmax = np.array([x["work_max"] for x in info])
    wmean = np.array([x["work_mean"] for x in info])
    comp = np.array([x["composed"] for x in info])
    pairs = np.array([x["pairs"] for x in info])
    res = {"requests": n, "second_role": second, "kernel_ms": kern_ms, "kernel_ms_runs": spans, "waves": int(live.sum()),
           "wave_us": {"p50": float(np.percentile(dur_us, 50)), "p90": float(np.percentile(dur_us, 90)),
                       "p99": float(np.percentile(dur_us, 99)), "max": float(dur_us.max()),
                       "mean": float(dur_us.mean())},
           "start_us_max": float(start_us.max()), "span_us": float((e[live].max() - a[live].min()) / 100.0),
           "corr_dur_work_max": float(np.corrcoef(dur_us, wmax)[0, 1]),
           "corr_dur_work_mean": float(np.corrcoef(dur_us, wmean)[0, 1]),
           "corr_dur_composed": float(np.corrcoef(dur_us, comp)[0, 1]),
           "corr_dur_pairs": float(np.corrcoef(dur_us, pairs)[0, 1]),
           "slowest": [dict(wave=int(w_idx[k]), us=float(dur_us[k]), start_us=float(start_us[k]), **info[k])
                       for k in order[:15]],
           "fastest_median_like": [dict(wave=int(w_idx[k]), us=float(dur_us[k]), **info[k])
                                   for k in order[len(order) // 2: len(order) // 2 + 5]]}
    print(json.dumps(res))
    t.close()


if __name__ == "__main__":
    main()
