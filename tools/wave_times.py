#!/usr/bin/env python3
"""Where K2's launch time goes, per wave: the -DACS_WAVE_TIMES build records each wave's first
start and last end (100 MHz wall clock), its first lane's class and its live lanes.

usage: python tools/wave_times.py [requests] [lib]
Prints the launch span, the wave-duration distribution, the longest waves with their class,
the class's candidate counts (sets / policies / rules in its class row) and lane count, and
how the launch span compares with the sum of wave durations per wave slot.
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
from acs_mi355x.device import DeviceBatch, what_is_allowed_device  # noqa: E402
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS  # noqa: E402

WT_MAX = 1 << 16


def popc(a):
    return int(np.unpackbits(np.ascontiguousarray(a).view(np.uint8)).sum())


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    lib_path = sys.argv[2] if len(sys.argv) > 2 else build.build_variant("wavetimes", ["ACS_WAVE_TIMES=1"])
    lib = native.load(lib_path)
    U64, U32 = C.POINTER(C.c_ulonglong), C.POINTER(C.c_uint)
    lib.acs_wave_times_read.argtypes = [U64, U64, U32, U32, C.c_int]
    cs = compiler.compile_store(store.populate(synth.c3_store()), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, n, "c3", seed=0xACC1004)
    t = native.Tables(compiler.store_blob(cs), 0, lib=lib)
    t.set_timing(True)
    db = DeviceBatch(sb.batch, 0, compact=True)
    stream = torch.cuda.current_stream()
    bufs = what_is_allowed_device(t, db, None, stream)
    torch.cuda.synchronize()
    a = np.zeros(WT_MAX, np.uint64)
    b = np.zeros(WT_MAX, np.uint64)
    cls = np.zeros(WT_MAX, np.uint32)
    lanes = np.zeros(WT_MAX, np.uint32)

    def read():
        lib.acs_wave_times_read(a.ctypes.data_as(U64), b.ctypes.data_as(U64), cls.ctypes.data_as(U32),
                                lanes.ctypes.data_as(U32), WT_MAX)

    read()  # reset (the arrays start zeroed: the first read's values are meaningless)
    what_is_allowed_device(t, db, bufs, stream)
    torch.cuda.synchronize()
    read()
    kern_ms = float(t.kernel_times(1)[0])
    live = (lanes > 0) & (b > 0)
    w = np.flatnonzero(live)
    t0, t1 = a[w].astype(np.int64), b[w].astype(np.int64)
    dur_us = (t1 - t0) / 100.0
    span_us = (t1.max() - t0.min()) / 100.0
    B = sb.batch
    cand = getattr(B, "cand", None)
    res = {"requests": n, "waves": int(len(w)), "kernel_ms": kern_ms, "span_us": float(span_us),
           "dur_us": {q: float(np.percentile(dur_us, q)) for q in (0, 10, 50, 90, 99, 99.9, 100)},
           "sum_dur_us": float(dur_us.sum()), "mean_lanes": float(lanes[w].mean())}
    # when did the longest waves start (a late start + a long wave = the tail)
    order = np.argsort(-dur_us)[:25]
    top = []
    for j in order:
        c = int(cls[w[j]])
        row = {"wave": int(w[j]), "dur_us": float(dur_us[j]), "start_us": float((t0[j] - t0.min()) / 100.0),
               "cls": c, "lanes": int(lanes[w[j]])}
        if cand is not None and c < cand.shape[0]:
            row["cand_bits"] = popc(cand[c])
        top.append(row)
    res["top"] = top
    # duration by start time decile: does the tail come from waves that start late?
    st = (t0 - t0.min()) / 100.0
    res["late_starters"] = {"start_after_50pct_span": int((st > span_us / 2).sum()),
                            "ends_after_90pct_span": int(((t1 - t0.min()) / 100.0 > 0.9 * span_us).sum())}
    print(json.dumps(res, indent=1))
    t.close()


if __name__ == "__main__":
    main()
