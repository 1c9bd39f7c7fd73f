#!/usr/bin/env python3
"""Same-process A/B of the obligation-only pass's range count (resolve_overflow_device `chunks`):
one c4 batch through K2, then the pass for its overflowed logs at each chunk count, alternated,
timed with the stream synchronized around each pass; the joined logs compared across counts.

usage: python tools/obl_ab.py [requests] [chunks ...]   (default 1000000 16 32 64)
"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "access-control-srv_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from acs_mi355x import compiler, native  # noqa: E402
from acs_mi355x.device import DeviceBatch, what_is_allowed_device, resolve_overflow_device, overflow_logs  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    counts = [int(x) for x in sys.argv[2:]] or [16, 32, 64]
    reps = int(os.environ.get("AB_REPS", "10"))
    import op_count
    cs, sb = op_count.batch_for("c3", n)
    t = native.Tables(compiler.store_blob(cs), 0)
    db = DeviceBatch(sb.batch, 0, compact=True)
    st = torch.cuda.current_stream()
    bufs = what_is_allowed_device(t, db, None, st)
    torch.cuda.synchronize()
    times = {c: [] for c in counts}
    logs = {}
    for c in counts:  # warm
        resolve_overflow_device(t, db, bufs, chunks=c, stream=st)
    torch.cuda.synchronize()
    for _ in range(reps):
        for c in counts:
            t0 = time.perf_counter()
            passes = resolve_overflow_device(t, db, bufs, chunks=c, stream=st)
            torch.cuda.synchronize()
            times[c].append((time.perf_counter() - t0) * 1e3)
            logs[c] = passes
    ref = overflow_logs(logs[counts[0]])
    out = {"requests": n, "overflowed": len(ref), "reps": reps, "chunks": {}}
    for c in counts:
        got = overflow_logs(logs[c])
        same = got.keys() == ref.keys() and all(np.array_equal(got[k], ref[k]) for k in ref)
        out["chunks"][str(c)] = {"mean_ms": float(np.mean(times[c])), "min_ms": float(np.min(times[c])),
                                 "identical_to_first": bool(same)}
    print(json.dumps(out))
    t.close()


if __name__ == "__main__":
    main()
