#!/usr/bin/env python3
"""K1 (K2 for c4) on the encoder's coherence order with and without its wave-aligned class runs
(the holes dropped from the order: classes then share waves), same batch, same tables, launches
alternated; outputs compared.  usage: python tools/pad_ab.py <c3adv|c3|c3r1|c2|c4> <requests>"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "access-control-srv_amd"), os.path.join(ROOT, "tests"),
                os.path.join(ROOT, "tools")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from acs_mi355x import compiler, native  # noqa: E402
from acs_mi355x.device import DeviceBatch, is_allowed_device, what_is_allowed_device  # noqa: E402


class Unpadded:
    """The batch with its coherence order's holes removed (everything else delegated)."""

    def __init__(self, b):
        self._b = b
        p = np.asarray(b.perm)
        self.perm = np.ascontiguousarray(p[p < b.n])

    def __getattr__(self, k):
        return getattr(self._b, k)


def main():
    import op_count
    kind, n = sys.argv[1], int(sys.argv[2])
    what = kind == "c4"
    cs, sb = op_count.batch_for("c3" if what else kind, n)

    def run(db, out=None):
        return what_is_allowed_device(t, db, out) if what else is_allowed_device(t, db, out)
    t = native.Tables(compiler.store_blob(cs), 0)
    t.set_timing(True)
    dbs = {"padded": DeviceBatch(sb.batch, 0, compact=True), "unpadded": DeviceBatch(Unpadded(sb.batch), 0, compact=True)}
    lanes = {"padded": int(len(sb.batch.perm)), "unpadded": int(n)}
    outs, times = {}, {k: [] for k in dbs}
    for k, db in dbs.items():
        outs[k] = run(db)
    torch.cuda.synchronize()
    for _ in range(10):
        for k, db in dbs.items():
            outs[k] = run(db, outs[k])
            torch.cuda.synchronize()
            times[k].append(float(t.kernel_times(1)[0]))
    pick = (lambda o: [o[0], o[2], o[3]]) if what else (lambda o: [o])
    same = all(np.array_equal(a.cpu().numpy(), b.cpu().numpy()) for a, b in zip(pick(outs["padded"]), pick(outs["unpadded"])))
    print(json.dumps({"config": kind, "requests": n, "lanes": lanes, "identical": bool(same),
                      "mean_ms": {k: float(np.mean(v)) for k, v in times.items()},
                      "min_ms": {k: float(np.min(v)) for k, v in times.items()}}))
    t.close()


if __name__ == "__main__":
    main()
