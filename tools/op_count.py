#!/usr/bin/env python3
"""Per-wave attribution of K1's work: how many times the waves execute each evaluation step
(acs_eval.h OpCount), from the -DACS_OP_COUNT build (lib/variants/opcount.so; counts only, its
timing is not K1's).  Each step is counted once per wave that runs it, with the number of lanes
active at that point, so waves / lanes per step give both the per-wave issue count and the SIMD
efficiency of that step.

usage: python tools/op_count.py <c3|c3r1|c2|c5|c3adv> [requests]  -> one JSON object
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "access-control-srv_amd"), os.path.join(ROOT, "tests")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from acs_mi355x import build, compiler, native, store, synth  # noqa: E402
from acs_mi355x.device import DeviceBatch, is_allowed_device, what_is_allowed_device  # noqa: E402
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS  # noqa: E402

OPS = ["set_iter", "set_skip", "set_eval", "set_events", "set_target", "p2a_iter", "p2a_tm", "multi", "p2b_iter",
       "p2b_tm", "p2b_hr", "rule_loop", "rule_iter", "rule_tm", "rule_hr", "rule_acl", "word", "v_lds", "v_own",
       "v_own2", "rows", "rows2", "lane_done", "tpl_req", "tpl_word", "tpl_rule", "tpl_tm", "tpl_hit"]


def batch_for(kind, n):
    mk = {"c2": synth.c2_store, "c3": synth.c3_store, "c3r1": synth.c3_store, "c5": synth.c5_store,
          "c3adv": synth.c3_adverse_store}[kind]
    doc = mk()
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    second = 0.0 if kind in ("c3r1", "c2") else 0.5
    sb = synth.requests(cs, n, "c2" if kind == "c2" else "c3", second_role=second,
                        acl=0.1 if kind == "c3adv" else 0.0, classes=kind != "c3adv")
    if kind == "c3adv":
        from bench import codec_batch
        sb.batch = codec_batch(cs, sb)
    return cs, sb


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "c3"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    path = os.environ.get("ACS_OPCOUNT_LIB") or build.build_variant("opcount", ["ACS_OP_COUNT"])
    lib = native._declare(C.CDLL(path))
    lib.acs_op_read.argtypes = [C.POINTER(C.c_ulonglong), C.c_int]
    cs, sb = batch_for("c3" if kind == "c4" else kind, n)
    blob = compiler.store_blob(cs)

    class _T:  # the duck-typed tables handle device.py's launchers take
        pass
    t = _T()
    t.lib = lib
    t.h = lib.acs_compile(blob, len(blob), 0)
    assert t.h, native.last_error(lib)
    t.words = lib.acs_wia_words_per_request(t.h)
    db = DeviceBatch(sb.batch, 0, compact=True)
    acc = (C.c_ulonglong * (2 * len(OPS)))()
    lib.acs_op_read(acc, len(OPS))  # reset
    if kind == "c4":
        what_is_allowed_device(t, db)
    else:
        is_allowed_device(t, db)
    torch.cuda.synchronize()
    lib.acs_op_read(acc, len(OPS))
    waves = np.array(acc[:len(OPS)], np.float64)
    lanes = np.array(acc[len(OPS):2 * len(OPS)], np.float64)
    # waves that evaluated (reached the end of the walk; c4: took the template path)
    ew = max(waves[OPS.index("tpl_req" if kind == "c4" else "lane_done")], 1.0)
    res = {"config": kind, "requests": n, "evaluating_waves": int(ew),
           "lanes_per_wave": float(lanes[OPS.index("tpl_req" if kind == "c4" else "lane_done")] / ew),
           "per_wave": {o: float(waves[k] / ew) for k, o in enumerate(OPS)},
           "lanes_active": {o: float(lanes[k] / waves[k]) if waves[k] else 0.0 for k, o in enumerate(OPS)}}
    print(json.dumps(res))
    lib.acs_free(t.h)


if __name__ == "__main__":
    main()
