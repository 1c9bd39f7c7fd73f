#!/usr/bin/env python3
"""Benchmark: isAllowed decisions/sec of the MI355X evaluator (BASELINE.json metric).

A step = one K1 launch evaluating one full batch of synthetic requests that is
already resident in HBM (default: c2 = 1M requests x 1k rules, flat roles,
SURVEY.md §8(d)).  Multi-GPU: one process per GPU (torch.distributed.run), each
rank evaluates its own 1M-request shard against replicated tables (weak
scaling, no data-path collective); timing = barrier + sync on both sides, max
over ranks.  Rank 0 prints one JSON line with the roofline and CPU-baseline
objects described in DESIGN.md.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, os.path.join(ROOT, "access-control-srv_amd"), os.path.join(ROOT, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

WORKLOADS = {
    "c2": ("c2: isAllowed, 1M requests/GPU vs 100 policy sets / 200 policies / 1k rules, flat roles", 1_000_000),
    "c3": ("c3: isAllowed, 10M requests/GPU vs 10k rules, mixed CAs + HR role scoping (depth-8 org tree)", 10_000_000),
}
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s


def algorithmic_bytes(cs, batch):
    """Per-decision algorithmic bytes: B_req + B_ctx + B_out + B_scan/64."""
    h = batch.hdr
    b_req = 16 + 16 * h["nres"].astype(np.float64) + 8 * h["nsubj"] + 8 * h["nact"] + 4 * h["nroles"]
    # context arena words actually owned per request (shared arenas count once per request anyway)
    if batch.n > 1 and h["arena_off"][-1] > 0:
        ctx = batch.arena.size * 4.0 / batch.n
    else:
        ctx = float(batch.arena.size * 4)
    b_scan = float(cs.table_bytes())  # brute-force tile: the whole table per 64-request wave
    per = float(b_req.mean()) + ctx + 8.0 + b_scan / 64.0
    return per, {"B_req": float(b_req.mean()), "B_ctx": ctx, "B_out": 8.0, "B_scan_per_tile": b_scan, "T": 64}


def cpu_baseline(kind, doc, sb, gpu_dec, cs, seconds):
    """Oracle ('port') timed on a bounded sample of the same workload, single core;
    the same sample is checked against the GPU decisions."""
    from oracle.acs_oracle import Oracle, FULL_URNS
    from diff_utils import oracle_outcome, gpu_outcome
    o = Oracle(FULL_URNS)
    o.load(doc)
    rng = np.random.default_rng(1234)
    idx = rng.permutation(sb.batch.n)
    reqs = []
    mism = 0
    t0 = time.perf_counter()
    done = 0
    for i in idx:
        q = sb.decode(int(i))
        t1 = time.perf_counter()
        w = oracle_outcome(o, q)
        done += 1
        reqs.append(time.perf_counter() - t1)
        if w != gpu_outcome(cs, gpu_dec[i]):
            mism += 1
        if time.perf_counter() - t0 > seconds:
            break
    busy = sum(reqs)
    return {"value": done / busy, "unit": "decisions/s", "cores": 1, "kind": "port",
            "sample": f"{done} random requests of the same {kind} batch through oracle/acs_oracle.py "
                      f"(Python restatement of the reference TS, 1 thread), {busy:.1f}s of CPU work"}, \
        {"oracle_sample": done, "mismatches": mism}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c2", choices=sorted(WORKLOADS))
    ap.add_argument("--requests", type=int, default=0, help="requests per GPU (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-sort", action="store_true", help="disable the (entity, role, action) coherence sort")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)

    from acs_mi355x import compiler, native, store, synth
    from acs_mi355x.device import DeviceBatch, is_allowed_device, decisions_from_tensor
    from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS

    kind = args.config
    desc, n_default = WORKLOADS[kind]
    n = args.requests or n_default
    doc = synth.c2_store() if kind == "c2" else synth.c3_store()
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, n, kind, seed=0xACC1000 + 17 * rank)
    tables = native.Tables(compiler.store_blob(cs), local)
    tables.set_sort(not args.no_sort)
    tables.set_timing(True)
    db = DeviceBatch(sb.batch, local)
    out = torch.empty((n, 8), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)

    for _ in range(args.warmup):
        is_allowed_device(tables, db, out, stream)
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        tdist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        is_allowed_device(tables, db, out, stream)
        ev[k][1].record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    step_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))    # sort + K1, stream events
    kern_ms = float(np.mean(tables.kernel_times(args.steps)))       # K1 alone, library events
    if dist:
        t = torch.tensor([elapsed, kern_ms, step_ms], dtype=torch.float64, device=dev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed, kern_ms, step_ms = float(t[0]), float(t[1]), float(t[2])

    dec = decisions_from_tensor(out)
    if rank == 0:
        per_dec, parts = algorithmic_bytes(cs, sb.batch)
        achieved = per_dec * n / (kern_ms * 1e-3) / 1e9
        value = world * n * args.steps / elapsed
        mix = np.bincount(dec["decision"], minlength=7)
        line = {
            "metric": "authorization decisions/sec (isAllowed)", "value": value, "unit": "decisions/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": desc, "requests_per_gpu": n, "policy_sets": cs.n_sets, "policies": cs.n_pols,
                       "rules": cs.n_rules, "table_bytes": cs.table_bytes(), "parallelism": f"requests dp{world}",
                       "decision_mix": {"PERMIT": int(mix[2]), "DENY": int(mix[3]), "INDETERMINATE": int(mix[5])}},
            "coherence_sort": not args.no_sort,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": "is_allowed_kernel",
                         "kernel_ms": kern_ms, "step_gpu_ms": step_ms, "bytes_per_decision": per_dec,
                         "bytes_parts": parts},
        }
        if world == 1 and not args.no_cpu_baseline:
            cb, par = cpu_baseline(kind, doc, sb, dec, cs, args.cpu_seconds)
            line["cpu_baseline"] = cb
            line["parity"] = par
        print(json.dumps(line), flush=True)
    tables.close()
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
