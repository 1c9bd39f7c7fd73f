#!/usr/bin/env python3
"""Benchmark: isAllowed decisions/sec of the MI355X evaluator (BASELINE.json metric).

A step = one K1 launch evaluating one full batch of synthetic requests that is already
resident in HBM, in the coherence order the encoder wrote with the batch (the encoder assigns
every request's class, so it also groups them: no device sort on the step).  Default
workload: c3 = 10M requests x 10k rules, mixed combining algorithms + HR role scoping, each
request with 1-2 role associations (half of them two: SURVEY.md §8(d)), the north star's
10k-rule configuration.  Multi-GPU: one process per GPU; `--gpus N` without a
torch.distributed environment launches the N ranks itself (torch.distributed.run on
127.0.0.1, before anything touches the GPU).  Each rank evaluates its own batch against
replicated tables (weak scaling, no data-path collective); timing = barrier + sync on
both sides, max over ranks.  Rank 0 prints one JSON line with the roofline, CPU-baseline
and parity objects described in DESIGN.md §9; parity = a >= 1 % random sample of the timed
batch re-decided by the C++ oracle (BASELINE.md's gate).
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
    "c3": ("c3: isAllowed, 10M requests/GPU vs 10k rules, mixed CAs + HR role scoping (depth-8 org tree), 1-2 "
           "org-scoped role associations per request (half with two, SURVEY §8(d))", 10_000_000),
    "c3r1": ("c3r1: the c3 workload with one role association per request (the round-1..3 headline form)",
             10_000_000),
    "c3adv": ("c3adv: c3-adverse, 1M requests/GPU vs the c3 store with 0.5 % condition rules in the first 20 sets, a "
              "null policy behind a rare set target and ACLs on 10 % of the context resources (no early stop below "
              "the top sets); requests encoded from JSON by the native codec", 1_000_000),
    "c4": ("c4: whatIsAllowed, 1M reverse queries/GPU vs 10k rules (c3 store, 30% of rules with properties), "
           "inclusion bitsets over sets|policies|rules + maskedProperty logs", 1_000_000),
    "c5": ("c5: isAllowed, 1M-request batches/GPU vs 1M rules (1,000 sets x 10 policies x 100 rules, c3 rule mix "
           "+ HR scoping)", 1_000_000),
}


def make_store(kind):
    from acs_mi355x import synth
    return {"c2": synth.c2_store, "c3": synth.c3_store, "c3r1": synth.c3_store, "c3adv": synth.c3_adverse_store,
            "c4": synth.c3_store,
            "c5": synth.c5_store}[kind]()


def request_kind(kind):
    return "c2" if kind == "c2" else "c3"  # c4 / c5 draw c3-shaped requests (HR context)
# c3-shaped requests: share of subjects with a second org-scoped role association (§8(d): 1-2);
# set per config in main() (0.5; c3r1: 0) unless --second-role is given
SECOND_ROLE = 0.5
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8 TB/s
_T0 = time.time()


REHEARSAL = False


def allreduce_max(t):
    """torch.distributed all-reduce MAX in place (RCCL on device tensors; gloo rehearsal via host)."""
    import torch.distributed as tdist
    if REHEARSAL:
        c = t.cpu()
        tdist.all_reduce(c, op=tdist.ReduceOp.MAX)
        t.copy_(c)
    else:
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)


def log(msg):
    """Setup progress on stderr (large configs take minutes to compile / encode)."""
    print(f"[bench {time.time() - _T0:7.1f}s] {msg}", file=sys.stderr, flush=True)


def _node_bytes(nodes):
    """Bytes of a node record plus the pools it references (pairs 8 B, rule attrs 16 B, ACL roles 4 B)."""
    return (64 + 8 * (nodes["subj_n"].astype(np.int64) + nodes["act_n"]) + 16 * nodes["res_n"].astype(np.int64)
            + 4 * nodes["acl_roles_n"].astype(np.int64))


def measured_scan_bytes(blob, db, local, what="is_allowed"):
    """B_scan of the whole launch, measured: the counting build of the library
    (lib/libacs_mi355x_scan.so, -DACS_SCAN_COUNT) runs the same kernel once on the same device
    batch; every table read a wave issues (node records, pairs, resource attributes, class-row
    words) adds its bytes once per wave.  The traversal is deterministic, so this is exactly
    what the timed launches read from the tables, re-reads included."""
    import ctypes as C
    from acs_mi355x import build as B, native
    from acs_mi355x.device import is_allowed_device, what_is_allowed_device
    scan_lib = os.environ.get("ACS_SCAN_LIB", B.SCAN_LIB)  # A/B: another counting build
    if not os.path.exists(scan_lib):
        raise SystemExit(f"bench.py: counting build missing: {scan_lib} (run __graft_entry__.build())")
    lib = native._declare(C.CDLL(scan_lib))
    lib.acs_scan_read.argtypes = [C.POINTER(C.c_ulonglong)]

    class _T:  # the duck-typed tables handle device.py's launchers take
        pass
    t = _T()
    t.lib = lib
    t.h = lib.acs_compile(blob, len(blob), local)
    if not t.h:
        raise RuntimeError("counting build: acs_compile failed: " + native.last_error(lib))
    t.words = lib.acs_wia_words_per_request(t.h)
    v = C.c_ulonglong(0)
    try:
        lib.acs_scan_read(C.byref(v))  # reset
        if what == "is_allowed":
            is_allowed_device(t, db)
        else:
            what_is_allowed_device(t, db)
        torch.cuda.synchronize()
        if lib.acs_scan_read(C.byref(v)) != 0:
            raise RuntimeError("acs_scan_read: " + native.last_error(lib))
    finally:
        lib.acs_free(t.h)
    return int(v.value)


def table_bytes_full(cs):
    return int(_node_bytes(cs.sets).sum() + _node_bytes(cs.pols).sum() + _node_bytes(cs.rules).sum())


def algorithmic_bytes(cs, batch, scan_total):
    """Per-decision algorithmic bytes: B_req + B_ctx + B_out + B_scan/T, with
    B_scan the table bytes the 64-request tiles actually read (measured_scan_bytes)."""
    h = batch.hdr
    b_req = 16 + 16 * h["nres"].astype(np.float64) + 8 * h["nsubj"] + 8 * h["nact"] + 4 * h["nroles"]
    # context arena bytes each request reads (its own record; a shared record counts for every request)
    offs = h["arena_off"].astype(np.int64)
    uo = np.unique(offs)
    size = np.diff(np.append(uo, batch.arena.size))
    ctx = float(4.0 * size[np.searchsorted(uo, offs)].mean()) if batch.n else 0.0
    full = table_bytes_full(cs)
    b_scan_per_dec = scan_total / max(batch.n, 1)
    per = float(b_req.mean()) + ctx + 8.0 + b_scan_per_dec
    return per, {"B_req": float(b_req.mean()), "B_ctx": ctx, "B_out": 8.0, "B_scan_per_decision": b_scan_per_dec,
                 "B_scan_per_tile": b_scan_per_dec * 64, "table_bytes_full": full, "T": 64,
                 "bruteforce_bytes_per_decision": float(b_req.mean()) + ctx + 8.0 + full / 64.0}


def traffic_key(config, requests, world, mode):
    """profiles/traffic.json key: the run shape a PMC pass measured (config, requests per
    rank, ranks, request / rule sharding)."""
    return f"{config}/n{requests}/w{world}/{mode}"


def measured_traffic(key, kernel="is_allowed_kernel"):
    """HBM bytes per launch of `kernel` from the committed PMC passes of the same bench
    command (profiles/traffic.json, written by tools/pmc.sh + tools/pmc_traffic.py), or
    (None, None) when no pass measured this exact run shape.  Entry: FETCH_SIZE x 2 +
    WRITE_SIZE (MI355X_MICROARCH.md gfx950 note; the x2 is calibrated for wide streaming
    reads only, so the entry also carries the gather calibration when one was measured)."""
    p = os.path.join(ROOT, "profiles", "traffic.json")
    if not os.path.exists(p):
        return None, None
    with open(p) as f:
        d = json.load(f)
    e = d.get(key, {}).get(kernel)
    return (e["bytes_per_launch"], e) if e else (None, None)


def launch(args):
    """`--gpus N` outside a torch.distributed environment: run N ranks of this same command
    through torch.distributed.run (one process per GPU, rendezvous on 127.0.0.1) as CHILD
    processes — nothing here has touched the GPU — and exit with their status."""
    import socket
    import subprocess
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    log(f"launching {args.gpus} ranks: torch.distributed.run on 127.0.0.1:{port}")
    return subprocess.run(cmd, env=env).returncode


def selftest(world, rank):
    """`--selftest`: the launcher and the collective path without a GPU (gloo on CPU):
    every rank all-reduces its rank id with MAX, rank 0 prints what it saw."""
    import torch.distributed as tdist
    if world > 1:
        tdist.init_process_group("gloo")
        t = torch.tensor([float(rank)])
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        seen = int(t.item())
        assert tdist.get_world_size() == world
    else:
        seen = 0
    if rank == 0:
        print(json.dumps({"selftest": True, "world_size": world, "max_rank_seen": seen}), flush=True)
    if world > 1:
        tdist.destroy_process_group()


def oracle_parity(kind, doc, sb, gpu_dec, cs, fraction, seconds):
    """Parity gate + CPU baseline from ONE oracle run: a random sample of the timed batch
    (``fraction`` of it, BASELINE.md's >= 1 %; c5 too, with a longer time bound) is
    decoded to the reference's JSON request shape and re-decided by the C++ oracle
    (oracle/acs_oracle.cpp: the reference's per-request serial algorithm, 'port'),
    std::thread x up to 16 host cores (the GPU box's CPU share).  Every sampled outcome is
    compared with the GPU's decision record; the oracle's evaluation wall time (decode and
    JSON parse excluded) is the CPU baseline.  HR scope trees are shared between requests
    through {"$shared": k} placeholders so each is serialised and parsed once."""
    from oracle import acs_oracle_c
    from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS
    from diff_utils import gpu_outcome
    from acs_mi355x import layout as L
    from acs_mi355x.synth import SharedValues
    acs_oracle_c.build()
    threads = max(1, min(16, os.cpu_count() or 1))
    co = acs_oracle_c.COracle(FULL_URNS, DEFAULT_CAS, doc)
    n = sb.batch.n
    want_n = max(1, int(round(fraction * n)))
    idx = np.random.default_rng(1234).permutation(n)[:want_n]
    chunk = {"c2": 50_000, "c3": 10_000, "c3r1": 10_000, "c3adv": 10_000}.get(kind, 1000)
    done = busy = mism = unsup = host = host_both = 0
    wall0 = time.perf_counter()
    while done < len(idx) and busy < seconds and time.perf_counter() - wall0 < 2 * seconds + 30:
        part = idx[done:done + chunk]
        sh = SharedValues()
        reqs = [sb.decode(int(i), sh) for i in part]
        out, sec = co.raw(reqs, threads, shared=sh.values)
        busy += sec
        for i, r in zip(part, out):
            want = acs_oracle_c.outcome(r)
            got = gpu_outcome(cs, gpu_dec[i])
            cond = bool(gpu_dec[i]["flags"] & L.OF_HOST_COND)
            if want[0] == "UNSUPPORTED":  # the oracle met a rule condition (JS eval) or a subject token
                if got[0] == "HOST":
                    host_both += 1
                else:
                    unsup += 1
            elif cond:  # the GPU stopped at a condition the oracle's forward walk never reached
                mism += 1
            elif got[0] == "HOST":
                host += 1
            elif got != want:
                mism += 1
        done += len(part)
        log(f"oracle parity: {done}/{len(idx)} requests, {busy:.1f}s oracle evaluation, {mism} mismatches")
    co.close()
    cb = {"value": done / busy, "unit": "decisions/s", "cores": threads, "kind": "port",
          "sample": f"{done} random requests of the same {kind} batch through oracle/acs_oracle.cpp (C++17 "
                    f"restatement of the reference's per-request serial algorithm; per-request HR flattening "
                    f"memoised, so faster than the reference's own loop), std::thread x {threads}, "
                    f"{busy:.1f}s of evaluation wall time (requests decoded and parsed beforehand)"}
    par = {"oracle_sample": done, "sample_fraction": done / n, "mismatches": mism,
           "oracle_unsupported": unsup, "gpu_host_path": host, "host_path_both": host_both,
           "checker": "oracle/acs_oracle.cpp"}
    return cb, par


def codec_batch(cs, sb):
    """The batch of ``sb``'s JSON text through the native codec (the product encoder), its HR
    forests registered first (the per-subject cache)."""
    from acs_mi355x.codec import NativeCodec
    codec = NativeCodec(compiler_blob(cs))
    for k, v in sb.hrs_forests().items():
        codec.set_subject_scopes(k, v)
    b = codec.encode(sb.json_text(), threads=max(1, min(16, os.cpu_count() or 1)))
    if b.host_reasons:
        raise SystemExit(f"codec sent {len(b.host_reasons)} requests to the host: {next(iter(b.host_reasons.values()))}")
    return b


def compiler_blob(cs):
    from acs_mi355x import compiler
    return compiler.store_blob(cs)


def end_to_end(kind, cs, sb, tables, dec_resident, n_e2e, threads):
    """JSON -> decision, the product path: the JSON text of the first n_e2e requests of the
    timed batch through acs_pipeline (csrc/acs_kernels.hip) — the request array delimited on
    `threads` host threads, then chunk k+1 encoded by the native codec (csrc/acs_codec.cpp) on
    those threads while chunk k is uploaded from the codec's page-locked blocks, sorted, decided
    by K1 and downloaded on a second stream.  c3 subjects name their HR forests by reference
    ("$hrs": the per-subject cache, registered once before timing, as the reference's Redis HR
    cache is warm in steady state); one untimed run warms the codec's caches (HR forests,
    candidate-class rows, page-locked blocks), as a service's steady state has them.  The
    records must equal those of the resident (synthetic-packed) path bit for bit.  Also
    reported: the same requests encoded in one call, then decided (no overlap), and the share
    of a steady-state encode spent on candidate classes."""
    from acs_mi355x import compiler
    from acs_mi355x.codec import NativeCodec, Pipeline
    idx = np.arange(min(n_e2e, sb.batch.n))
    n = len(idx)
    t0 = time.perf_counter()
    text = sb.json_text(idx)
    gen_s = time.perf_counter() - t0
    forests = sb.hrs_forests(idx) if kind != "c2" else {}

    def new_codec():
        c = NativeCodec(compiler.store_blob(cs))
        for k, v in forests.items():
            c.set_subject_scopes(k, v)
        return c

    codec = new_codec()
    registered = len(forests)
    # chunk sizes: the device work of a chunk is ~1/20 of its encode (c3), so the overlap hides
    # little and each chunk repeats per-batch codec work (class keys, thread-local string and
    # forest caches); the fastest chunk size is reported, every one in requests_per_s_by_chunk
    by_chunk, st, same = {}, None, True
    for chunk in (131072, 262144, 524288):
        pipe = Pipeline(tables, codec, threads=threads, chunk=chunk)
        pipe.is_allowed(text, n)  # warm: HR forests, class rows, regex columns, page-locked blocks
        dec, s1 = pipe.is_allowed(text, n)
        same = same and bool(np.array_equal(dec.view(np.uint64), dec_resident[idx].view(np.uint64)))
        pipe.close()
        by_chunk[chunk] = n / s1["total_s"]
        if st is None or s1["total_s"] < st["total_s"]:
            st, best_chunk = s1, chunk
    # cold: the first batch of a fresh codec (HR forests registered as above; no class rows, regex
    # columns or page-locked blocks yet), at the fastest chunk size
    codec_c = new_codec()
    pipe = Pipeline(tables, codec_c, threads=threads, chunk=best_chunk)
    dec, sc = pipe.is_allowed(text, n)
    same = same and bool(np.array_equal(dec.view(np.uint64), dec_resident[idx].view(np.uint64)))
    pipe.close()
    codec_c.close()
    cold = {"requests_per_s": n / sc["total_s"], "total_s": sc["total_s"], "encode_s": sc["encode_s"],
            "what": "the same pipeline's first batch on a fresh codec (class rows, regex columns and "
                    "page-locked blocks computed inside the timed run)"}
    # sequential: one encode call, then acs_is_allowed on its (compact, page-locked) buffers
    t0 = time.perf_counter()
    b = codec.encode(text, threads=threads)
    t1 = time.perf_counter()
    dec2 = tables.is_allowed(b)
    t2 = time.perf_counter()
    bst = b.stats()
    wire = b.nbytes()
    same = same and bool(np.array_equal(dec2.view(np.uint64), dec_resident[idx].view(np.uint64)))
    b.close()
    codec.close()
    return {"requests": n, "json_bytes": len(text), "json_bytes_per_request": len(text) / n,
            "json_generation_s": gen_s, "threads": threads,
            "requests_per_s": n / st["total_s"], "chunk": best_chunk,
            "requests_per_s_by_chunk": {str(k): v for k, v in by_chunk.items()},
            "what": "JSON text -> acs_pipeline (delimit; per chunk: native encode into page-locked "
                    "blocks || upload + coherence sort + K1 + download of the previous chunk on a second stream) -> "
                    "decision records in host memory; codec caches warm (steady state)",
            "stages": {"total_s": st["total_s"], "split_s": st["split_s"], "encode_s": st["encode_s"],
                       "check_s": st["check_s"], "device_wait_s": st["wait_s"],
                       "device_ms": st["gpu_ms"], "chunks": int(st["chunks"]),
                       "upload_bytes_per_request": st["upload_bytes"] / n,
                       "host_path_requests": int(st["host_requests"])},
            "sequential": {"requests_per_s": n / (t2 - t0), "encode_s": t1 - t0, "decide_s": t2 - t1,
                           "encode_parts_s": {k: bst[k] for k in ("encode_s", "regex_s", "classes_s")},
                           "class_share_of_encode": bst["classes_s"] / max(bst["total_s"], 1e-9),
                           "classes": bst["classes"], "classes_computed": bst["classes_new"],
                           "wire_bytes_per_request": wire / n,
                           "hr_forests_registered": registered, "hr_cache_hits": bst["hr_cache_hits"],
                           "hr_cache_misses": bst["hr_cache_misses"]},
            "cold": cold, "identical_to_resident_path": same}


def pinned_compact(batch):
    """The batch's compact arrays (lines, extension records, arena, regex matrix, class rows,
    coherence order) copied into page-locked host memory (torch pin_memory), as the native codec
    leaves them: what a service hands to acs_is_allowed."""
    import types
    out = types.SimpleNamespace(n=batch.n, rx_rows=batch.rx_rows, cand_wp=batch.cand_wp, cand_wr=batch.cand_wr,
                                cand_wsu=batch.cand_wsu, cand_wpu=batch.cand_wpu, cand_wv=batch.cand_wv,
                                hints=getattr(batch, "hints", 0))
    keep = []
    # perm: the encoder's coherence order travels with the batch (as the codec leaves it), so the
    # host-buffer path runs K1 in that order instead of re-sorting on the device
    for k in ("lines", "ext", "arena", "rx", "cand", "role_key", "role_bits", "perm"):
        a = getattr(batch, k)
        if a is None:
            setattr(out, k, None)
            continue
        t = torch.empty(max(a.nbytes, 16), dtype=torch.uint8, pin_memory=True)
        v = t.numpy()[:a.nbytes].view(a.dtype).reshape(a.shape)
        v[...] = a
        keep.append(t)
        setattr(out, k, v)
    out._keep = keep
    return out


def bench_what_is_allowed(args, desc, n, doc, full_map, world, rank, local, dev, dist):
    """c4: one step = K2 over a resident batch of whatIsAllowed requests (c3 store and request
    generator); outputs: per-request inclusion bitset over (sets | policies | rules), the
    maskedProperty push log, its length and the 8-B record.  Parity: a random sample vs
    the Python oracle's whatIsAllowed (rule sets bit-exact, obligations in push order)."""
    from acs_mi355x import compiler, native, results, synth, layout as L
    from acs_mi355x.config import SERVICE_URNS as FULL_URNS, COMBINING_ALGORITHMS as DEFAULT_CAS
    from acs_mi355x.device import DeviceBatch, what_is_allowed_device, resolve_overflow_device, overflow_logs
    from oracle.acs_oracle import Oracle, FULL_URNS as ORACLE_URNS
    from diff_utils import norm_rq
    import torch.distributed as tdist
    cs = compiler.compile_store(full_map, FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, n, "c3", seed=0xACC1004 + 17 * rank, second_role=SECOND_ROLE)
    log(f"compiled {cs.n_rules} rules; encoded {n} requests")
    blob = compiler.store_blob(cs)
    tables = native.Tables(blob, local)
    tables.set_timing(True)
    db = DeviceBatch(sb.batch, local, compact=True)  # the product form: request lines + extension records
    stream = torch.cuda.current_stream(dev)
    bufs = what_is_allowed_device(tables, db, None, stream)

    def step():  # K2 (+ transpose), then the obligation-only pass for overflowed logs
        what_is_allowed_device(tables, db, bufs, stream)
        return resolve_overflow_device(tables, db, bufs, stream=stream)

    for _ in range(args.warmup):
        step()
    # K2 alone (its overflowed logs left unresolved), reported beside the whole-job step
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        what_is_allowed_device(tables, db, bufs, stream)
    torch.cuda.synchronize(dev)
    k2_only_ms = (time.perf_counter() - t0) / args.steps * 1e3
    if dist:
        tdist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        passes = step()
    torch.cuda.synchronize(dev)
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean(tables.kernel_times(2 * args.steps)))  # K2 launches of both loops
    if dist:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        allreduce_max(t)
        elapsed, kern_ms = float(t[0]), float(t[1])
    if rank == 0:
        bits = bufs[0].cpu().numpy().view(np.uint32)
        obl = bufs[1].cpu().numpy().view(np.uint32)
        obl_n = bufs[2].cpu().numpy().view(np.uint32)
        rec = bufs[3].cpu().numpy().reshape(-1).view(L.DECISION_DT)
        words = bits.shape[1]
        per_req, parts = algorithmic_bytes(cs, sb.batch, measured_scan_bytes(blob, db, local, "what_is_allowed"))
        # K2 writes the inclusion bitset, the log entries it pushes, the log length and the record
        out_b = 4 * words + 8 * float(obl_n.mean()) + 4 + 8
        per = per_req - 8.0 + out_b
        parts.update({"B_out": out_b, "bitset_bytes": 4 * words, "obligation_entries_mean": float(obl_n.mean())})
        achieved = per * n / (kern_ms * 1e-3) / 1e9
        # parity: every overflowed request (bounded) and a random >= 1 % sample of the rest vs
        # the C++ oracle's whatIsAllowed (rule sets + maskedProperty pushes in order)
        from oracle import acs_oracle_c
        from oracle.acs_oracle import DEFAULT_CAS as ORACLE_CAS
        from diff_utils import gpu_reverse_query_compact
        from acs_mi355x.synth import SharedValues
        acs_oracle_c.build()
        co = acs_oracle_c.COracle(ORACLE_URNS, ORACLE_CAS, doc)
        rng = np.random.default_rng(4321)
        long_logs = overflow_logs(passes)
        over = (rec["flags"] & L.OF_OBL_OVERFLOW) != 0
        resolved = np.zeros(n, bool)
        resolved[list(long_logs)] = True
        rec["flags"][resolved] &= np.uint8(~L.OF_OBL_OVERFLOW & 0xFF)
        ok = np.flatnonzero((rec["flags"] & (L.OF_OBL_OVERFLOW | L.OF_HOST_REQ)) == 0)
        want_n = max(1, int(round(args.parity_fraction * n)))
        order = np.concatenate([rng.permutation(np.flatnonzero(resolved))[:2000],
                                rng.permutation(np.setdiff1d(ok, np.flatnonzero(resolved)))[:want_n]])
        mism = checked = unsup = 0
        busy = 0.0
        threads = max(1, min(16, os.cpu_count() or 1))
        t1 = time.perf_counter()
        for c0 in range(0, len(order), 5000):
            part = order[c0:c0 + 5000]
            sh = SharedValues()
            reqs = [sb.decode(int(i), sh) for i in part]
            res, sec = co.what_is_allowed(reqs, threads, shared=sh.values)
            busy += sec
            for i, want in zip(part, res):
                log_i = long_logs[i] if resolved[i] else obl[i][:obl_n[i]]
                got = gpu_reverse_query_compact(cs, sb.batch.overlay, bits[i], log_i, rec[i])
                if want["k"] == 2 or got is None:
                    unsup += 1
                    continue
                checked += 1
                mism += got != want
            log(f"whatIsAllowed parity: {checked + unsup}/{len(order)} queries, {mism} mismatches")
            if time.perf_counter() - t1 > 3 * args.cpu_seconds + 60:
                break
        co.close()
        line = {
            "metric": "whatIsAllowed reverse queries/sec", "value": world * n * args.steps / elapsed,
            "unit": "queries/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": desc, "requests_per_gpu": n, "policy_sets": cs.n_sets, "policies": cs.n_pols,
                       "rules": cs.n_rules, "bitset_words_per_request": words, "parallelism": f"requests dp{world}",
                       "host_path_fraction": float(1 - len(ok) / n),
                       "obligation_overflow_fraction": float(over.mean()),
                       "obligation_pass": {"requests": int(over.sum()), "passes": len(passes),
                                           "k2_only_ms_per_step": k2_only_ms,
                                           "k2_only_queries_per_s": n / (k2_only_ms * 1e-3),
                                           "max_log": int(max((len(v) for v in long_logs.values()), default=0))}},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": measured_traffic(traffic_key("c4", n, world, "requests"),
                                                                                      "what_is_allowed_kernel")[0],
                         "kernel": "what_is_allowed_kernel",
                         "kernel_ms": kern_ms, "bytes_per_query": per,
                         "bytes_parts": parts, "output_GBps": (4 * words + 8 * float(obl_n.mean()) + 12) * n /
                         (kern_ms * 1e-3) / 1e9},
            "parity": {"oracle_sample": checked, "sample_fraction": checked / n, "mismatches": int(mism),
                       "oracle_unsupported": unsup, "overflowed_checked": int(min(resolved.sum(), 2000)),
                       "checker": "oracle/acs_oracle.cpp whatIsAllowed (rule sets + maskedProperty pushes in order)"},
            "cpu_baseline": {"value": (checked + unsup) / max(busy, 1e-9), "unit": "queries/s", "cores": threads,
                             "kind": "port",
                             "sample": f"{checked + unsup} queries of the same batch through oracle/acs_oracle.cpp "
                                       f"whatIsAllowed, std::thread x {threads}, {busy:.1f}s of evaluation"},
        }
        print(json.dumps(line), flush=True)
    tables.close()
    if dist:
        tdist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--requests", type=int, default=0, help="requests per GPU (default: the config's)")
    ap.add_argument("--parity-fraction", type=float, default=0.01,
                    help="fraction of the timed batch re-decided by the C++ oracle (BASELINE.md: >= 1 %%)")
    ap.add_argument("--cpu-seconds", type=float, default=None,
                    help="bound on the oracle's evaluation time (default 90 s; c5: 400 s, the time the C++ oracle "
                         "needs for 1 %% of a 1M-request batch against 1M rules on 16 threads)")
    ap.add_argument("--no-cpu-baseline", action="store_true", help="skip the oracle parity + CPU baseline leg")
    ap.add_argument("--selftest", action="store_true", help="launcher / collective check on CPU (gloo), no GPU")
    ap.add_argument("--e2e-requests", type=int, default=1_000_000,
                    help="requests of the JSON -> decision measurement (0: skip)")
    ap.add_argument("--second-role", type=float, default=None,
                    help="c3-shaped requests: fraction with a second role association (SURVEY §8(d): 1-2)")
    ap.add_argument("--no-sort", action="store_true", help="disable the (class, action) coherence sort")
    ap.add_argument("--no-pcie", action="store_true", help="skip the host-buffer (PCIe-inclusive) measurement")
    ap.add_argument("--lib", default=None, help="evaluate with another build of libacs_mi355x (experiments)")
    ap.add_argument("--rule-shard", action="store_true",
                    help="configs[4] variant ii: whole policy sets sharded over ranks, every rank evaluates the "
                         "same requests, one all-reduce MAX of 64-bit decision keys (RCCL) combines them")
    args = ap.parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch(args))  # parent: spawns the ranks, touches no GPU

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world} (launch with --nproc-per-node "
                         f"{args.gpus}, or run without a torch.distributed environment)")
    if args.selftest:
        return selftest(world, rank)
    if args.cpu_seconds is None:
        args.cpu_seconds = 400.0 if args.config == "c5" else 90.0
    globals()["SECOND_ROLE"] = args.second_role if args.second_role is not None else (0.0 if args.config == "c3r1" else 0.5)
    dist = world > 1
    global REHEARSAL
    # ACS_BENCH_REHEARSAL=1: several ranks on ONE GPU over gloo (collectives through host
    # copies) — exercises the multi-rank code paths on a 1-GPU box; its numbers are not a
    # measurement.  Real runs: one rank per GPU over RCCL ("nccl").
    REHEARSAL = dist and os.environ.get("ACS_BENCH_REHEARSAL") == "1"
    if REHEARSAL:
        local = 0
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        if REHEARSAL:
            tdist.init_process_group("gloo")
        else:
            tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    if dist:
        assert tdist.get_world_size() == args.gpus

    from acs_mi355x import compiler, native, shard, store, synth, layout as L
    from acs_mi355x.config import SERVICE_URNS as FULL_URNS, COMBINING_ALGORITHMS as DEFAULT_CAS
    from acs_mi355x.device import DeviceBatch, is_allowed_device, decisions_from_tensor

    kind = args.config
    desc, n_default = WORKLOADS[kind]
    n = args.requests or n_default
    log(f"config {kind}: generating the store")
    doc = make_store(kind)
    full_map = store.populate(doc)
    log("store populated")
    if kind == "c4":
        return bench_what_is_allowed(args, desc, n, doc, full_map, world, rank, local, dev, dist)
    if args.rule_shard:
        # variant ii: this rank's run of whole policy sets; the same requests on every rank
        set_lo, set_hi = shard.partition(full_map, world)[rank]
        sbase = shard.base(full_map, set_lo)
        cs = compiler.compile_store(shard.slice_store(full_map, set_lo, set_hi), FULL_URNS, DEFAULT_CAS)
        sb = synth.requests(cs, n, request_kind(kind), seed=0xACC1000, second_role=SECOND_ROLE)
    else:
        cs = compiler.compile_store(full_map, FULL_URNS, DEFAULT_CAS)
        sb = synth.requests(cs, n, request_kind(kind), seed=0xACC1000 + 17 * rank, second_role=SECOND_ROLE,
                            acl=0.1 if kind == "c3adv" else 0.0, classes=kind != "c3adv")
        if kind == "c3adv":  # ACL maps are not packed by synth: the product codec encodes the JSON
            sb.batch = codec_batch(cs, sb)
    log(f"compiled {cs.n_rules} rules; encoded {n} requests ({sb.batch.cand.shape[0]} classes)")
    if args.lib:
        native.load(args.lib)
    blob = compiler.store_blob(cs)
    tables = native.Tables(blob, local)
    tables.set_sort(not args.no_sort)
    tables.set_timing(True)
    db = DeviceBatch(sb.batch, local, compact=True)  # the product form: request lines + extension records
    out = torch.empty((n, 8), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    if args.rule_shard:
        local_out = torch.empty((n, 8), dtype=torch.uint8, device=dev)
        keys = torch.empty((n,), dtype=torch.int64, device=dev)

    def step():
        if not args.rule_shard:
            is_allowed_device(tables, db, out, stream)
            return
        is_allowed_device(tables, db, local_out, stream)
        shard.keys_device(tables, local_out, sbase, keys, stream)
        if dist:
            allreduce_max(keys)  # C1: RCCL over xGMI, 8 B per request
        shard.decode_device(tables.lib, keys, out, stream)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist:
        tdist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record(stream)
        step()
        ev[k][1].record(stream)
    torch.cuda.synchronize(dev)
    if dist:
        tdist.barrier()
    elapsed = time.perf_counter() - t0
    step_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))    # sort + K1, stream events
    kern_ms = float(np.mean(tables.kernel_times(args.steps)))       # K1 alone, library events
    if dist:
        t = torch.tensor([elapsed, kern_ms, step_ms], dtype=torch.float64, device=dev)
        allreduce_max(t)
        elapsed, kern_ms, step_ms = float(t[0]), float(t[1]), float(t[2])

    log("timed steps done")
    dec = decisions_from_tensor(out)
    shard_check = None
    if args.rule_shard and rank == 0:
        # size-independent property: the set-sharded + all-reduced records equal an
        # unsharded evaluation of the whole store on the same requests, bit for bit
        cs_full = compiler.compile_store(full_map, FULL_URNS, DEFAULT_CAS)
        sb_full = synth.requests(cs_full, n, request_kind(kind), seed=0xACC1000, second_role=SECOND_ROLE)
        t_full = native.Tables(compiler.store_blob(cs_full), local)
        want = decisions_from_tensor(is_allowed_device(t_full, DeviceBatch(sb_full.batch, local)))
        t_full.close()
        shard_check = {"ranks": world, "sets": [set_lo, set_hi], "requests": n,
                       "identical_to_unsharded": bool(np.array_equal(want.view(np.uint64), dec.view(np.uint64)))}
    pcie = None
    if rank == 0 and not args.no_pcie and not args.rule_shard:
        # host buffers through acs_is_allowed: H2D + sort + K1 + D2H (reported beside, never
        # `value`), from the compact form in page-locked memory, as the codec leaves a batch
        hb = pinned_compact(sb.batch)
        pinned_out = torch.empty(n * 8, dtype=torch.uint8, pin_memory=True)
        host_dec = pinned_out.numpy().view(L.DECISION_DT)
        tables.is_allowed(hb, compact=True, out=host_dec)
        # one upload, one launch, one download (ACS_OPT_CHUNK 0), beside the default overlapped chunks
        tables.set_chunk(0)
        tables.is_allowed(hb, compact=True, out=host_dec)
        t1 = time.perf_counter()
        tables.is_allowed(hb, compact=True, out=host_dec)
        serial_s = time.perf_counter() - t1
        tables.set_chunk(262144)
        tables.is_allowed(hb, compact=True, out=host_dec)
        t1 = time.perf_counter()
        tables.is_allowed(hb, compact=True, out=host_dec)
        pcie_s = time.perf_counter() - t1
        in_bytes = int(sb.batch.compact_nbytes())
        pcie = {"value": n / pcie_s, "unit": "decisions/s", "ms": pcie_s * 1e3,
                "effective_gb_s": (in_bytes + 8 * n) / pcie_s / 1e9,
                "unchunked": {"value": n / serial_s, "ms": serial_s * 1e3},
                "input_bytes": in_bytes,
                "input": "compact batch (request lines + extension records + arena + regex matrix + class rows + "
                         "coherence order) in page-locked host memory, records into page-locked memory",
                "identical_to_device_path": bool(np.array_equal(host_dec.view(np.uint64), dec.view(np.uint64)))}
        del hb
    if rank == 0:
        log("counting algorithmic bytes")
        per_dec, parts = algorithmic_bytes(cs, sb.batch, measured_scan_bytes(blob, db, local))
        achieved = per_dec * n / (kern_ms * 1e-3) / 1e9
        mode = "rules" if args.rule_shard else "requests"
        traffic, traffic_src = measured_traffic(traffic_key(kind, n, world, mode))
        # request sharding: every rank decides its own n requests; rule sharding: the ranks
        # decide the same n requests together
        value = (1 if args.rule_shard else world) * n * args.steps / elapsed
        mix = np.bincount(dec["decision"], minlength=7)
        host = int(((dec["flags"] & (L.OF_HOST_REQ | L.OF_HOST_COND)) != 0).sum())
        line = {
            "metric": "authorization decisions/sec (isAllowed)", "value": value, "unit": "decisions/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong" if args.rule_shard else "weak",
            "vs_baseline": None, "dtype": "u32", "data": "synthetic",
            "config": {"workload": desc + (" [policy sets sharded over ranks + all-reduce MAX]" if args.rule_shard
                                           else ""),
                       "requests_per_gpu": n, "policy_sets": cs.n_sets, "policies": cs.n_pols,
                       "rules": cs.n_rules, "table_bytes": cs.table_bytes(),
                       "parallelism": f"policy-set shards x{world}" if args.rule_shard else f"requests dp{world}",
                       "decision_mix": {"PERMIT": int(mix[2]), "DENY": int(mix[3]), "INDETERMINATE": int(mix[5])},
                       "host_fallback_fraction": host / n, "request_classes": int(sb.batch.cand.shape[0]),
                       "role_factor_rows": (int(sb.batch.role_bits.shape[0])
                                            if getattr(sb.batch, "role_key", None) is not None else 0),
                       "second_role_fraction": SECOND_ROLE if request_kind(kind) == "c3" else 0.0,
                       "ranks_confirmed": world},
            "coherence_sort": not args.no_sort,
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS,
                         "traffic": traffic, "traffic_unit": "HBM bytes per K1 launch (rocprofv3 PMC)",
                         "traffic_key": traffic_key(kind, n, world, mode), "traffic_source": traffic_src,
                         "algorithmic_bytes_per_launch": per_dec * n,
                         "kernel": "is_allowed_kernel", "kernel_ms": kern_ms, "step_gpu_ms": step_ms,
                         "bytes_per_decision": per_dec, "bytes_parts": parts},
        }
        if pcie:
            line["pcie_inclusive"] = pcie
        if shard_check:
            line["rule_shard"] = shard_check
        if world == 1 and args.e2e_requests and not args.rule_shard:
            log("end to end: JSON -> native codec -> GPU -> decisions")
            line["end_to_end"] = end_to_end(kind, cs, sb, tables, dec, args.e2e_requests,
                                            max(1, min(16, os.cpu_count() or 1)))
        if REHEARSAL:
            line["rehearsal"] = "gloo, all ranks on one GPU: code-path check, not a measurement"
        if world == 1 and not args.no_cpu_baseline:
            log("oracle parity + CPU baseline (C++ oracle)")
            cb, par = oracle_parity(kind, doc, sb, dec, cs, args.parity_fraction, args.cpu_seconds)
            line["cpu_baseline"] = cb
            line["parity"] = par
        print(json.dumps(line), flush=True)
    tables.close()
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
