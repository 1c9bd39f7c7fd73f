"""Multi-rank paths on the CPU (gloo, world size 2) and the shard arithmetic.

* request sharding (the default bench mode): each rank evaluates a
  contiguous slice of the batch against replicated tables; the gathered records
  equal a single-rank evaluation.
* rule sharding (configs[4] variant ii): each rank compiles only its run of whole
  policy sets, turns its decisions into 64-bit keys (csrc/acs_eval.h shard_key),
  and one all-reduce MAX over ranks gives records bit-identical to evaluating the
  whole store — including errors, rule conditions and "last applicable set wins".

Evaluation uses the CPU build of the evaluator core (tests/native), the same
code the GPU kernels run; the collective is torch.distributed over gloo.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import host_core
import randgen
from acs_mi355x import compiler, encoder, shard, store, synth, layout as L
from oracle.acs_oracle import DEFAULT_CAS, FULL_URNS


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _cases():
    out = []
    for seed in range(40):
        urns, doc, reqs = randgen.rand_case(seed)
        out.append((urns, doc, reqs))
    doc = synth.c3_store(n_sets=12, n_pols=3, n_rules=4)
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 200, "c3", seed=5, tree=synth.OrgTree(fanout=3, depth=4))
    out.append((FULL_URNS, doc, [sb.decode(i) for i in range(200)]))
    return out


def _full(urns, doc, reqs):
    cs = compiler.compile_store(store.populate(doc), urns, DEFAULT_CAS)
    b = encoder.Encoder(cs).encode(reqs)
    return host_core.is_allowed(cs, b)


def _rank_keys(urns, doc, reqs, rank, world):
    full = store.populate(doc)
    a, b = shard.partition(full, world)[rank]
    cs = compiler.compile_store(shard.slice_store(full, a, b), urns, DEFAULT_CAS)
    batch = encoder.Encoder(cs).encode(reqs)
    dec = host_core.is_allowed(cs, batch)
    return host_core.shard_keys(cs, dec, shard.base(full, a))


def _worker(rank, world, port, mode, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        for k, (urns, doc, reqs) in enumerate(_cases()):
            if mode == "rules":
                keys = torch.from_numpy(_rank_keys(urns, doc, reqs, rank, world))
                dist.all_reduce(keys, op=dist.ReduceOp.MAX)
                got = host_core.shard_decode(keys.numpy())
            else:  # request sharding: contiguous slices, replicated tables
                n = len(reqs)
                lo, hi = n * rank // world, n * (rank + 1) // world
                cs = compiler.compile_store(store.populate(doc), urns, DEFAULT_CAS)
                part = host_core.is_allowed(cs, encoder.Encoder(cs).encode(reqs[lo:hi]))
                parts = [None] * world
                dist.all_gather_object(parts, part.tobytes())
                got = np.frombuffer(b"".join(parts), L.DECISION_DT)
            if rank == 0:
                np.save(os.path.join(out_dir, f"{mode}_{k}.npy"), got.view(np.uint64))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["requests", "rules"])
def test_gloo_world2(mode, tmp_path):
    mp.spawn(_worker, args=(2, _free_port(), mode, str(tmp_path)), nprocs=2, join=True)
    for k, (urns, doc, reqs) in enumerate(_cases()):
        want = _full(urns, doc, reqs)
        got = np.load(tmp_path / f"{mode}_{k}.npy")
        assert np.array_equal(got, want.view(np.uint64)), (mode, k)


@pytest.mark.parametrize("world", [1, 2, 3, 5])
def test_rule_shard_keys_any_world(world):
    """The MAX over any number of set shards reproduces the whole-store records."""
    terminal = 0
    for urns, doc, reqs in _cases():
        want = _full(urns, doc, reqs)
        keys = np.stack([_rank_keys(urns, doc, reqs, r, world) for r in range(world)])
        got = host_core.shard_decode(keys.max(axis=0))
        assert np.array_equal(got.view(np.uint64), want.view(np.uint64)), world
        terminal += int(((want["flags"] & (L.OF_ERR | L.OF_HOST_COND)) != 0).sum())
    assert terminal > 0  # errors / conditions are among the cases


def test_partition_balanced_and_contiguous():
    full = store.populate(synth.c3_store())
    for world in (1, 2, 3, 8):
        parts = shard.partition(full, world)
        assert parts[0][0] == 0 and parts[-1][1] == len(full)
        assert all(parts[i][1] == parts[i + 1][0] for i in range(world - 1))
        sizes = [b - a for a, b in parts]
        assert max(sizes) - min(sizes) <= max(2, len(full) // 10)
    assert shard.partition(full, 300)[-1] == (len(full), len(full)) or len(full) >= 300


# ---------------------------------------------------------------- the bench launcher
def _bench(*args, env=None):
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *args], capture_output=True, text=True,
                       timeout=240, env=e)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    return r.returncode, lines, r.stderr


@pytest.mark.parametrize("n", [1, 2, 3])
def test_bench_launcher_spawns_ranks(n):
    """`bench.py --gpus N` (no torch.distributed env) launches N ranks itself through
    torch.distributed.run; every rank joins the collective (gloo here, RCCL on GPUs) and
    rank 0 alone prints the line."""
    rc, lines, err = _bench("--gpus", str(n), "--selftest")
    assert rc == 0, err
    assert lines == [{"selftest": True, "world_size": n, "max_rank_seen": n - 1}]


def test_bench_launcher_rejects_world_mismatch():
    rc, lines, err = _bench("--gpus", "2", "--selftest", env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc != 0 and not lines and "--gpus 2 but WORLD_SIZE=1" in err
