"""Rule-sharded isAllowed across ranks (SURVEY.md §8(e), configs[4] variant ii).

The policy store is split into contiguous runs of WHOLE policy sets (Map order
kept), balanced by node count; rank r compiles only its run and evaluates every
request of the batch against it.  Sets are independent in the reference except
for two cross-set rules (accessController.ts:125-295): the last set with a
policy effect decides, and the first set that throws (or reaches a rule
condition) ends the request.  ``acs_shard_keys_device`` encodes each local
decision as a 64-bit key whose integer MAX over ranks is the unsharded answer
(csrc/acs_eval.h: shard_key); one RCCL all-reduce (ncclMax, int64; 8 B per
request) combines the ranks and ``acs_shard_decode_device`` writes the same
decision records an unsharded evaluation does.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from .native import ShardC, last_error


def _weights(store_map: dict) -> np.ndarray:
    w = []
    for ps in store_map.values():
        pols = ps.get("combinables") or {} if isinstance(ps, dict) else {}
        n = 1 + len(pols)
        for p in pols.values():
            if isinstance(p, dict):
                n += len(p.get("combinables") or {})
        w.append(n)
    return np.array(w, np.int64)


def partition(store_map: dict, world: int) -> list[tuple[int, int]]:
    """Contiguous set ranges [a, b) per rank, balanced by sets + policies + rules."""
    w = _weights(store_map)
    n = len(w)
    if world <= 1 or n == 0:
        return [(0, n)] + [(n, n)] * max(world - 1, 0)
    cum = np.concatenate([[0], np.cumsum(w)])
    total = cum[-1]
    cuts = [0]
    for r in range(1, world):
        c = int(np.searchsorted(cum, total * r / world, side="left"))
        cuts.append(min(max(c, cuts[-1]), n))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def slice_store(store_map: dict, a: int, b: int) -> dict:
    """The Map of sets [a, b) (same objects, same order)."""
    items = list(store_map.items())[a:b]
    return dict(items)


def base(store_map: dict, a: int) -> tuple[int, int, int]:
    """Global (set, policy, rule) index of the first node of set a in the full snapshot."""
    n_pols = n_rules = 0
    for k, ps in enumerate(store_map.values()):
        if k >= a:
            break
        pols = ps.get("combinables") or {}
        n_pols += len(pols)
        for p in pols.values():
            if isinstance(p, dict):
                n_rules += len(p.get("combinables") or {})
            # a null policy has no rules (compiler: child range empty)
    return a, n_pols, n_rules


def keys_device(tables, dec_t, shard_base, keys_t=None, stream=None):
    """Enqueue acs_shard_keys_device: uint8 [n, 8] decisions -> int64 [n] keys (torch tensors)."""
    import torch
    n = dec_t.shape[0]
    if keys_t is None:
        keys_t = torch.empty((n,), dtype=torch.int64, device=dec_t.device)
    s = (stream or torch.cuda.current_stream(dec_t.device)).cuda_stream
    sc = ShardC(*shard_base)
    rc = tables.lib.acs_shard_keys_device(tables.h, dec_t.data_ptr(), n, C.byref(sc), keys_t.data_ptr(), C.c_void_p(s))
    if rc != 0:
        raise RuntimeError(f"acs_shard_keys_device: {last_error(tables.lib)}")
    return keys_t


def decode_device(lib, keys_t, out_t=None, stream=None):
    """Enqueue acs_shard_decode_device: reduced int64 keys -> uint8 [n, 8] decision records."""
    import torch
    n = keys_t.shape[0]
    if out_t is None:
        out_t = torch.empty((n, 8), dtype=torch.uint8, device=keys_t.device)
    s = (stream or torch.cuda.current_stream(keys_t.device)).cuda_stream
    rc = lib.acs_shard_decode_device(keys_t.data_ptr(), n, out_t.data_ptr(), C.c_void_p(s))
    if rc != 0:
        raise RuntimeError(f"acs_shard_decode_device: {last_error(lib)}")
    return out_t
