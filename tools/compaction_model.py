#!/usr/bin/env python3
"""Cost model of a two-phase K1: lanes still walking after U union set
iterations regrouped 64 to a wave for a second launch.  Wave cost = union set iterations until its
last lane reaches its deciding set (c3: every set clean), from the host core's records on the
synthetic c3 batch.  usage: python tools/compaction_model.py [requests]"""

import sys, time
sys.path[:0]=['/root/repo','/root/repo/access-control-srv_amd','/root/repo/tests']
import numpy as np
from acs_mi355x import compiler, store, synth, candidates, layout as L
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS
import host_core
n = int(sys.argv[1]) if len(sys.argv) > 1 else 500_000
cs = compiler.compile_store(store.populate(synth.c3_store()), FULL_URNS, DEFAULT_CAS)
sb = synth.requests(cs, n, "c3", second_role=0.5)
b = sb.batch
t0=time.time(); dec = host_core.is_allowed(cs, b); print("host core", time.time()-t0, file=sys.stderr)
S = cs.n_sets
wsu = b.cand_wsu
cls = (b.hdr["flags"] >> L.RQ_PCOL_SHIFT).astype(np.int64)
cls2 = b.cls2.astype(np.int64) if hasattr(b,'cls2') and b.cls2 is not None else b.lines["cls2"].astype(np.int64)
rows = b.cand
def useful_bits(r):
    w = rows[r, wsu:wsu + (S + 31)//32]
    bits = np.unpackbits(w.view(np.uint8), bitorder='little')[:S]
    return bits.astype(bool)
cache = {}
def ub(r):
    if r not in cache: cache[r] = useful_bits(r)
    return cache[r]
lane_use = lambda i: ub(cls[i]) | (ub(cls2[i]-1) if cls2[i] else False)
dset = np.where(dec["flags"] & L.OF_HAS_EFFECT, dec["aux"].astype(np.int64) - 1, -1)  # deciding set
perm = b.perm if b.perm is not None else np.arange(n)
perm = perm[perm < n]
waves = [perm[k:k+64] for k in range(0, len(perm), 64)]
def wave_cost(lanes, tops):
    # lanes: request idx; tops: per-lane exclusive upper bound of sets still to walk
    top = max(tops)
    u = np.zeros(S, bool)
    for i in lanes: u |= lane_use(i)
    order = np.flatnonzero(u[:top])[::-1]   # descending union walk below the max top
    ranks = []
    for i, tp in zip(lanes, tops):
        d = dset[i]
        # iterations until the lane's deciding set is visited (or the walk's end)
        k = len(order) if d < 0 else int(np.searchsorted(-order, -d, side='left')) + 1
        ranks.append(k)
    return order, ranks
base = 0; ph1 = {1: 0, 2: 0, 3: 0}; left = {1: [], 2: [], 3: []}
for w in waves:
    order, ranks = wave_cost(w, [S]*len(w))
    c = max(ranks); base += c
    for U in ph1:
        ph1[U] += min(U, c)
        if c > U:
            stop = order[U-1]  # the U-th set visited; resume below it
            left[U] += [(i, stop) for i, r in zip(w, ranks) if r > U]
print("lanes", len(perm), "waves", len(waves), "base iterations/wave %.3f" % (base/len(waves)))
for U in ph1:
    L2 = left[U]; ph2 = 0; nw2 = 0
    for k in range(0, len(L2), 64):
        grp = L2[k:k+64]
        order, ranks = wave_cost([g[0] for g in grp], [g[1] for g in grp])
        ph2 += max(ranks); nw2 += 1
    print("U=%d phase1 %.0f + phase2 %.0f (%d waves, %.1f%% lanes left) = %.3f of base; waves total %d" %
          (U, ph1[U], ph2, nw2, 100*len(L2)/len(perm), (ph1[U]+ph2)/base, len(waves)+nw2))
# diagnostics
us = [lane_use(i).sum() for i in perm[:5000]]
print("mean own useful sets per lane %.2f" % np.mean(us))
print("deciding set: effect fraction %.3f" % np.mean(dset[perm] >= 0))
import collections
r1 = [wave_cost(w, [S]*len(w)) for w in waves[:200]]
print("mean union size %.2f, mean max rank %.2f, mean lane rank %.2f" % (np.mean([len(o) for o,_ in r1]), np.mean([max(r) for _,r in r1]), np.mean([np.mean(r) for _,r in r1])))
print("class rows", rows.shape[0], "lanes per class %.1f" % (n / rows.shape[0]))
