"""Candidate filtering never changes a decision: the filters only skip nodes that cannot
match, throw or push (candidates.py).  The evaluator core (CPU build) gives bit-identical
records with the full class rows (entity x roles x action), with the coarser class rows
plus the role factor used for large stores, with entity-only rows, and with no filter."""
import numpy as np
import pytest

import host_core
import randgen
from acs_mi355x import candidates, compiler, encoder, store, synth
from oracle.acs_oracle import DEFAULT_CAS, FULL_URNS

LEVELS = ["entity+roles+action", "entity+action", "entity"]


def _eval_all(cs, make_batch, monkeypatch, stats=None):
    outs = {}
    for level in LEVELS:
        monkeypatch.setattr(candidates, "FORCE_LEVEL", level)
        b = make_batch()
        if stats is not None and b.role_key is not None:
            stats["role_factor"] += 1
        outs[level] = host_core.is_allowed(cs, b).view(np.uint64)
    monkeypatch.setattr(candidates, "FORCE_LEVEL", None)
    b = make_batch()
    b.cand = None  # no filtering at all
    b.role_key = b.role_bits = None
    outs["none"] = host_core.is_allowed(cs, b).view(np.uint64)
    return outs


@pytest.mark.parametrize("seed", range(0, 300, 10))
def test_filters_do_not_change_decisions_random(seed, monkeypatch):
    stats = {"role_factor": 0}
    for s in range(seed, seed + 10):
        urns, doc, reqs = randgen.rand_case(s)
        cs = compiler.compile_store(store.populate(doc), urns, DEFAULT_CAS)
        outs = _eval_all(cs, lambda: encoder.Encoder(cs).encode(reqs), monkeypatch, stats)
        for k, v in outs.items():
            assert np.array_equal(v, outs["none"]), (s, k)
    assert stats["role_factor"] > 0


@pytest.mark.parametrize("kind", ["c2", "c3"])
def test_filters_do_not_change_decisions_synthetic(kind, monkeypatch):
    doc = synth.c2_store() if kind == "c2" else synth.c3_store(n_sets=40)
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    stats = {"role_factor": 0}
    outs = _eval_all(cs, lambda: synth.requests(cs, 20_000, kind, tree=synth.OrgTree(fanout=3, depth=5)).batch,
                     monkeypatch, stats)
    assert stats["role_factor"] == 2
    for k, v in outs.items():
        assert np.array_equal(v, outs["none"]), k
