"""Candidate filtering never changes a decision: the filters only skip nodes that cannot
match, throw or push (candidates.py).  The evaluator core (CPU build) gives bit-identical
records — isAllowed decisions, and whatIsAllowed inclusion rows and maskedProperty logs — with
the full class rows (entity x roles x action), with per-role rows composed by the kernel (two
required roles: ReqLine.cls2, role-relaxed useful sections), with the coarser class rows plus
the role factor used for large stores, with entity-only rows, and with no filter."""
import numpy as np
import pytest

import host_core
import randgen
from acs_mi355x import candidates, compiler, encoder, store, synth
from oracle.acs_oracle import DEFAULT_CAS, FULL_URNS

LEVELS = list(candidates.LEVELS)


def _eval_all(cs, make_batch, monkeypatch, stats=None, wia=False):
    outs = {}
    for level in LEVELS:
        monkeypatch.setattr(candidates, "FORCE_LEVEL", level)
        b = make_batch()
        if stats is not None:
            stats["role_factor"] += b.role_key is not None
            stats["composed"] += int((b.lines["cls2"] != 0).sum())
        outs[level] = host_core.is_allowed(cs, b).view(np.uint64)
        if wia:
            bits, obl, obl_n, rec = host_core.what_is_allowed(cs, b)
            outs[level + "/wia"] = (bits, [obl[i, :obl_n[i]].tobytes() for i in range(b.n)], rec.view(np.uint64))
    monkeypatch.setattr(candidates, "FORCE_LEVEL", None)
    b = make_batch()
    b.cand = None  # no filtering at all
    b.role_key = b.role_bits = None
    b.lines["cls2"] = 0
    outs["none"] = host_core.is_allowed(cs, b).view(np.uint64)
    if wia:
        bits, obl, obl_n, rec = host_core.what_is_allowed(cs, b)
        outs["none/wia"] = (bits, [obl[i, :obl_n[i]].tobytes() for i in range(b.n)], rec.view(np.uint64))
    return outs


def _same(outs):
    for k, v in outs.items():
        if k.endswith("/wia"):
            w = outs["none/wia"]
            assert np.array_equal(v[0], w[0]) and v[1] == w[1] and np.array_equal(v[2], w[2]), k
        else:
            assert np.array_equal(v, outs["none"]), k


@pytest.mark.parametrize("seed", range(0, 300, 10))
def test_filters_do_not_change_decisions_random(seed, monkeypatch):
    stats = {"role_factor": 0, "composed": 0}
    for s in range(seed, seed + 10):
        urns, doc, reqs = randgen.rand_case(s)
        cs = compiler.compile_store(store.populate(doc), urns, DEFAULT_CAS)
        outs = _eval_all(cs, lambda: encoder.Encoder(cs).encode(reqs), monkeypatch, stats, wia=s % 3 == 0)
        try:
            _same(outs)
        except AssertionError as e:
            raise AssertionError(f"seed {s}: {e}")
    assert stats["role_factor"] > 0
    assert stats["composed"] > 0  # two-role requests took composed rows


@pytest.mark.parametrize("kind,second", [("c2", 0.0), ("c3", 0.0), ("c3", 0.5)])
def test_filters_do_not_change_decisions_synthetic(kind, second, monkeypatch):
    doc = synth.c2_store() if kind == "c2" else synth.c3_store(n_sets=40)
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    stats = {"role_factor": 0, "composed": 0}
    outs = _eval_all(cs, lambda: synth.requests(cs, 20_000, kind, tree=synth.OrgTree(fanout=3, depth=5),
                                                second_role=second).batch,
                     monkeypatch, stats, wia=kind == "c3")
    assert stats["role_factor"] == 2
    assert (stats["composed"] > 0) == (second > 0)
    _same(outs)


def test_composed_level_taken_when_joint_keys_exceed_the_budget(monkeypatch):
    """c3 with second role associations: the joint (entity, action, role set) keys exceed the
    row budget, so the automatic level choice composes per-role rows."""
    doc = synth.c3_store(n_sets=40)
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    monkeypatch.setattr(candidates, "MAX_CLASSES", 4000)  # joint: ~5.6k rows, composed: ~3.1k
    b = synth.requests(cs, 20_000, "c3", tree=synth.OrgTree(fanout=3, depth=5), second_role=0.5).batch
    assert (b.lines["cls2"] != 0).mean() > 0.3 and b.role_key is None
    monkeypatch.setattr(candidates, "MAX_CLASSES", 0xFFFF)
    monkeypatch.setattr(candidates, "FORCE_LEVEL", "entity+roles+action")
    joint = synth.requests(cs, 20_000, "c3", tree=synth.OrgTree(fanout=3, depth=5), second_role=0.5).batch
    assert np.array_equal(host_core.is_allowed(cs, b).view(np.uint64), host_core.is_allowed(cs, joint).view(np.uint64))


@pytest.mark.parametrize("role_factor", [False, True])
def test_coherence_order(role_factor, monkeypatch):
    """candidates.coherence_order: every request exactly once, holes only as wave padding, and
    each (bucket, second class) key in one contiguous run (role-major with a role factor)."""
    doc = synth.c3_store(n_sets=40)
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    if role_factor:
        monkeypatch.setattr(candidates, "FORCE_LEVEL", "entity+action")
    b = synth.requests(cs, 5000, "c3", tree=synth.OrgTree(fanout=3, depth=5), second_role=0.5).batch
    perm = b.perm
    real = perm[perm != 0xFFFFFFFF]
    assert sorted(real.tolist()) == list(range(b.n))
    cls = (b.hdr["flags"] >> 16).astype(np.int64)
    if role_factor:
        assert b.role_key is not None and len(perm) == b.n
        key = b.role_key[real].astype(np.int64) * 70000 + cls[real]
    else:
        key = cls[real] * 70000 + b.lines["cls2"][real].astype(np.int64)
        if len(perm) > b.n:  # padded: every run of a class starts on a 64-lane boundary
            holes = perm == 0xFFFFFFFF
            starts = np.flatnonzero(~holes & np.concatenate([[True], holes[:-1] | (cls[np.minimum(perm, b.n - 1)][1:]
                                                                                      != cls[np.minimum(perm, b.n - 1)][:-1])]))
            assert (starts % 64 == 0).all()
    change = np.flatnonzero(key[1:] != key[:-1])
    assert len(np.unique(key)) == len(change) + 1  # each key one contiguous run
