"""Cutting a combining loop short (acs_eval.h: eval_set, Fold::final) and stopping the
last-to-first walk over the sets (is_allowed_body, NF_CLEAN_BELOW) never change a record.  Random stores with injected rule conditions, RegExp SyntaxErrors in rule entities and
invalid combining algorithms — the only things that can still matter after a fold's result
is final — are evaluated with the cut (default) and with ACS_NO_CUT=1; the records must be
bit-identical (decision, ec, flags, error kind and aux: set index / condition rule index)."""
import copy
import random

import numpy as np
import pytest

import host_core
import randgen
from diff_utils import build
from acs_mi355x import encoder, layout as L

BAD_ENTITY = "urn:restorecommerce:acs:model:bad(Ent"  # new RegExp(...) throws SyntaxError


def cut_case(seed):
    urns, doc, reqs = randgen.rand_case(10_000 + seed)
    r = random.Random(seed)
    doc = copy.deepcopy(doc)
    pols = [p for s in doc["policy_sets"] for p in s["policies"] if p.get("rules") is not None]
    for p in pols:
        x = r.random()
        if x < 0.3:
            tgt = randgen.rand_target(r, urns, "rule")
            p["rules"].append({"id": p["id"] + "c", "target": tgt, "effect": r.choice(["PERMIT", "DENY"]),
                               "condition": "context && context.subject && context.subject.id === 'Alice'"})
        elif x < 0.5:
            tgt = randgen.rand_target(r, urns, "rule")
            tgt["resources"] = [{"id": randgen.U["entity"], "value": BAD_ENTITY}]
            p["rules"].append({"id": p["id"] + "x", "target": tgt, "effect": r.choice(["PERMIT", "DENY"])})
        elif x < 0.6:
            p["combining_algorithm"] = "urn:bogus:ca"
    for ps in doc["policy_sets"]:  # invalid set combining algorithms end requests where sets decide
        if r.random() < 0.15:
            ps["combining_algorithm"] = "urn:bogus:ca"
    return urns, doc, reqs


def _records(cs, b, monkeypatch, cut):
    if cut:
        monkeypatch.delenv("ACS_NO_CUT", raising=False)
    else:
        monkeypatch.setenv("ACS_NO_CUT", "1")
    return host_core.is_allowed(cs, b).view(np.uint64).copy()


@pytest.mark.parametrize("seed", range(300))
def test_cut_invariance_host(seed, monkeypatch):
    urns, doc, reqs = cut_case(seed)
    o, cs = build(urns, doc)
    b = encoder.Encoder(cs).encode(reqs)
    assert np.array_equal(_records(cs, b, monkeypatch, True), _records(cs, b, monkeypatch, False)), seed


def test_cut_flags():
    """NF_COND_FREE marks exactly the condition-free policies (and sets without condition rules
    or invalid combining algorithms); RES_RX_SAFE marks entity attributes of clean columns."""
    urns, doc, reqs = cut_case(3)
    o, cs = build(urns, doc)
    pol_free = (cs.pols["nflags"] & L.NF_COND_FREE) != 0
    for k, P in enumerate(cs.pols):
        if P["nflags"] & L.NF_NULL:
            continue
        has_cond = any(cs.rules["nflags"][P["child_begin"]:P["child_end"]] & L.NF_HAS_CONDITION)
        assert pol_free[k] == (not has_cond)
    for S in cs.sets:
        ps = cs.pols[S["child_begin"]:S["child_end"]]
        live = ps[(ps["nflags"] & L.NF_NULL) == 0]
        want = all(live["nflags"] & L.NF_COND_FREE) and not any(live["ca"] == L.CA_INVALID)
        assert bool(S["nflags"] & L.NF_COND_FREE) == want
    b = encoder.Encoder(cs).encode(reqs + [{"target": {"subjects": [], "actions": [], "resources": [
        {"id": randgen.U["entity"], "value": "urn:restorecommerce:acs:model:ent1.Ent1"}]}, "context": {}}])
    bad = (b.rx & (L.RX_THROW_TYPE | L.RX_THROW_SYNTAX | L.RX_HOST)).any(axis=1)
    for i in range(b.n):
        for j in range(b.hdr["nres"][i]):
            q = b.res[j, i]
            if q["kind"] & L.K_ENT_LOOSE:
                assert bool(q["pad"] & L.RES_RX_SAFE) == (not bad[q["col"]])
