"""AccessController mirror (acs_mi355x.controller) against the oracle.

CPU tests inject the CPU build of the evaluator core as the engine (the product
default is the GPU library); the gpu-marked test runs the default engine.
Covers: the reference's surface and Map-assignment idiom, recompile on every
store mutator (accessController.ts:79,897-937), per-request rejection, host
fallback delegation, constructor validation of combining algorithms.
"""
import copy
import random

import pytest

import host_core
import randgen
from diff_utils import oracle_outcome, _norm
from kat_utils import load_kats, load_fixture, urns_for, oracle_for
from oracle.acs_oracle import Oracle, DEFAULT_CAS, populate_store, NodeConditionEvaluator, _Key
from oracle.jsval import JSError
from acs_mi355x import store as pstore
from acs_mi355x.controller import AccessController, InvalidCombiningAlgorithm, HostPathRequired, EvaluationError

KATS = load_kats()


def _ctl(urns, **kw):
    return AccessController({"urns": urns, "combiningAlgorithms": DEFAULT_CAS}, engine=host_core.Tables, **kw)


def _outcome(r):
    if isinstance(r, EvaluationError):
        return ("ERR", r.kind)
    if isinstance(r, Exception):
        return ("HOST",)
    return ("OK", r["decision"], _norm(r["evaluation_cacheable"]), r["operation_status"]["code"])


def test_invalid_combining_algorithm_rejected():
    with pytest.raises(InvalidCombiningAlgorithm):
        AccessController({"urns": {}, "combiningAlgorithms": [{"urn": "x", "method": "nope"}]},
                         engine=host_core.Tables)


@pytest.mark.parametrize("fixture", sorted({v["fixture"] for v in KATS if v["op"] == "isAllowed"}))
def test_controller_kats(fixture):
    vecs = [v for v in KATS if v["fixture"] == fixture and v["op"] == "isAllowed"]
    for urns_kind in sorted({v["urns"] for v in vecs}):
        group = [v for v in vecs if v["urns"] == urns_kind]
        oracle = oracle_for(group[0], NodeConditionEvaluator())
        ctl = _ctl(urns_for(group[0]), host_evaluator=lambda op, req: oracle.is_allowed(req))
        ctl.policySets = pstore.populate(load_fixture(fixture))  # accessControlService.ts:50 idiom
        got = ctl.isAllowed_batch([v["request"] for v in group])
        for v, r in zip(group, got):
            assert not isinstance(r, Exception), (v["spec"], r)
            assert r["decision"] == v["expect"]["decision"], v["spec"]
        assert ctl.stats["compiles"] == 1


def test_what_is_allowed_through_controller():
    from kat_utils import check_asserts
    vecs = [v for v in KATS if v["op"] == "whatIsAllowed"]
    for v in vecs:
        ctl = _ctl(urns_for(v))
        ctl.policySets = pstore.populate(load_fixture(v["fixture"]))
        rq = ctl.whatIsAllowed(v["request"])
        assert check_asserts(rq, v["expect"]["asserts"]) == [], v["spec"]


def _wrap(ry=None, py=None, ps=None):
    """One rule / policy / set in both representations (product store, oracle store)."""
    if ry is not None:
        doc = {"policy_sets": [{"id": "w", "policies": [{"id": "w", "rules": [ry]}]}]}
        pick = lambda st, k: next(iter(next(iter(st[k]["combinables"].values()))["combinables"].values()))  # noqa: E731
    elif py is not None:
        doc = {"policy_sets": [{"id": "w", "policies": [py]}]}
        pick = lambda st, k: next(iter(st[k]["combinables"].values()))  # noqa: E731
    else:
        doc = {"policy_sets": [ps]}
        pick = lambda st, k: next(iter(st.values()))  # noqa: E731
    return pick(pstore.populate(copy.deepcopy(doc)), "w"), pick(populate_store(copy.deepcopy(doc)), _Key("w"))


@pytest.mark.parametrize("seed", range(0, 60, 3))
def test_controller_mutations_match_oracle(seed):
    urns, doc, reqs = randgen.rand_case(seed)
    r = random.Random(seed)
    o = Oracle(urns=urns)
    o.load(doc)
    ctl = _ctl(urns)
    ctl.policySets = pstore.populate(doc)

    def check():
        got = ctl.isAllowed_batch(reqs)
        for q, g in zip(reqs, got):
            if _outcome(g)[0] == "HOST":
                continue
            try:
                want = oracle_outcome(o, q)
            except Exception:  # noqa: BLE001 — oracle-unsupported shapes
                continue
            assert _outcome(g) == want

    check()
    n0 = ctl.stats["compiles"]
    # mutate only entries with string ids (None / absent ids are distinct JS Map keys)
    ids = [(ps["id"], [(p["id"], [ru["id"] for ru in (p.get("rules") or []) if isinstance(ru.get("id"), str)])
                       for p in (ps.get("policies") or []) if isinstance(p, dict) and isinstance(p.get("id"), str)])
           for ps in doc["policy_sets"] if isinstance(ps.get("id"), str)]
    for step in range(6):
        op = r.choice(["rule+", "rule-", "pol+", "pol-", "set+", "set-"])
        sid, pols = r.choice(ids)
        if op in ("rule+", "rule-") and pols:
            pid, rids = r.choice(pols)
            if op == "rule+":
                ry = {"id": r.choice(rids + ["new"]), "effect": r.choice(["PERMIT", "DENY"]),
                      "target": randgen.rand_target(r, urns, "rule")}
                a, b = _wrap(ry=ry)
                ctl.updateRule(sid, pid, a)
                o.update_rule(sid, pid, b)
            elif rids:
                rid = r.choice(rids)
                ctl.removeRule(sid, pid, rid)
                o.remove_rule(sid, pid, rid)
        elif op == "pol+":
            py = {"id": r.choice([p for p, _ in pols] + ["newp"]), "effect": r.choice(["PERMIT", "DENY", None]),
                  "combining_algorithm": r.choice(randgen.CAS), "target": randgen.rand_target(r, urns, "policy"),
                  "rules": [{"id": "nr", "effect": "PERMIT", "target": randgen.rand_target(r, urns, "rule")}]}
            a, b = _wrap(py=py)
            ctl.updatePolicy(sid, a)
            o.update_policy(sid, b)
        elif op == "pol-" and pols:
            pid = r.choice(pols)[0]
            ctl.removePolicy(sid, pid)
            o.remove_policy(sid, pid)
        elif op == "set+":
            ps = {"id": r.choice([sid, "news"]), "combining_algorithm": r.choice(randgen.CAS),
                  "policies": [{"id": "p", "effect": "DENY", "combining_algorithm": randgen.CAS[0],
                                "rules": [{"id": "x", "effect": r.choice(["PERMIT", "DENY"]),
                                           "target": randgen.rand_target(r, urns, "rule")}]}]}
            a, b = _wrap(ps=ps)
            ctl.updatePolicySet(a)
            o.update_policy_set(b)
        elif op == "set-":
            ctl.removePolicySet(sid)
            o.remove_policy_set(sid)
        check()
    assert ctl.stats["compiles"] >= n0
    ctl.clearPolicies()
    o.clear_policies()
    check()


def test_recompile_only_after_mutation():
    urns, doc, reqs = randgen.rand_case(5)
    ctl = _ctl(urns)
    ctl.policySets = pstore.populate(doc)
    ctl.isAllowed_batch(reqs)
    ctl.isAllowed_batch(reqs)
    assert ctl.stats["compiles"] == 1
    ctl.removePolicySet("definitely-not-there")  # Map.delete of a missing key still counts as a write
    ctl.isAllowed_batch(reqs)
    assert ctl.stats["compiles"] == 2
    ctl.updateRule("no-set", "no-policy", {"id": "r"})  # _.isNil guard: no change
    ctl.isAllowed_batch(reqs)
    assert ctl.stats["compiles"] == 2


def test_host_path_without_evaluator_raises():
    vec = next(v for v in KATS if v["fixture"] == "conditions.yml" and v["op"] == "isAllowed")
    ctl = _ctl(urns_for(vec))
    ctl.policySets = pstore.populate(load_fixture(vec["fixture"]))
    got = ctl.isAllowed_batch([v["request"] for v in KATS
                               if v["fixture"] == "conditions.yml" and v["op"] == "isAllowed"])
    assert any(isinstance(g, HostPathRequired) for g in got)
    with pytest.raises(HostPathRequired):
        for v in KATS:
            if v["fixture"] == "conditions.yml" and v["op"] == "isAllowed":
                ctl.isAllowed(v["request"])


def test_no_target_and_rejections():
    urns, doc, _ = randgen.rand_case(7)
    ctl = _ctl(urns)
    ctl.policySets = pstore.populate(doc)
    r = ctl.isAllowed({"context": {}})
    assert r["decision"] == "DENY" and r["operation_status"]["code"] == 400
    bad = copy.deepcopy(doc)
    bad["policy_sets"][0]["policies"][0]["combining_algorithm"] = "urn:unknown"
    ctl.policySets = pstore.populate(bad)
    o = Oracle(urns=urns)
    o.load(bad)
    _, _, reqs = randgen.rand_case(7)
    for q, g in zip(reqs, ctl.isAllowed_batch(reqs)):
        try:
            want = oracle_outcome(o, q)
        except Exception:  # noqa: BLE001
            continue
        if _outcome(g)[0] != "HOST":
            assert _outcome(g) == want


@pytest.mark.gpu
def test_controller_default_engine_gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    vecs = [v for v in KATS if v["fixture"] == "roleScopes.yml" and v["op"] == "isAllowed"]
    ctl = AccessController({"urns": urns_for(vecs[0]), "combiningAlgorithms": DEFAULT_CAS}, device=0)
    ctl.policySets = pstore.populate(load_fixture("roleScopes.yml"))
    for v, r in zip(vecs, ctl.isAllowed_batch([v["request"] for v in vecs])):
        assert r["decision"] == v["expect"]["decision"]
    ctl.close()


def test_many_updates_keep_tables_bounded():
    """Hundreds of updateRule / removeRule cycles on one controller, each with a new entity
    value: stale dictionary entries / regex rows are reclaimed by a fresh compile, decisions
    stay equal to the oracle's, and the append-only tables stay near the live store's size."""
    urns = randgen.U
    doc = {"policy_sets": [{"id": "s", "combining_algorithm": randgen.CAS[0], "policies": [
        {"id": "p", "combining_algorithm": randgen.CAS[1], "rules": []}]}]}
    ctl = _ctl(urns)
    ctl.policySets = pstore.populate(doc)
    o = Oracle(urns=urns)
    o.load(doc)

    def rule(k):
        return {"id": f"r{k % 3}", "effect": "PERMIT" if k % 2 else "DENY",
                "target": {"subjects": [{"id": urns["role"], "value": "u"}],
                           "resources": [{"id": urns["entity"], "value": f"urn:x:model:e{k}.E{k}"}]}}

    def req(k):
        return {"target": {"subjects": [{"id": urns["role"], "value": "u"}],
                           "resources": [{"id": urns["entity"], "value": f"urn:x:model:e{k}.E{k}"}]},
                "context": {"subject": {"id": "a", "role_associations": [{"role": "u"}], "hierarchical_scopes": []},
                            "resources": []}}
    for k in range(400):
        a, b = _wrap(ry=rule(k))
        ctl.updateRule("s", "p", a)
        o.update_rule("s", "p", b)
        if k % 7 == 0:
            ctl.removeRule("s", "p", f"r{(k + 1) % 3}")
            o.remove_rule("s", "p", f"r{(k + 1) % 3}")
        if k % 4 == 0:  # a compile: each one interns the live rules' values
            ctl.isAllowed(req(k))
        if k % 25 == 0:
            for q in (req(k), req(k - 1), req(k + 1)):
                assert _outcome(ctl.isAllowed(q)) == oracle_outcome(o, q)
    assert ctl.stats["compiler_resets"] >= 2
    assert len(ctl._compiler.b.rx_rows) <= 2 * 3 + 64
