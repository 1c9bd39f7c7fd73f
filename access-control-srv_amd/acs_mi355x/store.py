"""In-memory policy store with the reference's JS-Map semantics.

``AccessController.policySets`` (accessController.ts:32) is a Map of policy
sets whose ``combinables`` are Maps of policies whose ``combinables`` are Maps
of rules.  Python dicts keep insertion order and keep a key's position when it
is re-assigned, exactly like ``Map.prototype.set``; keys are ids (str, or
MISSING for an undefined id).  The compiler snapshots this structure.
"""
from __future__ import annotations

from .jsops import MISSING, truthy

_RULE_FIELDS = ("id", "name", "description", "target", "effect", "condition", "context_query",
                "evaluation_cacheable")
_POLICY_FIELDS = ("id", "name", "description", "target", "effect", "combining_algorithm",
                  "evaluation_cacheable")


def format_target(t):
    """utils.ts:35-45 formatTarget."""
    if not truthy(t):
        return None
    return {k: (t[k] if truthy(t.get(k, MISSING)) else []) for k in ("subjects", "resources", "actions")}


def make_rule(ry: dict) -> dict:
    rule = {k: ry[k] for k in _RULE_FIELDS if k in ry}
    rule["target"] = format_target(ry.get("target", MISSING))
    return rule


def make_policy(py: dict, rules=None) -> dict:
    pol = {k: py[k] for k in _POLICY_FIELDS if k in py}
    pol["target"] = format_target(py.get("target", MISSING))
    pol["combinables"] = rules if rules is not None else {}
    return pol


def make_policy_set(ps: dict, policies=None) -> dict:
    out = {k: ps[k] for k in ("id", "name", "description", "combining_algorithm") if k in ps}
    out["target"] = format_target(ps.get("target", MISSING))
    out["combinables"] = policies if policies is not None else {}
    out["policies"] = []
    return out


def populate(doc: dict, store: dict | None = None) -> dict:
    """Load a ``{policy_sets: [...]}`` document the way the reference's tests do
    (test/utils.ts:345-383): nested YAML -> Maps, later duplicates overwrite in place."""
    store = {} if store is None else store
    for ps in doc.get("policy_sets") or []:
        policies = {}
        for py in ps.get("policies") or []:
            if isinstance(py, dict) and py.get("$null"):  # a null Map entry under this id (fixture form:
                policies[py.get("id", MISSING)] = None  # resourceManager re-reads, accessController.ts:138)
                continue
            rules = {}
            for ry in py.get("rules") or []:
                r = make_rule(ry)
                rules[r.get("id", MISSING)] = r
            p = make_policy(py, rules)
            policies[p.get("id", MISSING)] = p
        s = make_policy_set(ps, policies)
        store[s.get("id", MISSING)] = s
    return store


def stitch_db_documents(policy_sets: list, policies: list, rules: list) -> dict:
    """Flat DB-shaped documents (data/seed_data, resourceManager.ts:765-797,612-643,125-139)
    -> store.  Missing policy ids are skipped; missing rule ids are skipped too
    (the reference only sets a null entry when a per-id re-read finds it)."""
    rule_by_id = {r.get("id"): r for r in rules}
    pol_by_id = {p.get("id"): p for p in policies}
    store = {}
    for ps in policy_sets:
        if not ps.get("policies"):
            continue
        pmap = {}
        for pid in ps["policies"]:
            if pid not in pol_by_id:
                continue
            py = pol_by_id[pid]
            rmap = {}
            for rid in py.get("rules") or []:
                if rid in rule_by_id:
                    rmap[rid] = make_rule(rule_by_id[rid])
            pmap[pid] = make_policy(py, rmap)
        s = make_policy_set(ps, pmap)
        store[s.get("id", MISSING)] = s
    return store
