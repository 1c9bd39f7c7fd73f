"""Shared helpers for the golden-vector (KAT) tests."""
import json
import os

from oracle.acs_oracle import Oracle, CORE_SPEC_URNS, FULL_URNS, NodeConditionEvaluator
from oracle.jsval import UNDEF

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load_kats():
    with open(os.path.join(GOLDEN, "kats.json")) as f:
        return json.load(f)["vectors"]


def load_fixture(name):
    with open(os.path.join(GOLDEN, "fixtures", name.replace(".yml", ".json"))) as f:
        return json.load(f)


def urns_for(vec):
    return CORE_SPEC_URNS if vec["urns"] == "core" else FULL_URNS


def oracle_for(vec, cond=None):
    o = Oracle(urns=urns_for(vec), condition_eval=cond)
    o.load(load_fixture(vec["fixture"]))
    return o


def _walk(obj, path):
    cur = obj
    for k in path:
        if isinstance(cur, dict):
            cur = cur.get(k, UNDEF)
        elif isinstance(cur, list) and isinstance(k, int):
            cur = cur[k] if k < len(cur) else UNDEF
        elif isinstance(cur, list) and k == "length":
            cur = len(cur)
        else:
            return UNDEF
        if cur is UNDEF or cur is None:
            return cur
    return cur


def check_asserts(result, asserts):
    """Evaluate the spec's path assertions against a whatIsAllowed result.
    ``not_exists`` on a repeated field accepts the empty list (proto3 default)."""
    failures = []
    for path, op, val in asserts:
        v = _walk(result, path)
        ok = True
        if op == "exists":
            ok = v is not UNDEF and v is not None
        elif op == "not_exists":
            ok = v is UNDEF or v is None or v == []
        elif op == "len":
            ok = isinstance(v, list) and len(v) == val
        elif op == "eq":
            ok = v == val
        if not ok:
            failures.append((path, op, val, v))
    return failures
