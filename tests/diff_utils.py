"""Differential comparison helpers: evaluator outcome vs oracle outcome."""
from oracle.acs_oracle import Oracle, DEFAULT_CAS, populate_store, _Key
from oracle.jsval import OracleUnsupported, JSError, UNDEF
from acs_mi355x import store as pstore, compiler, encoder, results
from acs_mi355x.jsops import MISSING


def _norm(v):
    return "undefined" if (v is UNDEF or v is MISSING) else v


def oracle_outcome(o, req):
    try:
        r = o.is_allowed(req)
    except JSError as e:
        return ("ERR", e.kind)
    return ("OK", r["decision"], _norm(r["evaluation_cacheable"]), r["operation_status"]["code"])


def gpu_outcome(cs, d):
    oc = results.outcome(cs, d)
    if oc[0] == "OK":
        return ("OK", oc[1], _norm(oc[2]), oc[3])
    return oc


def build(urns, doc, cond=None):
    o = Oracle(urns=urns, condition_eval=cond)
    o.load(doc)
    cs = compiler.compile_store(pstore.populate(doc), urns, DEFAULT_CAS)
    return o, cs


def norm_rq(x):
    """Normalise a ReverseQuery (oracle or decoded) for equality: undefined-valued keys dropped."""
    if isinstance(x, dict):
        return {k: norm_rq(v) for k, v in x.items() if not (v is UNDEF or v is MISSING)}
    if isinstance(x, list):
        return [norm_rq(v) for v in x]
    return x


def oracle_from_store(urns, policy_sets):
    """An Oracle holding the product's policySets Map (acs_mi355x.store shape: MISSING for
    undefined, plain keys) in its own shape (UNDEF, SameValueZero _Key keys)."""
    def v(x):
        if x is MISSING:
            return UNDEF
        if isinstance(x, dict):
            return {k: v(y) for k, y in x.items()}
        if isinstance(x, list):
            return [v(y) for y in x]
        return x

    def level(m, depth):
        out = {}
        for k, obj in m.items():
            if isinstance(obj, dict) and depth < 2:
                o = {kk: v(vv) for kk, vv in obj.items() if kk != "combinables"}
                o["combinables"] = level(obj.get("combinables") or {}, depth + 1)
            else:
                o = v(obj)
            out[_Key(v(k))] = o
        return out

    o = Oracle(urns=urns)
    o.policy_sets = level(policy_sets, 0)
    return o


def controller_outcome(r):
    """A controller isAllowed_batch entry (Response dict or exception) -> outcome tuple."""
    if isinstance(r, results.HostPathRequired):
        return ("HOST", r.reason)
    if isinstance(r, results.EvaluationError):
        return ("ERR", r.kind)
    if isinstance(r, Exception):
        return ("EXC", repr(r))
    return ("OK", r["decision"], _norm(r["evaluation_cacheable"]), r["operation_status"]["code"])
