"""Differential comparison helpers: evaluator outcome vs oracle outcome."""
from oracle.acs_oracle import Oracle, DEFAULT_CAS, populate_store
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
