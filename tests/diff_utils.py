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


def gpu_reverse_query_compact(cs, overlay, bits_row, log, rec):
    """A whatIsAllowed result of the evaluator (inclusion bitset row, maskedProperty log of
    (entity id, mask id) pairs, decision record) in the C++ oracle's compact form
    (oracle/acs_oracle_c.COracle.what_is_allowed), or None for a host-path request."""
    from acs_mi355x import layout as L
    from acs_mi355x.results import bits_layout
    import numpy as np
    f = int(rec["flags"])
    if f & (L.OF_HOST_REQ | L.OF_HOST_COND | L.OF_OBL_OVERFLOW):
        return None
    if f & L.OF_ERR:
        if int(rec["err"]) == L.ERR_REGEX_HOST:
            return None
        return {"k": 1, "e": int(rec["err"])}
    wp, wr, _ = bits_layout(cs.n_sets, cs.n_pols, cs.n_rules)
    row = np.asarray(bits_row, np.uint32)

    def members(off, count):
        words = row[off:off + (count + 31) // 32]
        bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:count]
        return [int(i) for i in np.flatnonzero(bits)]

    def val(i):
        v = overlay.string(int(i))
        if v is MISSING:
            return {"$undef": 1}
        return v

    return {"k": 0, "s": members(0, cs.n_sets), "p": members(wp, cs.n_pols), "r": members(wr, cs.n_rules),
            "o": [[val(e), val(m)] for e, m in np.asarray(log).reshape(-1, 2)]}


class _ListOverlay:
    """id -> value over a plain list (MISSING for {"$undef": 1})."""

    def __init__(self, values):
        self.values = values

    def string(self, i):
        v = self.values[int(i)]
        return MISSING if isinstance(v, dict) and "$undef" in v else v


def compact_reverse_query(cs, c):
    """The C++ oracle's compact whatIsAllowed result -> the reference's ReverseQuery shape
    (results.reverse_query over the same inclusion sets and push log), or ('ERR', kind) /
    None (unsupported)."""
    import numpy as np
    from acs_mi355x import layout as L
    from acs_mi355x.results import bits_layout
    if c["k"] == 2:
        return None
    if c["k"] == 1:
        return ("ERR", {1: "TypeError", 2: "InvalidCombiningAlgorithm", 3: "SyntaxError"}.get(c["e"], "Error"))
    wp, wr, words = bits_layout(cs.n_sets, cs.n_pols, cs.n_rules)
    row = np.zeros(max(words, 1), np.uint32)
    for off, idx in ((0, c["s"]), (wp, c["p"]), (wr, c["r"])):
        for i in idx:
            row[off + (i >> 5)] |= np.uint32(1 << (i & 31))
    vals = [x for pair in c["o"] for x in pair]
    pairs = [(2 * k, 2 * k + 1) for k in range(len(c["o"]))]
    rec = np.zeros(1, L.DECISION_DT)[0]
    return norm_rq(results.reverse_query(cs, _ListOverlay(vals), row, pairs, rec))
