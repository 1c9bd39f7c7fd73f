"""Decode evaluator output records into the reference's response shapes.

isAllowed  -> ``Response`` (accessController.ts:91-102, 299-323)
whatIsAllowed -> ``ReverseQuery`` (accessController.ts:349-427): the inclusion
bitset selects the policy sets / policies / rules of the compiled snapshot and
the maskedProperty push log is folded exactly like the reference's
``maskPropertyList`` find-or-append (accessController.ts:599-613, 624-638).
"""
from __future__ import annotations

import numpy as np

from . import layout as L
from .jsops import MISSING


class HostPathRequired(Exception):
    """The request needs host-side work the GPU path does not do (JS condition
    eval, subject-token I/O, unsupported shape)."""

    def __init__(self, reason, rule_index=None):
        super().__init__(reason)
        self.reason = reason
        self.rule_index = rule_index


class EvaluationError(Exception):
    """The reference's isAllowed/whatIsAllowed promise rejects with this error kind
    (TypeError, InvalidCombiningAlgorithm, SyntaxError)."""

    def __init__(self, kind):
        super().__init__(kind)
        self.kind = kind


def _raise_err(d):
    """An error record: the reference's rejection, or — ERR_REGEX_HOST — an entity RegExp
    cell outside the precomputed subset, which only the host can decide."""
    if int(d["flags"]) & L.OF_ERR:
        if int(d["err"]) == L.ERR_REGEX_HOST:
            raise HostPathRequired("entity RegExp outside the precomputed subset")
        raise EvaluationError(L.ERR_NAMES.get(int(d["err"]), "Error"))


def _ec_value(cs, code):
    return cs.ec_values[code] if code < len(cs.ec_values) else MISSING


def decision_record(cs, d, reason=None):
    """One Decision record -> Response dict (raises for error / host-path records)."""
    flags = int(d["flags"])
    if flags & L.OF_HOST_REQ:
        raise HostPathRequired(reason or "request flagged for the host path")
    if flags & L.OF_HOST_COND:
        raise HostPathRequired("rule condition (JS eval)", int(d["aux"]))
    _raise_err(d)
    if flags & L.OF_NO_TARGET:
        return {"decision": "DENY", "evaluation_cacheable": False, "obligations": [],
                "operation_status": {"code": 400, "message": "Access request had no target. Skipping request"}}
    return {"decision": L.DECISION_NAMES[int(d["decision"])], "evaluation_cacheable": _ec_value(cs, int(d["ec"])),
            "obligations": [], "operation_status": {"code": 200, "message": "success"}}


def outcome(cs, d):
    """Normalised outcome for parity checks: ('OK', decision, ec) / ('ERR', kind) / ('HOST', why)."""
    try:
        r = decision_record(cs, d)
    except HostPathRequired as e:
        return ("HOST", e.reason)
    except EvaluationError as e:
        return ("ERR", e.kind)
    return ("OK", r["decision"], r["evaluation_cacheable"], r["operation_status"]["code"])


def fold_obligations(cs, overlay, pairs):
    """maskedProperty push log -> obligations list (find by entity value, else append)."""
    ent = cs.urns.get("entity", MISSING)
    masked = cs.urns.get("maskedProperty", MISSING)
    out = []
    for ent_id, mask_id in pairs:
        ev = overlay.string(int(ent_id))
        mv = overlay.string(int(mask_id))
        entry = {"id": masked, "value": mv, "attributes": []}
        hit = None
        for m in out:
            if m["value"] == ev and type(m["value"]) is type(ev):
                hit = m
                break
        if hit is None:
            out.append({"id": ent, "value": ev, "attributes": [entry]})
        else:
            hit["attributes"].append(entry)
    return out


def bits_layout(n_sets, n_pols, n_rules):
    """Word offsets of the policy / rule sections and the row length of a whatIsAllowed
    inclusion bitset (csrc/acs_eval.h BitsLayout): each section starts on a 4-word boundary."""
    def up4(x):
        return (x + 3) & ~3
    wp = up4((n_sets + 31) // 32)
    wr = wp + up4((n_pols + 31) // 32)
    return wp, wr, wr + up4((n_rules + 31) // 32)


def inclusion(cs, bits_row):
    """Bitset row -> (set indices, policy indices, rule indices)."""
    b = np.unpackbits(bits_row.view(np.uint8), bitorder="little")
    ns, npol, nr = cs.n_sets, cs.n_pols, cs.n_rules
    wp, wr, _ = bits_layout(ns, npol, nr)
    return (np.flatnonzero(b[:ns]), np.flatnonzero(b[32 * wp:32 * wp + npol]),
            np.flatnonzero(b[32 * wr:32 * wr + nr]))


def _pick(obj, keys):
    return {k: obj[k] for k in keys if k in obj}


def reverse_query(cs, overlay, bits_row, obl_pairs, d, reason=None):
    """whatIsAllowed response for one request (raises for error / host records)."""
    flags = int(d["flags"])
    if flags & L.OF_HOST_REQ:
        raise HostPathRequired(reason or "request flagged for the host path")
    _raise_err(d)
    if flags & L.OF_OBL_OVERFLOW:
        raise HostPathRequired("maskedProperty log overflow")
    sets, pols, rules = inclusion(cs, bits_row)
    pol_set, rule_set = set(pols.tolist()), set(rules.tolist())
    out = []
    for s in sets.tolist():
        ps = cs.set_objs[s]
        rec = {"combining_algorithm": ps.get("combining_algorithm", MISSING), **_pick(ps, ("id", "target", "effect")),
               "policies": []}
        for p in range(int(cs.sets[s]["child_begin"]), int(cs.sets[s]["child_end"])):
            if p not in pol_set:
                continue
            po = cs.pol_objs[p]
            prq = {"combining_algorithm": po.get("combining_algorithm", MISSING),
                   **_pick(po, ("id", "target", "effect", "evaluation_cacheable")), "rules": [],
                   "has_rules": bool(po.get("combinables"))}
            for r in range(int(cs.pols[p]["child_begin"]), int(cs.pols[p]["child_end"])):
                if r in rule_set:
                    ro = cs.rule_objs[r]
                    prq["rules"].append({"context_query": ro.get("context_query", MISSING),
                                         **_pick(ro, ("id", "target", "effect", "condition", "evaluation_cacheable"))})
            rec["policies"].append(prq)
        out.append(rec)
    return {"policy_sets": out, "obligations": fold_obligations(cs, overlay, obl_pairs),
            "operation_status": {"code": 200, "message": "success"}}
