"""Packed layout of compiled tables and request batches (host side).

Constants are read from ``csrc/acs_layout.h`` / ``csrc/acs_eval.h`` at import
time so the host compiler/encoder and the HIP evaluator cannot drift; the
numpy dtypes below mirror the C structs byte for byte (checked against the
library's own ``sizeof`` by ``acs_layout_sizes`` in the tests).
"""
from __future__ import annotations

import os
import re

import numpy as np

CSRC = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "csrc")


def _parse_constants(*headers):
    consts = {}
    pat = re.compile(r"\b([A-Z][A-Z0-9_]+)\s*=\s*([^,;{}\n/]+)")
    for h in headers:
        with open(os.path.join(CSRC, h)) as f:
            src = f.read()
        src = re.sub(r"//[^\n]*", "", src)
        for name, expr in pat.findall(src):
            e = re.sub(r"(\d+)u\b", r"\1", expr.strip())
            e = e.replace("0xFFFFFFFFu", "0xFFFFFFFF")
            try:
                consts[name] = int(eval(e, {"__builtins__": {}}, dict(consts)))
            except Exception:
                pass
    return consts


C = _parse_constants("acs_layout.h", "acs_eval.h")
globals().update(C)

u8, u16, u32 = np.uint8, np.uint16, np.uint32

NODE_DT = np.dtype([("tflags", u32), ("role", u32), ("se", u32), ("subj_off", u32), ("act_off", u32),
                    ("res_off", u32), ("acl_roles_off", u32), ("last_prop_value", u32),
                    ("subj_n", u16), ("act_n", u16), ("res_n", u16), ("acl_roles_n", u16),
                    ("child_begin", u32), ("child_end", u32), ("map_size", u32), ("fe", u32),
                    ("effect", u8), ("ec", u8), ("ca", u8), ("nflags", u8), ("pe_at", u8), ("pad", u8, 3)])
RULE_RES_DT = np.dtype([("value", u32), ("hash_sfx", u32), ("row", u16), ("kind", u8), ("pad", u8),
                        ("pad2", u32)])
PAIR_DT = np.dtype([("id", u32), ("value", u32)])
REQ_HDR_DT = np.dtype([("flags", u32), ("nres", u8), ("nsubj", u8), ("nact", u8), ("nroles", u8),
                       ("arena_off", u32), ("subject_id", u32)])
REQ_RES_DT = np.dtype([("value", u32), ("hash_sfx", u32), ("col", u16), ("contains", u16), ("kind", u8),
                       ("slot_a", u8), ("slot_b", u8), ("pad", u8)])
DECISION_DT = np.dtype([("decision", u8), ("ec", u8), ("flags", u8), ("err", u8), ("aux", u32)])
# acs_layout.h ReqLine: a request's first rows packed into one 128-B line
REQ_LINE_DT = np.dtype([("h", REQ_HDR_DT), ("res", REQ_RES_DT, (4,)), ("s0", PAIR_DT), ("s1", PAIR_DT),
                        ("a0", PAIR_DT), ("r0", u32), ("r1", u32), ("ar0", u32), ("ar1", u32), ("ext", u32),
                        ("cls2", u32)])
assert REQ_LINE_DT.itemsize == 128


def ext_geom(nres, nsubj, nact, nroles):
    """acs_layout.h ext_geom (vectorised): word offsets of the res / subj / act / roles parts
    of each request's extension record and its padded size."""
    z = np.zeros_like(np.asarray(nres, np.int64))
    g_subj = 4 * np.maximum(np.asarray(nres, np.int64) - LINE_RES, z)
    g_act = g_subj + 2 * np.maximum(np.asarray(nsubj, np.int64) - LINE_SUBJ, z)
    g_roles = g_act + 2 * np.maximum(np.asarray(nact, np.int64) - LINE_ACT, z)
    end = g_roles + np.maximum(np.asarray(nroles, np.int64) - LINE_ROLES, z)
    return z, g_subj, g_act, g_roles, (end + 3) & ~3

SIZES = {"NodeRec": NODE_DT.itemsize, "RuleResAttr": RULE_RES_DT.itemsize, "ReqHdr": REQ_HDR_DT.itemsize,
         "ReqRes": REQ_RES_DT.itemsize, "Decision": DECISION_DT.itemsize}
assert SIZES == {"NodeRec": 64, "RuleResAttr": 16, "ReqHdr": 16, "ReqRes": 16, "Decision": 8}, SIZES

DECISION_NAMES = {C["DEC_PERMIT"]: "PERMIT", C["DEC_DENY"]: "DENY", C["DEC_NOT_APPLICABLE"]: "NOT_APPLICABLE",
                  C["DEC_INDETERMINATE"]: "INDETERMINATE", C["DEC_UNRECOGNIZED"]: "UNRECOGNIZED"}
ERR_NAMES = {C["ERR_TYPE"]: "TypeError", C["ERR_INVALID_CA"]: "InvalidCombiningAlgorithm",
             C["ERR_REGEX_SYNTAX"]: "SyntaxError", C["ERR_REGEX_HOST"]: "RegexHost"}
