"""Per-entity candidate bitsets over (sets | policies | rules).

resourceAttributesMatch (accessController.ts:465-654) can only return true —
or push a maskedProperty obligation, or throw — when some request entity
attribute hits a rule entity attribute (exact ===, or the namespace/RegExp test
of accessController.ts:528-566), or when the rule has operation attributes or
no resources.  So, for a request entity value (a regex-matrix column), every
target whose entity rows cannot hit it is provably inert: skipping it changes
no decision, no evaluation_cacheable, no obligation and no error.  Combined
with the per-policy ``pe_at`` / ``fe`` prefixes (policyEffect and
evaluation_cacheable do not depend on which nodes are visited), the kernel
iterates only candidate nodes, in table order.

Layout: ``cand[col][W]`` u32 words, W = ws + wp + wr with the set, policy and
rule sections concatenated; row ``ncols`` is the "no entity attribute" column.
"""
from __future__ import annotations

import numpy as np
from scipy import sparse

from . import layout as L
from .jsops import MISSING

_HIT_LIKE = L.RX_HIT | L.RX_THROW_TYPE | L.RX_THROW_SYNTAX | L.RX_HOST


def words(n):
    return (n + 31) // 32


def section_words(cs):
    return words(cs.n_sets), words(cs.n_pols), words(cs.n_rules)


def _key(v):
    return ("m",) if v is MISSING else (("n",) if v is None else ("s", v))


def _spec_matrix(spec, nrows):
    """(always bool[n], sparse [n, nrows]) from per-node specs."""
    n = len(spec)
    always = np.zeros(n, bool)
    ptr, idx = [0], []
    for k, sp in enumerate(spec):
        if sp is None:
            always[k] = True
        else:
            idx.extend(sp)
        ptr.append(len(idx))
    data = np.ones(len(idx), np.int32)
    A = sparse.csr_matrix((data, np.array(idx, np.int64), np.array(ptr, np.int64)), shape=(n, max(nrows, 1)))
    return always, A


def _pack(bits: np.ndarray, nwords: int) -> np.ndarray:
    """bool [ncols, n] -> u32 [ncols, nwords], bit i of word w = node 32w+i."""
    ncols, n = bits.shape
    padded = np.zeros((ncols, nwords * 32), bool)
    padded[:, :n] = bits
    b = np.packbits(padded, axis=1, bitorder="little")
    return np.ascontiguousarray(b).view("<u4").reshape(ncols, nwords)


def build(cs, col_values, rx: np.ndarray) -> np.ndarray:
    """Candidate words for each regex-matrix column (plus the no-entity column)."""
    nrows = len(cs.rx_rows)
    ncols = len(col_values)
    rowmask = np.zeros((ncols + 1, max(nrows, 1)), np.int32)
    if nrows and ncols:
        rowmask[:ncols, :nrows] = (rx[:ncols, :nrows] & _HIT_LIKE) != 0
        row_of = {_key(v): r for r, v in enumerate(cs.rx_rows)}
        for c, v in enumerate(col_values):
            if not (v is MISSING or v is None or isinstance(v, str)):
                continue  # padding column
            r = row_of.get(_key(v))
            if r is not None:
                rowmask[c, r] = 1  # exact === on the same value
    spec_s, spec_p, spec_r = cs.cand_spec
    out = []
    cand = {}
    for name, spec in (("s", spec_s), ("p", spec_p), ("r", spec_r)):
        always, A = _spec_matrix(spec, nrows)
        hit = (sparse.csr_matrix(rowmask) @ A.T).toarray() > 0 if A.nnz else np.zeros((ncols + 1, len(spec)), bool)
        cand[name] = hit | always[None, :]
    # a set is only worth visiting when one of its policies is a candidate
    pols_any = np.zeros((ncols + 1, cs.n_sets), bool)
    for s in range(cs.n_sets):
        b, e = int(cs.sets[s]["child_begin"]), int(cs.sets[s]["child_end"])
        if e > b:
            pols_any[:, s] = cand["p"][:, b:e].any(axis=1)
    cand["s"] &= pols_any
    ws, wp, wr = section_words(cs)
    out = np.concatenate([_pack(cand["s"], ws), _pack(cand["p"], wp), _pack(cand["r"], wr)], axis=1)
    return np.ascontiguousarray(out, dtype=np.uint32)


def primary_columns(res_kind, res_col, nres, ncols):
    """Per request: the column of its entity attributes if they all share one, else the
    no-entity column (none) or PCOL_ALL (several distinct entity columns)."""
    n = len(nres)
    pcol = np.full(n, ncols, np.uint32)
    seen = np.zeros(n, bool)
    for j in range(res_kind.shape[0]):
        has = (j < nres) & ((res_kind[j] & L.K_ENT) != 0)
        c = res_col[j].astype(np.uint32)
        diff = has & seen & (pcol != c)
        pcol = np.where(has & ~seen, c, pcol)
        pcol = np.where(diff, L.PCOL_ALL, pcol)
        seen |= has
    return pcol
