"""Candidate bitsets over (sets | policies | rules), one row per request class.

A node can only influence a request — match, push an effect, throw, or push a
maskedProperty obligation — when its target passes ``checkSubjectMatches``
(accessController.ts:793-823) and ``resourceAttributesMatch`` can return
something other than a plain ``false`` (:465-654).  Both tests are cheap to
bound per request *class*:

* entity: ``resourceAttributesMatch`` needs some request entity attribute to hit
  a rule entity attribute (exact ===, or the namespace/RegExp test of :528-566),
  unless the target has operation attributes or no resources;
* role: a target whose subjects carry a role (``TF_SUBJ_ROLE``) matches only
  when one of ``context.subject.role_associations[*].role`` equals the target's
  last role value (:797-806); ``checkSubjectMatches`` runs before anything that
  can throw or push, so a failed role test makes the node inert.

A class is (entity column of the request's entity attributes, set of the
request's role-association roles that some target requires).  Its row is the
AND of the two node filters; a set is kept only if one of its policies is.
``policyEffect`` / ``evaluation_cacheable`` do not depend on which nodes are
visited (the compiler's ``pe_at`` / ``fe`` prefixes), so the kernel may iterate
only the class's candidates, in table order.

Layout: ``cand[class][W]`` u32 words, W = ws + wp + wr (set, policy, rule
sections).  The class id sits in the request header's flags (``RQ_PCOL_SHIFT``);
``PCOL_ALL`` means "evaluate every node" (several distinct entity columns).
"""
from __future__ import annotations

import numpy as np
from scipy import sparse

from . import layout as L
from .jsops import MISSING

_HIT_LIKE = L.RX_HIT | L.RX_THROW_TYPE | L.RX_THROW_SYNTAX | L.RX_HOST
MAX_CLASSES = L.PCOL_ALL  # ids 0 .. 0xFFFE
_CHUNK = 2048


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
    """bool [rows, n] -> u32 [rows, nwords], bit i of word w = node 32w+i."""
    rows, n = bits.shape
    padded = np.zeros((rows, nwords * 32), bool)
    padded[:, :n] = bits
    b = np.packbits(padded, axis=1, bitorder="little")
    return np.ascontiguousarray(b).view("<u4").reshape(rows, nwords)


def entity_candidates(cs, col_values, rx: np.ndarray):
    """bool [ncols + 1, n] per section (sets, policies, rules): nodes whose targets can
    hit a request entity value of that regex-matrix column (row ncols: no entity attr)."""
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
    out = []
    for spec in cs.cand_spec:
        always, A = _spec_matrix(spec, nrows)
        hit = (sparse.csr_matrix(rowmask) @ A.T).toarray() > 0 if A.nnz else np.zeros((ncols + 1, len(spec)), bool)
        out.append(hit | always[None, :])
    return tuple(out)


def role_requirements(cs):
    """(sorted role ids some target requires, per-section int arrays: role row or -1)."""
    req = []
    for nodes in (cs.sets, cs.pols, cs.rules):
        tf, nf = nodes["tflags"], nodes["nflags"]
        need = ((nf & L.NF_HAS_TARGET) != 0) & ((tf & L.TF_SUBJ_ROLE) != 0) & ((tf & L.TF_SUBJ_EMPTY) == 0)
        req.append(np.where(need, nodes["role"].astype(np.int64), -1))
    role_ids = np.unique(np.concatenate([r[r >= 0] for r in req])) if req else np.zeros(0, np.int64)
    rows = [np.where(r >= 0, np.searchsorted(role_ids, np.maximum(r, 0)), -1) for r in req]
    return role_ids, rows


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


def _role_sets(hdr, roles, role_ids):
    """Per request: sorted role rows of its role associations (-1 padded), [n, R]."""
    n = len(hdr)
    R = roles.shape[0]
    ra = (hdr["flags"] & L.RQ_RA_TRUTHY) != 0
    rows = np.full((n, R), -1, np.int64)
    if len(role_ids) == 0:
        return rows
    for k in range(R):
        v = roles[k].astype(np.int64)
        pos = np.searchsorted(role_ids, v)
        posc = np.minimum(pos, len(role_ids) - 1)
        hit = (role_ids[posc] == v) & (k < hdr["nroles"]) & ra
        rows[:, k] = np.where(hit, posc, -1)
    rows.sort(axis=1)
    # drop duplicates inside a request so equal sets give equal keys
    dup = np.zeros_like(rows, bool)
    dup[:, 1:] = rows[:, 1:] == rows[:, :-1]
    rows[dup] = -1
    rows.sort(axis=1)
    return rows


def classes(cs, hdr, roles, pcol, ent):
    """Class id per request (u32, PCOL_ALL = unfiltered) and the class rows [C, W] u32."""
    role_ids, req_rows = role_requirements(cs)
    nrr = len(role_ids)
    n = len(hdr)
    active = (pcol != L.PCOL_ALL) & ((hdr["flags"] & (L.RQ_HOST | L.RQ_NO_TARGET)) == 0)
    rs = _role_sets(hdr, roles, role_ids)
    used = rs[:, ::-1]  # largest rows first; -1 padding last
    width = int((used >= 0).sum(axis=1).max()) if n else 0
    key = np.concatenate([pcol.astype(np.int64)[:, None], used[:, :max(width, 1)]], axis=1)
    cls = np.full(n, L.PCOL_ALL, np.uint32)
    if not active.any():
        return cls, np.zeros((1, sum(section_words(cs))), np.uint32)
    if key.shape[1] <= 4 and nrr < (1 << 15):
        # pack into one int64 for a fast unique: pcol:16 | up to 3 rows of 15 bits (+1 offset)
        packed = key[:, 0].copy()
        for j in range(1, key.shape[1]):
            packed = (packed << 15) | (key[:, j] + 1)
        uk, inv = np.unique(packed[active], return_inverse=True)
        first = np.zeros(len(uk), np.int64)
        first[inv[::-1]] = np.flatnonzero(active)[::-1]
        ckey = key[first]
    else:
        ckey, inv = np.unique(key[active], axis=0, return_inverse=True)
        inv = inv.reshape(-1)
    if len(ckey) > MAX_CLASSES:  # too many classes: entity-only filtering
        ckey, inv = np.unique(key[active, :1], axis=0, return_inverse=True)
        ckey = np.concatenate([ckey, np.full((len(ckey), 1), -1, np.int64)], axis=1)
        inv = inv.reshape(-1)
        role_filter = False
    else:
        role_filter = True
    cls[active] = inv.astype(np.uint32)

    E_s, E_p, E_r = ent
    ws, wp, wr = section_words(cs)
    b_s = cs.sets["child_begin"].astype(np.int64)
    e_s = cs.sets["child_end"].astype(np.int64)
    nonempty = e_s > b_s
    out = np.zeros((len(ckey), ws + wp + wr), np.uint32)
    for c0 in range(0, len(ckey), _CHUNK):
        ck = ckey[c0:c0 + _CHUNK]
        pc = ck[:, 0]
        M = np.zeros((len(ck), nrr + 1), bool)
        M[:, nrr] = True  # "no role requirement" column
        if role_filter:
            for j in range(1, ck.shape[1]):
                v = ck[:, j]
                ok = v >= 0
                M[np.flatnonzero(ok), v[ok]] = True
        else:
            M[:, :] = True

        def role_ok(rr):
            return M[:, np.where(rr >= 0, rr, nrr)]

        p = E_p[pc] & role_ok(req_rows[1])
        r = E_r[pc] & role_ok(req_rows[2])
        s = E_s[pc] & role_ok(req_rows[0])
        if cs.n_pols:
            cum = np.concatenate([np.zeros((len(ck), 1), np.int64), np.cumsum(p, axis=1)], axis=1)
            pol_any = (cum[:, e_s] - cum[:, b_s]) > 0
        else:
            pol_any = np.zeros((len(ck), cs.n_sets), bool)
        s &= pol_any & nonempty[None, :]
        out[c0:c0 + len(ck)] = np.concatenate([_pack(s, ws), _pack(p, wp), _pack(r, wr)], axis=1)
    # heaviest classes first: the kernel's sort key orders waves by class id, so the longest
    # waves are dispatched first (longest-processing-time-first; no tail of heavy waves)
    cost = np.unpackbits(out.view(np.uint8), axis=1).sum(axis=1)
    rank = np.empty(len(cost), np.int64)
    rank[np.argsort(-cost, kind="stable")] = np.arange(len(cost))
    out = np.ascontiguousarray(out[np.argsort(rank)])
    cls[active] = rank[inv].astype(np.uint32)
    return cls, out
