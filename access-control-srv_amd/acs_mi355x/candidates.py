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

Useful sections (isAllowed only).  Most candidate sets and policies cannot change an
isAllowed result: a policy contributes only when one of its rules can match (a candidate
rule), when it is an effect-only policy (no rules, truthy effect: accessController.ts:
159-163), or when its own target evaluation can throw (a RegExp cell that throws or needs
the host for the class's entity column; a subjects list, whose checkHierarchicalScope can
throw; a target-bearing policy without an entity filter).  A set contributes only through
such a policy, or by throwing in loop 2a (a null policy).  Visiting anything else leaves
the decision, evaluation_cacheable and the error state exactly as they were, so K1 walks
the *useful* sets, scans loop 2a over the candidate policies (they decide `exact` and
`policyEffect`) and walks loop 2b over the useful policies only.  whatIsAllowed keeps the
candidate sections (its obligations are pushed by any matching target).

Composed rows (two required roles).  A request whose role associations name two roles some
target requires has the key (entity, action, {a, b}); at 10M c3 requests with 1-2 roles there
are ~0.7M such keys, too many rows.  The "composed" level keys rows by one role — (entity,
action, a) and (entity, action, b) — and the kernel ORs the request's two rows
(ReqLine.cls2).  checkSubjectMatches' role test is an OR over the request's roles, so the
candidate rule and policy sections compose exactly; the derived sections are built
role-relaxed so that their OR covers the joint key's: candidate sets ignore set targets' role
tests (a set kept because a role-free candidate policy is in it), and a policy is useful
through a candidate rule when its target passes with the role test ignored (``_useful_relaxed``).
The target verdicts compose too: known true = OR, known false = AND (both rows know it).  For
stores whose set / policy targets carry no role (c3, c5) the relaxed rows equal the exact ones.

Layout: ``cand[class][W]`` u32 words, sections in this order: candidate sets (ws words),
candidate policies (wp), useful sets (ws), useful policies (wp), candidate rules (wr);
W = 2 ws + 2 wp + wr.  The class id sits in the request header's flags
(``RQ_PCOL_SHIFT``); ``PCOL_ALL`` means "evaluate every node" (several distinct entity
columns).
"""
from __future__ import annotations

import numpy as np
from scipy import sparse

from . import layout as L
from .jsops import MISSING

_HIT_LIKE = L.RX_HIT | L.RX_THROW_TYPE | L.RX_THROW_SYNTAX | L.RX_HOST
MAX_CLASSES = L.PCOL_ALL  # ids 0 .. 0xFFFE
_CHUNK = 2048
_CHUNK_NODE_BITS = 1 << 27  # bools per section array of one chunk (large stores: fewer keys)
_MAX_ACTION_KEYS = 62
_KEY_ROW_BYTES = 512 << 20  # candidate rows computed per batch before dedupe
_ROLE_ROW_BYTES = 256 << 20  # role-factor rows per batch
FORCE_LEVEL = None  # tests: pin the class key level (and with it the role factor)


_THROW_LIKE = L.RX_THROW_TYPE | L.RX_THROW_SYNTAX | L.RX_HOST


def words(n):
    return (n + 31) // 32


def section_words(cs):
    return words(cs.n_sets), words(cs.n_pols), words(cs.n_rules)


def row_layout(cs):
    """Word offsets of a class row's sections: (wp, wsu, wpu, wr, W) — candidate policies,
    useful sets, useful policies, candidate rules, row length (candidate sets start at 0;
    the target verdicts follow the rules at verdict_offset)."""
    ws, wp, wr = section_words(cs)
    return ws, ws + wp, 2 * ws + wp, 2 * ws + 2 * wp, 2 * ws + 6 * wp + 2 * wr


def verdict_offset(cs):
    """Word offset of the target-verdict sections: policies known exact-true, exact-false,
    RegExp-true, RegExp-false (wp words each), then rules whose retried match is known true
    (wr words)."""
    ws, wp, wr = section_words(cs)
    return 2 * ws + 2 * wp + wr


def _assemble(s, p, us, up, r, cs, verdicts=None):
    ws, wp, wr = section_words(cs)
    parts = [_pack(s, ws), _pack(p, wp), _pack(us, ws), _pack(up, wp), _pack(r, wr)]
    if verdicts is None:
        parts.append(np.zeros((s.shape[0], 4 * wp + wr), np.uint32))
    else:
        pxt, pxf, prt, prf, qt = verdicts
        parts += [_pack(pxt, wp), _pack(pxf, wp), _pack(prt, wp), _pack(prf, wp), _pack(qt, wr)]
    return np.concatenate(parts, axis=1)


# ------------------------------------------------------------------ target verdicts
# For a request class, a target whose subjects are empty or a role test, whose actions are
# none or a single pair the class fixes, and whose resources are empty or entity-only has
# the same targetMatches result for every request of the class: checkSubjectMatches is role
# membership (the class holds the request's required roles), attributesMatch on actions
# compares against the class's single action pair, and an entity-only
# resourceAttributesMatch depends only on the entity value of the class's column — exactly
# (===), or through the RegExp cells in the rule attribute order (the last cell that resets
# or hits decides; a throwing cell leaves the verdict unknown).  K1 reads these bits for a
# wave whose lanes share one class and skips the matching (accessController.ts:661-672).

def resource_verdicts(cs, col_values, rx, sec):
    """Per column (ncols + 1 rows; the last = no entity attribute) and node of section `sec`
    (1 policies, 2 rules): (exact true, exact false, RegExp true, RegExp false) of an empty or
    entity-only resourceAttributesMatch; all False where unknown."""
    nodes = (cs.sets, cs.pols, cs.rules)[sec]
    spec = cs.cand_spec[sec]
    n = len(nodes)
    ncols = len(col_values)
    out = [np.zeros((ncols + 1, n), bool) for _ in range(4)]
    if n == 0:
        return out
    tf = nodes["tflags"]
    empty = (tf & L.TF_RES_EMPTY) != 0
    ent = ((tf & L.TF_RES_ENT_ONLY) != 0) & ~empty
    for k in (0, 2):
        out[k][:, empty] = True
    real = np.array([v is MISSING or v is None or isinstance(v, str) for v in col_values] + [True], bool)
    # no entity attribute: an entity-only match never sets entityMatch
    out[1][ncols, ent] = True
    out[3][ncols, ent] = True
    idx = np.flatnonzero(ent)
    if len(idx) == 0 or ncols == 0:
        return out
    K = max((len(spec[i]) for i in idx), default=0)
    rows = np.full((len(idx), max(K, 1)), -1, np.int64)
    for j, i in enumerate(idx):
        sp = spec[i]
        rows[j, :len(sp)] = sp
    nrows = len(cs.rx_rows)
    row_of = {_key(v): r for r, v in enumerate(cs.rx_rows)}
    exact_row = np.array([row_of.get(_key(v), -1) if real[c] else -1 for c, v in enumerate(col_values)], np.int64)
    cells = np.zeros((ncols, max(nrows, 1)), np.uint8)
    if nrows:
        cells[:, :nrows] = rx[:ncols, :nrows]
    xt = np.zeros((ncols, len(idx)), bool)
    em = np.zeros((ncols, len(idx)), bool)
    thrown = np.zeros((ncols, len(idx)), bool)
    for k in range(rows.shape[1]):
        rk = rows[:, k]
        valid = rk >= 0
        xt |= valid[None, :] & (rk[None, :] == exact_row[:, None]) & (exact_row[:, None] >= 0)
        c = np.where(valid[None, :], cells[:, np.maximum(rk, 0)], 0)
        thrown |= (c & _THROW_LIKE) != 0
        em = np.where((c & L.RX_HIT) != 0, True, np.where((c & L.RX_RESET) != 0, False, em))
    ok = real[:ncols, None]
    out[0][:ncols, idx] = xt & ok
    out[1][:ncols, idx] = ~xt & ok
    out[2][:ncols, idx] = em & ~thrown & ok
    out[3][:ncols, idx] = ~em & ~thrown & ok
    return out


def _verdicts(cs, sec, pc, a, A_sec, role_ok_sec, role_filter, action_filter, res):
    """(known true, known false) of targetMatches in exact and RegExp mode for section `sec`
    of a chunk of classes: four bool [C, n] arrays (xt, xf, rt, rf)."""
    nodes = (cs.sets, cs.pols, cs.rules)[sec]
    nf, tf = nodes["nflags"], nodes["tflags"]
    tgt = ((nf & L.NF_HAS_TARGET) != 0)[None, :]
    sub_empty = ((tf & L.TF_SUBJ_EMPTY) != 0)[None, :]
    sub_role = (((tf & L.TF_SUBJ_ROLE) != 0) & ((tf & L.TF_SUBJ_EMPTY) == 0))[None, :]
    if role_filter:
        subj_t = sub_empty | (sub_role & role_ok_sec)
        subj_f = sub_role & ~role_ok_sec
    else:
        subj_t = np.broadcast_to(sub_empty, (len(pc), len(nodes)))
        subj_f = np.zeros((len(pc), len(nodes)), bool)
    need = (((nf & L.NF_HAS_TARGET) != 0) & (nodes["act_n"] > 0))[None, :]
    fixed = (a != 1)[:, None] if action_filter else np.zeros((len(pc), 1), bool)
    act = A_sec[a]
    act_t = ~need | (fixed & act)
    act_f = need & fixed & ~act
    xt_r, xf_r, rt_r, rf_r = (v[pc] for v in res)
    both_t = subj_t & act_t
    any_f = subj_f | act_f
    return (tgt & both_t & xt_r, tgt & (any_f | xf_r), tgt & both_t & rt_r, tgt & (any_f | rf_r))


def useful_static(cs):
    """(policies useful for every class that has them as candidates, sets holding a null
    policy) — see the module docstring."""
    P = cs.pols
    nf, tf = P["nflags"], P["tflags"]
    always = np.array([x is None for x in cs.cand_spec[1]], bool) if cs.n_pols else np.zeros(0, bool)
    pol = ((nf & L.NF_EFFECT_TRUTHY) != 0) & (P["map_size"] == 0)
    pol |= ((nf & L.NF_HAS_TARGET) != 0) & (((tf & L.TF_HAS_SUBJECTS) != 0) | always)
    null = (nf & L.NF_NULL) != 0
    cum = np.concatenate([[0], np.cumsum(null, dtype=np.int64)])
    b_s = cs.sets["child_begin"].astype(np.int64)
    e_s = cs.sets["child_end"].astype(np.int64)
    return pol, (cum[e_s] - cum[b_s]) > 0


def throw_policies(cs, col_values, rx):
    """bool [ncols + 1, P]: policies whose target reads a RegExp cell that throws (or needs
    the host) for a request entity value of that column (row ncols: no entity attr)."""
    nrows = len(cs.rx_rows)
    ncols = len(col_values)
    out = np.zeros((ncols + 1, cs.n_pols), bool)
    if not (nrows and ncols and cs.n_pols):
        return out
    real = np.array([v is MISSING or v is None or isinstance(v, str) for v in col_values], bool)
    rowmask = ((rx[:ncols, :nrows] & _THROW_LIKE) != 0) & real[:, None]
    if rowmask.any():
        _, A = _spec_matrix(cs.cand_spec[1], nrows)
        if A.nnz:
            out[:ncols] = (sparse.csr_matrix(rowmask.astype(np.int32)) @ A.T).toarray() > 0
    return out


def _useful(cs, s, p, r, thr_rows, pol_static, set_null):
    """Useful sets / policies of a chunk of class rows (bool [C, S], [C, P])."""
    C = s.shape[0]
    if cs.n_pols and cs.n_rules:
        cr = np.concatenate([np.zeros((C, 1), np.int64), np.cumsum(r, axis=1)], axis=1)
        has_rule = (cr[:, cs.pols["child_end"].astype(np.int64)] - cr[:, cs.pols["child_begin"].astype(np.int64)]) > 0
    else:
        has_rule = np.zeros((C, cs.n_pols), bool)
    up = p & (has_rule | pol_static[None, :] | thr_rows)
    if cs.n_pols:
        cu = np.concatenate([np.zeros((C, 1), np.int64), np.cumsum(up, axis=1)], axis=1)
        any_up = (cu[:, cs.sets["child_end"].astype(np.int64)] - cu[:, cs.sets["child_begin"].astype(np.int64)]) > 0
    else:
        any_up = np.zeros((C, cs.n_sets), bool)
    us = s & (any_up | set_null[None, :])
    return us, up


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


def action_keys(hdr, act):
    """Per request: index of its action key — 0: no action attribute, 1: several (unfiltered),
    2 + k: the k-th distinct single (id, value) pair of the batch — and the pairs [K, 2]."""
    nact = hdr["nact"].astype(np.int64)
    ak = np.where(nact == 0, 0, 1).astype(np.int64)
    one = nact == 1
    packed = (act["id"][0].astype(np.uint64) << np.uint64(32)) | act["value"][0].astype(np.uint64)
    uk, inv = np.unique(packed[one], return_inverse=True)
    if len(uk) > _MAX_ACTION_KEYS:  # a batch of exotic actions: keep the most frequent ones
        cnt = np.bincount(inv, minlength=len(uk))
        keep = np.argsort(-cnt, kind="stable")[:_MAX_ACTION_KEYS]
        remap = np.full(len(uk), -1, np.int64)
        remap[keep] = np.arange(len(keep))
        uk = uk[keep]
        inv = remap[inv]
        ak[np.flatnonzero(one)] = np.where(inv >= 0, inv + 2, 1)
    else:
        ak[np.flatnonzero(one)] = inv + 2
    pairs = np.stack([(uk >> np.uint64(32)).astype(np.int64), (uk & np.uint64(0xFFFFFFFF)).astype(np.int64)],
                     axis=1) if len(uk) else np.zeros((0, 2), np.int64)
    return ak, pairs


def _loose(a, b):
    return (a == b) | ((a <= L.ID_NULL) & (b <= L.ID_NULL))


def action_candidates(cs, pairs):
    """bool [2 + K, n] per section: nodes whose target can pass ``attributesMatch(rule.actions,
    request.actions)`` (accessController.ts:681-699: every target action attribute loosely equal
    to some request action attribute) for a request with no action (row 0), several actions
    (row 1: unfiltered) or the single action pair k (row 2 + k).  Nodes without a target or
    without action attributes are candidates in every row."""
    out = []
    pool = cs.pairs
    for nodes in (cs.sets, cs.pols, cs.rules):
        n = len(nodes)
        need = ((nodes["nflags"] & L.NF_HAS_TARGET) != 0) & (nodes["act_n"] > 0)
        rows = np.ones((2 + len(pairs), n), bool)
        rows[0] = ~need
        idx = np.flatnonzero(need)
        if len(idx) and len(pairs):
            cnt = nodes["act_n"][idx].astype(np.int64)
            owner = np.repeat(idx, cnt)
            start = np.repeat(nodes["act_off"][idx].astype(np.int64) - np.cumsum(cnt) + cnt, cnt)
            pidx = start + np.arange(cnt.sum())
            pid = pool["id"][pidx].astype(np.int64)
            pval = pool["value"][pidx].astype(np.int64)
            for k, (qi, qv) in enumerate(pairs):
                bad = ~(_loose(pid, qi) & _loose(pval, qv))
                fails = np.bincount(owner[bad], minlength=n)
                rows[2 + k] = (~need) | (fails == 0)
        out.append(rows)
    return tuple(out)


def _useful_relaxed(cs, s_free, p, p_free, r, thr_rows, pol_static, set_null):
    """Useful sets / policies of composed-level rows (module docstring): a candidate policy is
    useful when it may throw or is effect-only (its own role test applied), or when a candidate
    rule sits under it and its target passes with the role test ignored; a role-free candidate
    set is useful when one of its policies is (or it holds a null policy).  Each piece is an OR
    over the roles of the row, so the OR of two rows covers the joint key's useful sections."""
    C = s_free.shape[0]
    if cs.n_pols and cs.n_rules:
        cr = np.concatenate([np.zeros((C, 1), np.int64), np.cumsum(r, axis=1)], axis=1)
        has_rule = (cr[:, cs.pols["child_end"].astype(np.int64)] - cr[:, cs.pols["child_begin"].astype(np.int64)]) > 0
    else:
        has_rule = np.zeros((C, cs.n_pols), bool)
    up = (p & (pol_static[None, :] | thr_rows)) | (p_free & has_rule)
    if cs.n_pols:
        cu = np.concatenate([np.zeros((C, 1), np.int64), np.cumsum(up, axis=1)], axis=1)
        any_up = (cu[:, cs.sets["child_end"].astype(np.int64)] - cu[:, cs.sets["child_begin"].astype(np.int64)]) > 0
    else:
        any_up = np.zeros((C, cs.n_sets), bool)
    us = s_free & (any_up | set_null[None, :])
    return us, up


LEVELS = ("entity+roles+action", "composed", "entity+action", "entity")


def classes(cs, hdr, roles, pcol, ent, act=None, thr=None, res=None):
    """Class id per request (u32, PCOL_ALL = unfiltered), the second class per request (u32,
    1 + class id; 0 = none: composed rows), the class rows [C, W] u32 and the role factor.

    A class row is the AND of three node filters — entity column, role associations,
    action — and requests whose rows come out identical share a class (so the coherence
    sort groups them).  When the keys would need too much memory the key is coarsened:
    per-role rows composed by the kernel (two required roles), then (entity, action) with a
    role factor, then entity alone."""
    role_ids, req_rows = role_requirements(cs)
    nrr = len(role_ids)
    n = len(hdr)
    active = (pcol != L.PCOL_ALL) & ((hdr["flags"] & (L.RQ_HOST | L.RQ_NO_TARGET)) == 0)
    cls = np.full(n, L.PCOL_ALL, np.uint32)
    cls2 = np.zeros(n, np.uint32)
    W = row_layout(cs)[4]
    if not active.any():
        return cls, cls2, np.zeros((1, W), np.uint32), None, None
    if act is not None:
        ak, apairs = action_keys(hdr, act)
    else:
        ak, apairs = np.ones(n, np.int64), np.zeros((0, 2), np.int64)
    A = action_candidates(cs, apairs)
    rs = _role_sets(hdr, roles, role_ids)
    used = rs[:, ::-1]  # largest rows first; -1 padding last
    nused = (used >= 0).sum(axis=1) if n else np.zeros(0, np.int64)
    width = max(int(nused.max()) if n else 0, 1)
    E_s, E_p, E_r = ent
    A_s, A_p, A_r = A
    b_s = cs.sets["child_begin"].astype(np.int64)
    e_s = cs.sets["child_end"].astype(np.int64)
    nonempty = e_s > b_s
    pol_static, set_null = useful_static(cs)
    if thr is None:
        thr = np.zeros((int(pcol[pcol != L.PCOL_ALL].max(initial=0)) + 1, cs.n_pols), bool)
    act_idx = np.flatnonzero(active)
    for level in (LEVELS if FORCE_LEVEL is None else (FORCE_LEVEL,)):
        if level == "composed" and nrr == 0:  # no target requires a role: the joint keys are role-free
            level = "entity+roles+action"
        composed = level == "composed"
        role_filter = level in ("entity+roles+action", "composed")
        action_filter = level != "entity"
        cols = [pcol.astype(np.int64)[:, None]]
        if action_filter:
            cols.append(ak[:, None])
        if level == "entity+roles+action":
            cols.append(used[:, :width])
        elif composed:
            # primary key: the request's first required role (all of them past two); secondary:
            # its second role, for the requests with exactly two
            prim = np.full((n, width), -1, np.int64)
            prim[:, 0] = used[:, 0]
            big = nused > 2
            prim[big] = used[big, :width]
            cols.append(prim)
        key = np.concatenate(cols, axis=1)
        kact = key[active]
        two = np.flatnonzero(active & (nused == 2))
        if composed and len(two):
            sec = key[two].copy()
            sec[:, 2] = used[two, 1]
            kact = np.concatenate([kact, sec])
        ckey, inv = _unique_rows(kact)
        if level != "entity" and (len(ckey) * W * 4 > _KEY_ROW_BYTES or
                                  (level == LEVELS[0] and FORCE_LEVEL is None and 4 * len(ckey) > len(pcol))):
            # over the row budget; or joint keys covering fewer than 4 requests each (waves could
            # not share them, and the rows would outweigh the requests: a pipeline chunk of c3
            # shipped 1.2 KB of joint rows per request, the composed level's rows 0.1 KB)
            continue
        out = np.zeros((len(ckey), W), np.uint32)
        chunk = max(8, min(_CHUNK, _CHUNK_NODE_BITS // max(1, cs.n_sets + cs.n_pols + cs.n_rules)))
        for c0 in range(0, len(ckey), chunk):
            ck = ckey[c0:c0 + chunk]
            pc = ck[:, 0]
            a = ck[:, 1] if action_filter else np.ones(len(ck), np.int64)
            M = np.zeros((len(ck), nrr + 1), bool)
            M[:, nrr] = True  # "no role requirement" column
            if role_filter:
                for j in range(2, ck.shape[1]):
                    v = ck[:, j]
                    ok = v >= 0
                    M[np.flatnonzero(ok), v[ok]] = True
            else:
                M[:, :] = True

            def role_ok(rr):
                return M[:, np.where(rr >= 0, rr, nrr)]

            p = E_p[pc] & role_ok(req_rows[1]) & A_p[a]
            r = E_r[pc] & role_ok(req_rows[2]) & A_r[a]
            thr_rows = thr[np.minimum(pc, len(thr) - 1)]
            if composed:  # role-relaxed derived sections (module docstring)
                p_free = E_p[pc] & A_p[a]
                s = E_s[pc] & A_s[a]
            else:
                s = E_s[pc] & role_ok(req_rows[0]) & A_s[a]
            pc_ = p_free if composed else p
            if cs.n_pols:
                cum = np.concatenate([np.zeros((len(ck), 1), np.int64), np.cumsum(pc_, axis=1)], axis=1)
                pol_any = (cum[:, e_s] - cum[:, b_s]) > 0
            else:
                pol_any = np.zeros((len(ck), cs.n_sets), bool)
            s &= pol_any & nonempty[None, :]
            if composed:
                us, up = _useful_relaxed(cs, s, p, p_free, r, thr_rows, pol_static, set_null)
            else:
                us, up = _useful(cs, s, p, r, thr_rows, pol_static, set_null)
            verdicts = None
            if res is not None:
                pxt, pxf, prt, prf = _verdicts(cs, 1, pc, a, A_p, role_ok(req_rows[1]), role_filter, action_filter,
                                               res[0])
                rxt, rxf, rrt, _ = _verdicts(cs, 2, pc, a, A_r, role_ok(req_rows[2]), role_filter, action_filter,
                                             res[1])
                verdicts = (pxt, pxf, prt, prf, rxt | (rxf & rrt))
            out[c0:c0 + len(ck)] = _assemble(s, p, us, up, r, cs, verdicts)
        # keys whose rows (filter + verdict sections) come out identical share one class; a
        # row depends only on its key, so the native codec caches rows per key across batches
        # (acs_codec.cpp ClassCache) and the classes of a batch are its distinct rows
        urows, rinv = _unique_rows(out)
        if len(urows) <= MAX_CLASSES or level == "entity":
            break
    if len(urows) > MAX_CLASSES:  # entity level: at most one class per entity column (< 0xFFFE)
        raise ValueError("too many request classes")
    # heaviest classes first: the kernel's sort key orders waves by class id, so the longest
    # waves are dispatched first (longest-processing-time-first; no tail of heavy waves)
    # (the filter sections only: the verdicts are not work)
    cost = np.unpackbits(np.ascontiguousarray(urows[:, :verdict_offset(cs)]).view(np.uint8), axis=1).sum(axis=1)
    rank = np.empty(len(cost), np.int64)
    rank[np.argsort(-cost, kind="stable")] = np.arange(len(cost))
    urows = np.ascontiguousarray(urows[np.argsort(rank)])
    kcls = rank[rinv[inv]]
    cls[act_idx] = kcls[:len(act_idx)].astype(np.uint32)
    if composed and len(two):
        # the heavier class first (the coherence order groups by it), the same row once
        c_a = cls[two].astype(np.int64)
        c_b = kcls[len(act_idx):]
        cls[two] = np.minimum(c_a, c_b).astype(np.uint32)
        cls2[two] = np.where(c_a == c_b, 0, np.maximum(c_a, c_b) + 1).astype(np.uint32)
    if role_filter or nrr == 0:
        return cls, cls2, urows, None, None
    rkey, rbits = _role_factor(cs, rs, active, req_rows, nrr, b_s, e_s, nonempty, thr.any(axis=0), pol_static, set_null)
    return cls, cls2, urows, rkey, rbits


def coherence_order(cls, cls2, cand_rows, role_key=None, pad=None):
    """The encoder's coherence order (acs_req_batch.perm): request indices grouped so that a
    wave shares its class row(s) — [bucket | second class] with bucket = 1 + class (0: an
    unfiltered request), or role-major [role key | bucket] with a role factor — stable (index
    order within a key).  pad (default: 32 to 256 requests per class on average — at least 32
    when no request has a second class — and no role factor): each bucket's run starts on a
    64-lane wave boundary, the holes 0xFFFFFFFF (shorter classes would multiply the launch
    width; with second classes a bucket's run mixes them anyway, so long runs gain nothing from
    the holes: same-call A/B at 10M requests, c3r1 K1 1.95 -> 1.78 ms padded, c3 3.11 -> 3.19,
    r04_o / r04_p).
    acs_codec.cpp writes the same order.  Returns u32 [lanes]."""
    n = len(cls)
    c = cls.astype(np.int64)
    bucket = np.where(c < cand_rows, c + 1, 0)
    if role_key is not None:  # role-major: [role row | second role row | bucket]
        rk = role_key.astype(np.int64)
        key = (((rk & 0xFFFF) << 16 | rk >> 16) << 17) | bucket
        pad = False
    else:
        key = (bucket << 17) | cls2.astype(np.int64)
    perm = np.argsort(key, kind="stable").astype(np.uint32)
    if pad is None:
        pad = 32 * cand_rows <= n and (n < 256 * cand_rows or not cls2.any())
    if not pad or n == 0:
        return perm
    b = bucket[perm]
    starts = np.flatnonzero(np.concatenate([[True], b[1:] != b[:-1]]))
    sizes = np.diff(np.append(starts, n))
    padded = (sizes + 63) & ~63
    dst0 = np.concatenate([[0], np.cumsum(padded)[:-1]])
    out = np.full(int(padded.sum()), 0xFFFFFFFF, np.uint32)
    pos = np.repeat(dst0 - starts, sizes) + np.arange(n)
    out[pos] = perm
    return out


def _role_factor(cs, rs, active, req_rows, nrr, b_s, e_s, nonempty, thr_any, pol_static, set_null):
    """Role factor for class rows keyed without roles (large stores): the nodes a request's
    role associations let through checkSubjectMatches (accessController.ts:797-806) and the
    sets / policies useful through them, AND-ed by the kernel with the class row; both are
    supersets of the joint filter, so their AND is too.

    One row per required role (and one for "no required role"), built role-relaxed like the
    composed class rows (module docstring): a request with two required roles ORs its two rows,
    one with more gets a row of its whole role set.  role_key[i] = row | (1 + second row) << 16
    (the high half 0: one row; 0xFFFF low: no role filtering).  Returns (role_key, rows) or
    (None, None) when the rows would not fit."""
    W = row_layout(cs)[4]
    n = len(rs)
    nused = (rs >= 0).sum(axis=1)
    desc = rs[:, ::-1]  # largest role rows first, -1 padding last
    width = max(int(nused.max()) if n else 0, 1)
    # keys: one role row (or none) per request, the whole set past two roles; second keys
    prim = np.full((n, width), -1, np.int64)
    prim[:, 0] = desc[:, 0]
    big = nused > 2
    prim[big] = desc[big, :width]
    act_idx = np.flatnonzero(active)
    two = np.flatnonzero(active & (nused == 2))
    sec = np.full((len(two), width), -1, np.int64)
    if len(two):
        sec[:, 0] = desc[two, 1]
    keys, inv = _unique_rows(np.concatenate([prim[act_idx], sec]))
    if len(keys) == 0 or len(keys) * W * 4 > _ROLE_ROW_BYTES or len(keys) >= 0xFFFF:
        return None, None
    kid = inv.astype(np.int64)
    rkey = np.full(n, 0xFFFF, np.uint32)
    rkey[act_idx] = kid[:len(act_idx)].astype(np.uint32)
    if len(two):
        a_, b_ = rkey[two].astype(np.int64), kid[len(act_idx):]
        lo, hi = np.minimum(a_, b_), np.maximum(a_, b_)
        rkey[two] = (lo | np.where(lo == hi, 0, hi + 1) << 16).astype(np.uint32)
    out = np.zeros((len(keys), W), np.uint32)
    chunk = max(8, min(_CHUNK, _CHUNK_NODE_BITS // max(1, cs.n_sets + cs.n_pols + cs.n_rules)))
    p_free = np.ones((1, cs.n_pols), bool)
    if cs.n_pols:
        s_free = nonempty[None, :]  # every set with policies (its policies role-free)
    else:
        s_free = np.zeros((1, cs.n_sets), bool)
    for c0 in range(0, len(keys), chunk):
        ck = keys[c0:c0 + chunk]
        M = np.zeros((len(ck), nrr + 1), bool)
        M[:, nrr] = True  # "no role requirement" column
        for j in range(ck.shape[1]):
            v = ck[:, j]
            ok = v >= 0
            M[np.flatnonzero(ok), v[ok]] = True

        def role_ok(rr):
            return M[:, np.where(rr >= 0, rr, nrr)]

        p, r = role_ok(req_rows[1]), role_ok(req_rows[2])
        s_ = np.broadcast_to(s_free, (len(ck), cs.n_sets))
        # role-relaxed useful sections: a policy that may throw for some column of the batch, or
        # is useful wherever it is a candidate, stays; one with a rule the roles reach is useful
        # whatever its own role test (composable: OR over the request's role rows)
        us, up = _useful_relaxed(cs, s_, p, np.broadcast_to(p_free, p.shape), r, thr_any[None, :], pol_static,
                                 set_null)
        # the verdict sections are the class row's: the role side keeps them (all nodes)
        ap = np.ones((len(ck), cs.n_pols), bool)
        ar = np.ones((len(ck), cs.n_rules), bool)
        out[c0:c0 + len(ck)] = _assemble(s_, p, us, up, r, cs, (ap, ap, ap, ap, ar))
    return rkey, out


def _unique_rows(a):
    """(unique rows, inverse) of a 2-D integer array; narrow keys are packed into one int64."""
    if a.shape[0] == 0:
        return a[:0], np.zeros(0, np.int64)
    if a.shape[1] == 0:
        return a[:1], np.zeros(a.shape[0], np.int64)
    if a.dtype.kind == "i":
        lo = a.min(axis=0)
        span = a.max(axis=0) - lo + 1
        bits = [int(x).bit_length() for x in span]
        if sum(bits) <= 63:
            packed = np.zeros(a.shape[0], np.int64)
            for j, b in enumerate(bits):
                packed = (packed << b) | (a[:, j] - lo[j])
            _, first, inv = np.unique(packed, return_index=True, return_inverse=True)
            return a[first], inv.reshape(-1)
    v = np.ascontiguousarray(a).view(np.dtype((np.void, a.dtype.itemsize * a.shape[1]))).reshape(-1)
    _, first, inv = np.unique(v, return_index=True, return_inverse=True)
    return a[first], inv.reshape(-1)
