"""Request encoder: post-unmarshall requests -> packed batch (see csrc/acs_layout.h).

Every sub-expression of the reference that depends on the request alone is
evaluated here once per request, so the GPU only does request x rule work:

  * attribute-id classification against the URN config (=== and == forms),
  * lodash ``_.find`` context-resource lookups (instance.id, then id)
    of hierarchicalScope.ts:106-112,133 and verifyACL.ts:40-48 -> slot indices,
  * the verifyACL request loop (verifyACL.ts:37-88) -> 2-bit outcome + the
    ordered targetScopeEntInstances map,
  * role associations -> (role, entity, instance) grants and (role, entity)
    pairs (hierarchicalScope.ts:166-181,222-238, verifyACL.ts:104-125),
  * the subject's hierarchical_scopes forest -> per-root subtree membership
    masks of owner instances (hierarchicalScope.ts:207-243) and the
    role -> org mapping of verifyACL.ts:129-145 as key masks,
  * String.indexOf / '#'-suffix / namespace-regex evaluations
    (accessController.ts:509-574) -> bitmasks, interned ids, matrix columns.

Shapes the packed form does not cover (subject ``token`` — it needs identity /
Redis I/O —, null list entries, non-string scalars, size limits) set RQ_HOST.
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import layout as L
from .compiler import CompiledStore, Overlay
from .jsops import (MISSING, Unsupported, check_scalar, find_by, get, is_empty, nullish, or_list,
                    strict_eq, truthy)
from . import candidates
from .regex import cell


@dataclass
class RequestBatch:
    n: int
    hdr: np.ndarray      # [n] REQ_HDR_DT
    res: np.ndarray      # [QMAX, n] REQ_RES_DT
    subj: np.ndarray     # [SMAX, n] PAIR_DT
    act: np.ndarray      # [AMAX, n] PAIR_DT
    roles: np.ndarray    # [RMAX, n] u32
    arena: np.ndarray    # u32
    rx: np.ndarray       # [ncols, rx_rows] u8
    rx_rows: int
    overlay: Overlay
    host_reasons: dict = field(default_factory=dict)
    cand: np.ndarray | None = None   # [rx_cols + 1, W] candidate bitsets (candidates.py)
    cand_wp: int = 0
    cand_wr: int = 0
    cand_wsu: int = 0                # useful sets / policies sections (candidates.py); 0: absent
    cand_wpu: int = 0
    cand_wv: int = 0                 # target-verdict sections (candidates.verdict_offset); 0: absent
    role_key: np.ndarray | None = None   # [n] u32 role-factor row per request (large stores)
    role_bits: np.ndarray | None = None  # [role rows, W] u32
    lines: np.ndarray | None = None      # [n] REQ_LINE_DT packed first rows (pack_lines)
    hints: int = 0                       # ACS_HINT_* (acs_req_batch.hints)
    ext: np.ndarray | None = None        # u32 extension records of the rows past each line (pack_ext)
    cls2: np.ndarray | None = None       # [n] u32 1 + second class (composed class rows; 0: none)
    perm: np.ndarray | None = None       # u32 coherence order (candidates.coherence_order)

    def nbytes(self):
        return sum(a.nbytes for a in (self.hdr, self.res, self.subj, self.act, self.roles, self.arena, self.rx)) + \
            (self.cand.nbytes if self.cand is not None else 0) + \
            (self.role_key.nbytes + self.role_bits.nbytes if self.role_key is not None else 0) + \
            (self.lines.nbytes if self.lines is not None else 0) + \
            (self.ext.nbytes if self.ext is not None else 0) + \
            (self.perm.nbytes if self.perm is not None else 0)

    def compact_nbytes(self):
        """Bytes of the compact form (acs_layout.h): lines + extension records + arena + regex
        matrix + class / role-factor rows — what the host-buffer path uploads."""
        return self.lines.nbytes + self.ext.nbytes + self.arena.nbytes + self.rx.nbytes + \
            (self.cand.nbytes if self.cand is not None else 0) + \
            (self.role_key.nbytes + self.role_bits.nbytes if self.role_key is not None else 0) + \
            (self.perm.nbytes if self.perm is not None else 0)


def _attr_list(v, what):
    lst = or_list(v)
    for a in lst:
        if not isinstance(a, dict):
            raise Unsupported(f"non-object entry in {what}")
        check_scalar(a.get("id", MISSING))
        check_scalar(a.get("value", MISSING))
    return lst


def _dict_list(v, what):
    if nullish(v):
        return []
    if not isinstance(v, list):
        raise Unsupported(f"{what} is not an array")
    for x in v:
        if not isinstance(x, dict):
            raise Unsupported(f"non-object entry in {what}")
    return v


def _acl_none(flags, tse, grants, rolese, sid, id_user, I):
    """ACL_NONE (csrc/acs_layout.h): the request's ACLs make verifyACL (verifyACL.ts:89-251) false
    for every rule, whatever the rule's scoped roles, and it throws nowhere — no role
    associations; an action other than create / read / modify / delete; a create with an ACL
    entity that no role association scopes; a read / modify / delete where no ACL instance is the
    subject (for the user entity) or a grant's instance of the same entity."""
    if flags & L.RQ_SUBJ_MISSING or not (flags & L.RQ_RA_EMPTY or flags & L.RQ_HRS_ITERABLE):
        return False
    if flags & L.RQ_RA_EMPTY or not flags & (L.RQ_ACT_CREATE | L.RQ_ACT_RMD):
        return True
    if not tse:
        return False
    if flags & L.RQ_ACT_CREATE:
        scoped = {se for _, se in rolese}
        return any(se != id_user and se not in scoped for se in tse)
    for se, insts in tse.items():
        ids = {I(v) for v in insts}
        if se == id_user and sid in ids:
            return False
        if any(g[1] == se and g[2] in ids for g in grants):
            return False
    return True


class Encoder:
    """Encodes request batches against one compiled store (reusable across batches)."""

    def __init__(self, cs: CompiledStore):
        self.cs = cs
        self.u = cs.urns
        self._rx_cache = {}  # column value key -> row of cells

    def U(self, name):
        return self.u.get(name, MISSING)

    # ------------------------------------------------------------------ per request
    def _encode_one(self, req, ov: Overlay, cols: dict):
        U = self.U
        I = ov.intern
        flags = 0
        if not isinstance(req, dict):
            raise Unsupported("request is not an object")
        target = req.get("target", MISSING)
        subjects, resources, actions = [], [], []
        if not truthy(target):
            flags |= L.RQ_NO_TARGET
        else:
            if not isinstance(target, dict):
                raise Unsupported("target is not an object")
            subjects = _attr_list(target.get("subjects", MISSING), "target.subjects")
            resources = _attr_list(target.get("resources", MISSING), "target.resources")
            actions = _attr_list(target.get("actions", MISSING), "target.actions")
        if len(subjects) > L.SMAX or len(resources) > L.QMAX or len(actions) > L.AMAX:
            raise Unsupported("request list exceeds packed capacity")

        ctx = req.get("context", MISSING)
        ctx_empty = is_empty(ctx)
        if not nullish(ctx) and not isinstance(ctx, dict):
            raise Unsupported("context is not an object")
        if ctx_empty:
            flags |= L.RQ_CTX_EMPTY
        subj = get(ctx, "subject")
        if not nullish(subj) and not isinstance(subj, dict):
            raise Unsupported("context.subject is not an object")
        if truthy(get(subj, "token")):
            raise Unsupported("subject token: identity-srv / HR-scope I/O (accessController.ts:110-123)")
        if ctx_empty or nullish(subj):
            flags |= L.RQ_SUBJ_MISSING
        ras = get(subj, "role_associations")
        if truthy(ras):
            flags |= L.RQ_RA_TRUTHY
        if is_empty(ras):
            flags |= L.RQ_RA_EMPTY
        ras = _dict_list(ras, "role_associations") if truthy(ras) else []
        if len(ras) > L.RMAX:
            raise Unsupported("too many role associations")
        hrs = get(subj, "hierarchical_scopes")
        if isinstance(hrs, list):
            flags |= L.RQ_HRS_ITERABLE
        elif not nullish(hrs):
            raise Unsupported("hierarchical_scopes is not an array")

        # ---- resources: kinds, ids, regex columns, suffixes, indexOf masks
        ent, prop, op, rid = U("entity"), U("property"), U("operation"), U("resourceID")
        res_rows = []
        n_ent = 0
        for a in resources:
            i, v = a.get("id", MISSING), a.get("value", MISSING)
            kind = 0
            if strict_eq(i, ent):
                kind |= L.K_ENT
                n_ent += 1
            if (nullish(i) and nullish(ent)) or strict_eq(i, ent):
                kind |= L.K_ENT_LOOSE
            if strict_eq(i, op):
                kind |= L.K_OP
            if strict_eq(i, prop):
                kind |= L.K_PROP
                flags |= L.RQ_ANY_PROP
            if (nullish(i) and nullish(rid)) or strict_eq(i, rid):
                kind |= L.K_RID_LOOSE
            if isinstance(v, str) and "#" in v:
                kind |= L.K_HAS_HASH
            res_rows.append([v, kind])
        if n_ent > 1:
            flags |= L.RQ_MULTI_ENT
        # the only entity attribute's slot for the kernel's entity-only fast path
        ent_slots = [j for j, (_, k) in enumerate(res_rows) if k & L.K_ENT]
        ent_field = 0 if not ent_slots else (ent_slots[0] + 1 if len(ent_slots) == 1 and ent_slots[0] < 6 else 7)
        flags |= ent_field << L.RQ_ENT_SHIFT

        ctx_res = []
        if not ctx_empty:
            cr = get(ctx, "resources")
            if truthy(cr):
                if not isinstance(cr, list):
                    raise Unsupported("context.resources is not an array")
                ctx_res = cr
        slot_ids = {}
        slot_objs = []

        def slot_of(obj):
            if not truthy(obj):
                return L.NONE8
            k = id(obj)
            if k not in slot_ids:
                if len(slot_objs) >= L.MAX_SLOTS:
                    raise Unsupported("too many context resources")
                slot_ids[k] = len(slot_objs)
                slot_objs.append(obj)
            return slot_ids[k]

        def resolve_a(v):  # hierarchicalScope.ts:106-112 / verifyACL.ts:40-48
            o = find_by(ctx_res, "instance.id", v)
            if truthy(o):
                return get(o, "instance")
            return find_by(ctx_res, "id", v)

        packed_res = []
        keys_a, keys_b = {}, {}
        for j, (v, kind) in enumerate(res_rows):
            sa = sb = L.NONE8
            if kind & (L.K_RID_LOOSE | L.K_OP):
                sa = slot_of(resolve_a(v))
            if kind & L.K_OP:
                sb = slot_of(find_by(ctx_res, "id", v))
            vid = I(v)
            if kind & L.K_RID_LOOSE:
                keys_a.setdefault(vid, sa)
            if kind & L.K_OP:
                keys_b.setdefault(vid, sb)
            hs = L.ID_UNDEF
            contains = 0
            if kind & L.K_PROP:
                if isinstance(v, str):
                    hs = I(v[v.rfind("#") + 1:])
                    for i2, (v2, k2) in enumerate(res_rows):
                        if k2 & L.K_ENT:
                            name = v2[v2.rfind(":") + 1:] if isinstance(v2, str) else "undefined"
                            if name in v:
                                contains |= 1 << i2
            col = 0
            if kind & L.K_ENT_LOOSE:
                key = ("m",) if v is MISSING else (("n",) if v is None else ("s", v))
                col = cols.setdefault(key, len(cols))
                if col >= 0xFFFE:
                    raise Unsupported("too many distinct entity values in batch")
            packed_res.append((vid, hs, col, contains, kind, sa, sb, 0))
        for vid, sb in keys_b.items():  # HR map key shared by a resource id and an operation name
            if vid in keys_a and keys_a[vid] != sb:
                raise Unsupported("resource-id / operation key collision in HR owners map")

        # ---- role associations -> roles, (role, se) pairs, (role, se, inst) grants
        rse_u, rsi_u = U("roleScopingEntity"), U("roleScopingInstance")
        roles, rolese, grants = [], [], []
        for ra in ras:
            role = check_scalar(ra.get("role", MISSING))
            rid_ = I(role)
            roles.append(rid_)
            for rae in _dict_list(ra.get("attributes", MISSING) if truthy(ra.get("attributes", MISSING)) else [],
                                  "role association attributes"):
                if strict_eq(rae.get("id", MISSING), rse_u):
                    se = I(check_scalar(rae.get("value", MISSING)))
                    rolese.append((rid_, se))
                    insts = rae.get("attributes", MISSING)
                    for inst in _dict_list(insts if truthy(insts) else [], "role scoping instances"):
                        if strict_eq(inst.get("id", MISSING), rsi_u):
                            grants.append((rid_, se, I(check_scalar(inst.get("value", MISSING)))))
        if len(grants) > 255 or len(rolese) > 255:
            raise Unsupported("too many role scoping grants")

        # ---- hierarchical_scopes: per-root subtree ids (HR) and effective-role org lists (ACL)
        roots, root_sets, hr_keys, role_orgs = [], [], [], {}
        if isinstance(hrs, list):
            if len(hrs) > L.MAX_ROOTS:
                raise Unsupported("too many HR scope roots")

            def walk(nodes, inherited, acc):
                for h in _dict_list(nodes, "hierarchical scope nodes"):
                    r = h.get("role", MISSING)
                    key = inherited if nullish(r) else check_scalar(r)
                    hid = h.get("id", MISSING)
                    if truthy(hid):
                        if isinstance(hid, str):
                            acc.add(hid)
                        kk = I(key)
                        if kk not in role_orgs:
                            role_orgs[kk] = set()
                            hr_keys.append(kk)
                        if isinstance(hid, str):
                            role_orgs[kk].add(hid)
                    ch = h.get("children", MISSING)
                    n = len(ch) if isinstance(ch, (list, str)) else (ch.get("length", 0) if isinstance(ch, dict) else 0)
                    if truthy(n) and n > 0:
                        walk(ch, key, acc)

            for root in _dict_list(hrs, "hierarchical_scopes"):
                roots.append(I(check_scalar(root.get("role", MISSING))))
                acc = set()
                walk([root], MISSING, acc)
                root_sets.append(acc)
            if len(hr_keys) > L.MAX_HRKEYS:
                raise Unsupported("too many HR effective roles")

        def rootmask(v):
            if not isinstance(v, str):
                return 0
            m = 0
            for r, s in enumerate(root_sets):
                if v in s:
                    m |= 1 << r
            return m

        # ---- verifyACL request loop (verifyACL.ts:37-88)
        acl_state = L.ACL_CONTINUE
        tse = {}
        aclie, acli = U("aclIndicatoryEntity"), U("aclInstance")
        for a in resources:
            aid = a.get("id", MISSING)
            if not ((nullish(aid) and nullish(rid)) or strict_eq(aid, rid) or strict_eq(aid, op)):
                continue
            obj = resolve_a(a.get("value", MISSING))
            acls = MISSING
            if truthy(obj):
                meta = get(obj, "meta")
                al = get(meta, "acls")
                if isinstance(al, list) and len(al) > 0:
                    acls = al
                elif truthy(al) and not isinstance(al, list):
                    raise Unsupported("meta.acls is not an array")
            if is_empty(acls):
                acl_state = L.ACL_RET_TRUE
                break
            stop = False
            for acl in _dict_list(acls, "acls"):
                if strict_eq(acl.get("id", MISSING), aclie):
                    se = I(check_scalar(acl.get("value", MISSING)))
                    tse.setdefault(se, [])
                    attrs = acl.get("attributes", MISSING)
                    if not truthy(attrs) or (isinstance(attrs, list) and len(attrs) == 0):
                        acl_state, stop = L.ACL_RET_FALSE, True
                        break
                    for at in _dict_list(attrs, "acl attributes"):
                        if strict_eq(at.get("id", MISSING), acli):
                            tse[se].append(check_scalar(at.get("value", MISSING)))
                        else:
                            acl_state, stop = L.ACL_RET_FALSE, True
                            break
                    if stop:
                        break
                else:
                    acl_state, stop = L.ACL_RET_FALSE, True
                    break
            if stop:
                break
        flags |= acl_state << L.RQ_ACL_SHIFT

        a0 = actions[0] if actions else MISSING
        if isinstance(a0, dict) and strict_eq(a0.get("id", MISSING), U("actionID")):
            v0 = a0.get("value", MISSING)
            if strict_eq(v0, U("create")):
                flags |= L.RQ_ACT_CREATE
            elif strict_eq(v0, U("read")) or strict_eq(v0, U("modify")) or strict_eq(v0, U("delete")):
                flags |= L.RQ_ACT_RMD

        # ---- arena
        oe_u, oi_u = U("ownerEntity"), U("ownerInstance")
        words = [0, 0]
        for g in grants:
            words.extend(g)
        for p in rolese:
            words.extend(p)
        words.extend(roots)
        words.extend(hr_keys)
        slot_base = len(words)
        words.extend([0] * len(slot_objs))
        tse_base = len(words)
        tse_items = list(tse.items())
        words.extend([0] * (3 * len(tse_items)))
        for s, obj in enumerate(slot_objs):
            words[slot_base + s] = len(words)
            meta = get(obj, "meta") if isinstance(obj, dict) else MISSING
            owners = get(meta, "owners")
            empty = is_empty(meta) or is_empty(owners)
            olist = [] if empty else _dict_list(owners, "meta.owners")
            words.extend([1 if empty else 0, len(olist)])
            for o in olist:
                attrs = o.get("attributes", MISSING)
                alist = _dict_list(attrs, "owner attributes") if not nullish(attrs) else []
                is_oe = 1 if strict_eq(o.get("id", MISSING), oe_u) else 0
                words.extend([is_oe | (len(alist) << 8), I(check_scalar(o.get("value", MISSING)))])
                for at in alist:
                    av = check_scalar(at.get("value", MISSING))
                    k = L.K_OI if strict_eq(at.get("id", MISSING), oi_u) else 0
                    words.extend([I(av), k, rootmask(av)])
        for e, (se, insts) in enumerate(tse_items):
            if len(insts) > 32:
                raise Unsupported("too many ACL instances for one scoping entity")
            words[tse_base + 3 * e: tse_base + 3 * e + 3] = [se, len(insts), len(words)]
            for v in insts:
                m = 0
                if isinstance(v, str):
                    for k, key in enumerate(hr_keys):
                        if v in role_orgs[key]:
                            m |= 1 << k
                words.extend([I(v), m])
        if len(tse_items) > 255:
            raise Unsupported("too many ACL scoping entities")
        words[0] = len(grants) | (len(rolese) << 8) | (len(slot_objs) << 16) | (len(roots) << 24)
        words[1] = len(tse_items) | (len(hr_keys) << 8)

        sid = I(check_scalar(get(subj, "id")))
        if acl_state == L.ACL_CONTINUE and _acl_none(flags, tse, grants, rolese, sid, self.cs.id_user, I):
            flags = (flags & ~(3 << L.RQ_ACL_SHIFT)) | (L.ACL_NONE << L.RQ_ACL_SHIFT)
        hdr = (flags, len(resources), len(subjects), len(actions), len(roles), 0, sid)
        subj_pairs = [(I(a.get("id", MISSING)), I(a.get("value", MISSING))) for a in subjects]
        act_pairs = [(I(a.get("id", MISSING)), I(a.get("value", MISSING))) for a in actions]
        return hdr, packed_res, subj_pairs, act_pairs, roles, words

    # ------------------------------------------------------------------ batch
    def encode(self, requests) -> RequestBatch:
        n = len(requests)
        ov = Overlay(self.cs.dictionary)
        cols = {}
        hdr = np.zeros(n, L.REQ_HDR_DT)
        res = np.zeros((L.QMAX, n), L.REQ_RES_DT)
        subj = np.zeros((L.SMAX, n), L.PAIR_DT)
        act = np.zeros((L.AMAX, n), L.PAIR_DT)
        roles = np.zeros((L.RMAX, n), np.uint32)
        arena = []
        reasons = {}
        for i, req in enumerate(requests):
            try:
                h, pr, sp, ap, rl, words = self._encode_one(req, ov, cols)
            except Unsupported as e:
                reasons[i] = str(e)
                h, pr, sp, ap, rl, words = (L.RQ_HOST, 0, 0, 0, 0, 0, 0), [], [], [], [], [0, 0]
            h = list(h)
            h[5] = len(arena)
            hdr[i] = tuple(h)
            for j, t in enumerate(pr):
                res[j, i] = t
            for j, t in enumerate(sp):
                subj[j, i] = t
            for j, t in enumerate(ap):
                act[j, i] = t
            for j, t in enumerate(rl):
                roles[j, i] = t
            arena.extend(words)
        rows = self.cs.rx_rows
        rx = np.zeros((max(len(cols), 1), max(len(rows), 1)), np.uint8)
        col_values = [None] * len(cols)
        for key, c in cols.items():
            v = MISSING if key[0] == "m" else (None if key[0] == "n" else key[1])
            col_values[c] = v
            cached = self._rx_cache.get(key)
            if cached is None:
                cached = np.array([cell(rv, v) for rv in rows] or [0], np.uint8)
                self._rx_cache[key] = cached
            rx[c, :] = cached
        b = RequestBatch(n=n, hdr=hdr, res=res, subj=subj, act=act, roles=roles,
                         arena=np.array(arena, np.uint32), rx=rx, rx_rows=max(len(rows), 1),
                         overlay=ov, host_reasons=reasons)
        attach_candidates(self.cs, b, col_values)
        return b


def mark_rx_safe(b: RequestBatch):
    """RES_RX_SAFE in ReqRes.pad of every entity attribute whose regex column holds no cell
    that throws or needs the host: K1 may then end a combining loop once its result is final
    (nothing left in it can throw).  acs_codec.cpp does the same."""
    bad = (b.rx & np.uint8(L.RX_THROW_TYPE | L.RX_THROW_SYNTAX | L.RX_HOST)).any(axis=1)
    j = np.arange(L.QMAX)[:, None]
    col = b.res["col"].astype(np.int64)
    ok = ((b.res["kind"] & L.K_ENT_LOOSE) != 0) & (j < b.hdr["nres"][None, :]) & (col < len(bad))
    ok &= ~bad[np.minimum(col, len(bad) - 1)]
    b.res["pad"] |= np.where(ok, np.uint8(L.RES_RX_SAFE), np.uint8(0))


def pack_lines(b: RequestBatch) -> np.ndarray:
    """[n] REQ_LINE_DT: every request's header, first 4 resource attributes, 2 subjects,
    action, 2 roles and arena counts in one 128-B line (acs_layout.h ReqLine), equal to the
    SoA rows, so K1 reads a request with one gather instead of ~8.  acs_codec.cpp does the same."""
    n = b.n
    h = b.hdr
    ln = np.zeros(n, L.REQ_LINE_DT)
    ln["h"] = h
    for j in range(4):
        ln["res"][:, j] = np.where(j < h["nres"], b.res[j], np.zeros(1, L.REQ_RES_DT))
    zp = np.zeros(1, L.PAIR_DT)
    ln["s0"] = np.where(h["nsubj"] > 0, b.subj[0], zp)
    ln["s1"] = np.where(h["nsubj"] > 1, b.subj[1], zp)
    ln["a0"] = np.where(h["nact"] > 0, b.act[0], zp)
    ln["r0"] = np.where(h["nroles"] > 0, b.roles[0], 0)
    ln["r1"] = np.where(h["nroles"] > 1, b.roles[1], 0)
    if b.cls2 is not None:
        ln["cls2"] = b.cls2
    live = (h["flags"] & np.uint32(L.RQ_HOST | L.RQ_NO_TARGET)) == 0
    off = h["arena_off"].astype(np.int64)
    if b.arena.size:
        ln["ar0"] = np.where(live, b.arena[np.minimum(off, b.arena.size - 1)], 0)
        ln["ar1"] = np.where(live, b.arena[np.minimum(off + 1, b.arena.size - 1)], 0)
    words = L.ext_geom(h["nres"], h["nsubj"], h["nact"], h["nroles"])[4]
    start = np.cumsum(words) - words
    ln["ext"] = np.where(words > 0, start // 4 + 1, 0).astype(np.uint32)
    return ln


def pack_ext(b: RequestBatch) -> np.ndarray:
    """u32 extension records (acs_layout.h ext_geom): per request, in request order, the rows
    its line cannot hold — resource attributes 4.., subjects 2.., actions 1.., roles 2.. —
    padded to 4 words; ReqLine.ext = 1 + the record's offset in 16-B units (pack_lines).
    With the lines, this is the compact batch (no SoA rows) the kernels read.  acs_codec.cpp
    writes the same records."""
    h = b.hdr
    _, g_subj, g_act, g_roles, words = L.ext_geom(h["nres"], h["nsubj"], h["nact"], h["nroles"])
    start = np.cumsum(words) - words
    ext = np.zeros(int(words.sum()), np.uint32)
    nres, nsubj, nact, nroles = (h[f].astype(np.int64) for f in ("nres", "nsubj", "nact", "nroles"))
    rw = b.res.view(np.uint32).reshape(L.QMAX, b.n, 4)
    for j in range(L.LINE_RES, L.QMAX):
        i = np.flatnonzero(nres > j)
        for k in range(4):
            ext[start[i] + 4 * (j - L.LINE_RES) + k] = rw[j, i, k]
    for rows, cnt, base, first in ((b.subj, nsubj, g_subj, L.LINE_SUBJ), (b.act, nact, g_act, L.LINE_ACT)):
        for j in range(first, rows.shape[0]):
            i = np.flatnonzero(cnt > j)
            ext[start[i] + base[i] + 2 * (j - first)] = rows["id"][j, i]
            ext[start[i] + base[i] + 2 * (j - first) + 1] = rows["value"][j, i]
    for j in range(L.LINE_ROLES, b.roles.shape[0]):
        i = np.flatnonzero(nroles > j)
        ext[start[i] + g_roles[i] + (j - L.LINE_ROLES)] = b.roles[j, i]
    return ext


def attach_candidates(cs, b: RequestBatch, col_values, role_filter: bool = True):
    """Candidate rows for the batch's request classes + each request's class id in its flags."""
    mark_rx_safe(b)
    ncols = b.rx.shape[0]
    assert len(col_values) <= ncols
    # pad: columns without a value (an all-empty batch) get no candidates beyond the "always" nodes
    vals = list(col_values) + [object()] * (ncols - len(col_values))
    ent = candidates.entity_candidates(cs, vals, b.rx)
    thr = candidates.throw_policies(cs, vals, b.rx)
    res = (candidates.resource_verdicts(cs, vals, b.rx, 1), candidates.resource_verdicts(cs, vals, b.rx, 2))
    b.cand_wp, b.cand_wsu, b.cand_wpu, b.cand_wr, _ = candidates.row_layout(cs)
    b.cand_wv = candidates.verdict_offset(cs)
    pcol = candidates.primary_columns(b.res["kind"], b.res["col"], b.hdr["nres"], ncols)
    roles = b.roles if role_filter else np.zeros((0, b.n), np.uint32)
    cls, b.cls2, b.cand, b.role_key, b.role_bits = candidates.classes(cs, b.hdr, roles, pcol, ent, b.act, thr, res)
    b.hdr["flags"] = (b.hdr["flags"] & np.uint32(0xFFFF)) | (cls.astype(np.uint32) << np.uint32(L.RQ_PCOL_SHIFT))
    b.lines = pack_lines(b)
    b.ext = pack_ext(b)
    # the coherence order the kernels run in (the encoder knows every class: no device sort)
    b.perm = candidates.coherence_order(cls, b.cls2, b.cand.shape[0], b.role_key)
    acl_none = ((b.hdr["flags"] >> np.uint32(L.RQ_ACL_SHIFT)) & np.uint32(3)) == L.ACL_NONE
    b.hints = L.HINT_ACL_NONE if acl_none.any() else 0
