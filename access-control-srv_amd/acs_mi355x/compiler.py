"""Policy-store compiler: ``policySets`` Map snapshot -> HBM tables.

Everything that depends on a rule/policy/set alone is evaluated here once
(targets' role / scoping-entity / hierarchicalRoleScoping scans, skipACL,
scopedRoles, property presence, effect / evaluation_cacheable / combining
algorithm codes, '#'-suffixes, regex rows).  What is left for the GPU is the
request x target work.  Reference anchors:

  targets' subject scan      accessController.ts:797-806, hierarchicalScope.ts:25-42,
                             verifyACL.ts:13-25
  policy effect / CA         accessController.ts:138-148, 832-838
  rule ec / condition flags  accessController.ts:202-211, 228
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

from . import layout as L
from .jsops import MISSING, Unsupported, check_scalar, get, nullish, strict_eq, truthy, OBJECT_PROTO_KEYS

CA_METHODS = {"denyOverrides": L.CA_DENY_OVERRIDES, "permitOverrides": L.CA_PERMIT_OVERRIDES,
              "firstApplicable": L.CA_FIRST_APPLICABLE}
_EFFECTS = {"PERMIT": L.EFF_PERMIT, "DENY": L.EFF_DENY, "NOT_APPLICABLE": L.EFF_NOT_APPLICABLE,
            "INDETERMINATE": L.EFF_INDETERMINATE, "UNRECOGNIZED": L.EFF_UNRECOGNIZED}


class Dictionary:
    """String interner: equal ids <=> JS ===.  0 undefined, 1 null, 2 ''."""

    def __init__(self):
        self.ids = {"": L.ID_EMPTY}
        self.strings = [MISSING, None, ""]

    def __len__(self):
        return len(self.strings)

    def intern(self, v) -> int:
        if v is MISSING:
            return L.ID_UNDEF
        if v is None:
            return L.ID_NULL
        if not isinstance(v, str):
            raise Unsupported(f"non-string value {v!r}")
        i = self.ids.get(v)
        if i is None:
            i = len(self.strings)
            self.ids[v] = i
            self.strings.append(v)
        return i

    def lookup(self, v):
        if v is MISSING:
            return L.ID_UNDEF
        if v is None:
            return L.ID_NULL
        return self.ids.get(v)

    def string(self, i):
        return self.strings[i]


class Overlay:
    """Batch-local extension of a frozen Dictionary (request-only strings)."""

    def __init__(self, base: Dictionary):
        self.base = base
        self.ids = {}
        self.strings = []

    def intern(self, v) -> int:
        i = self.base.lookup(v) if (v is MISSING or v is None or isinstance(v, str)) else None
        if i is not None:
            return i
        if not isinstance(v, str):
            raise Unsupported(f"non-string value {v!r}")
        i = self.ids.get(v)
        if i is None:
            i = len(self.base) + len(self.strings)
            self.ids[v] = i
            self.strings.append(v)
        return i

    def string(self, i):
        n = len(self.base)
        return self.base.string(i) if i < n else self.strings[i - n]


def effect_code(e) -> int:
    if e is MISSING:
        return L.EFF_UNDEF
    if e is None:
        return L.EFF_NULL
    if isinstance(e, str):
        if e in OBJECT_PROTO_KEYS:
            raise Unsupported(f"effect {e!r} resolves to an Object.prototype member")
        if e in _EFFECTS:
            return _EFFECTS[e]
    return L.EFF_OTHER_TRUTHY if truthy(e) else L.EFF_OTHER_FALSY


@dataclass
class CompiledStore:
    urns: dict
    dictionary: Dictionary
    sets: np.ndarray              # NODE_DT
    pols: np.ndarray              # NODE_DT
    rules: np.ndarray             # NODE_DT
    rres: np.ndarray
    pairs: np.ndarray
    u32pool: np.ndarray
    rx_rows: list                 # row index -> rule entity value (str / None / MISSING)
    ec_values: list               # ec code -> raw JS value
    id_user: int
    # host-side objects for whatIsAllowed / response reconstruction, in table order
    set_objs: list = field(default_factory=list)
    pol_objs: list = field(default_factory=list)
    rule_objs: list = field(default_factory=list)
    stats: dict = field(default_factory=dict)
    cand_spec: tuple = ((), (), ())  # per set/policy/rule: None (always), rows list

    @property
    def n_sets(self):
        return len(self.sets)

    @property
    def n_pols(self):
        return len(self.pols)

    @property
    def n_rules(self):
        return len(self.rules)

    def table_bytes(self):
        return sum(a.nbytes for a in (self.sets, self.pols, self.rules, self.rres, self.pairs, self.u32pool))


class _Builder:
    def __init__(self, urns, cas):
        self.urns = dict(urns)
        self.ca_map = {}
        for ca in cas:
            m = ca.get("method")
            if m not in CA_METHODS:
                raise Unsupported(f"combining algorithm method {m!r}")
            self.ca_map[ca.get("urn", MISSING)] = CA_METHODS[m]
        self.d = Dictionary()
        self.rres, self.pairs, self.u32pool = [], [], []
        self.rx_index = {}
        self.rx_rows = []
        self.ec_values = [MISSING, None, False, True]
        self.ec_truthy = [False, False, False, True]
        # URN ids (an absent URN is JS undefined and compares equal to undefined ids)
        self.U = {k: self.d.intern(v) for k, v in self.urns.items()}

    def urn(self, name):
        return self.urns.get(name, MISSING)

    def ca_code(self, urn):
        key = urn if (urn is MISSING or urn is None or isinstance(urn, str)) else repr(urn)
        return self.ca_map.get(key, L.CA_INVALID)

    def ec_code(self, v):
        for i, x in enumerate(self.ec_values):
            if (x is v) or (type(x) is type(v) and x == v and not isinstance(v, (dict, list))):
                return i
        if len(self.ec_values) >= 255:
            raise Unsupported("too many distinct evaluation_cacheable values")
        self.ec_values.append(v)
        self.ec_truthy.append(truthy(v))
        return len(self.ec_values) - 1

    def rx_row(self, value):
        key = ("m",) if value is MISSING else (("n",) if value is None else ("s", value))
        r = self.rx_index.get(key)
        if r is None:
            r = len(self.rx_rows)
            if r >= 0xFFFF:
                raise Unsupported("too many distinct rule entity values")
            self.rx_index[key] = r
            self.rx_rows.append(value)
        return r

    @staticmethod
    def _attrs(lst, what):
        if not isinstance(lst, list):
            raise Unsupported(f"target {what} is not an array")
        for a in lst:
            if not isinstance(a, dict):
                raise Unsupported(f"non-object entry in target {what}")
            check_scalar(a.get("id", MISSING))
            check_scalar(a.get("value", MISSING))
        return lst

    def add_pairs(self, lst):
        off = len(self.pairs)
        for a in lst:
            self.pairs.append((self.d.intern(a.get("id", MISSING)), self.d.intern(a.get("value", MISSING))))
        return off

    def target(self, t) -> dict:
        """Inline target fields of a node record ({} when the node has no target)."""
        if t is None or t is MISSING or not truthy(t):
            return {}
        if not isinstance(t, dict):
            raise Unsupported("target is not an object")
        subs = self._attrs(t.get("subjects", MISSING) if truthy(t.get("subjects", MISSING)) else [], "subjects")
        acts = self._attrs(t.get("actions", MISSING) if truthy(t.get("actions", MISSING)) else [], "actions")
        res = self._attrs(t.get("resources", MISSING) if truthy(t.get("resources", MISSING)) else [], "resources")
        if "subjects" in t and not isinstance(t["subjects"], list):
            raise Unsupported("subjects")
        U = self.urn
        rec = {}
        flags = 0
        # checkSubjectMatches: ruleRole = last role value (accessController.ts:802-806)
        role = MISSING
        for a in subs:
            if strict_eq(a.get("id", MISSING), U("role")):
                role = a.get("value", MISSING)
        if len(subs) == 0:
            flags |= L.TF_SUBJ_EMPTY
        elif truthy(role):
            flags |= L.TF_SUBJ_ROLE
        if len(subs) > 0:
            flags |= L.TF_HAS_SUBJECTS
        rec["role"] = self.d.intern(role)
        rec["subj_off"] = self.add_pairs(subs)
        rec["subj_n"] = len(subs)
        rec["act_off"] = self.add_pairs(acts)
        rec["act_n"] = len(acts)
        # checkHierarchicalScope subject scan (if / else-if chain, hierarchicalScope.ts:29-37)
        hr_check, se = "true", MISSING
        for a in subs:
            i = a.get("id", MISSING)
            if strict_eq(i, U("role")):
                pass
            elif strict_eq(i, U("hierarchicalRoleScoping")):
                hr_check = a.get("value", MISSING)
            elif strict_eq(i, U("roleScopingEntity")):
                se = a.get("value", MISSING)
        if len(subs) == 0 or not truthy(se):
            flags |= L.TF_HR_TRIVIAL
        if strict_eq(hr_check, "true"):
            flags |= L.TF_HR_CHECK
        rec["se"] = self.d.intern(se)
        # verifyACLList subject scan (verifyACL.ts:17-25)
        scoped = []
        for a in subs:
            i = a.get("id", MISSING)
            if strict_eq(i, U("role")):
                scoped.append(self.d.intern(a.get("value", MISSING)))
            elif strict_eq(i, U("skipACL")):
                flags |= L.TF_ACL_SKIP
                break
        rec["acl_roles_off"] = len(self.u32pool)
        rec["acl_roles_n"] = len(scoped)
        self.u32pool.extend(scoped)
        # resources
        if len(res) == 0:
            flags |= L.TF_RES_EMPTY
        rec["res_off"] = len(self.rres)
        rec["res_n"] = len(res)
        last_prop = MISSING
        for a in res:
            i, v = a.get("id", MISSING), a.get("value", MISSING)
            kind = 0
            if strict_eq(i, U("entity")):
                kind |= L.K_ENT
            if (nullish(i) and nullish(U("entity"))) or strict_eq(i, U("entity")):
                kind |= L.K_ENT_LOOSE
            if strict_eq(i, U("operation")):
                kind |= L.K_OP
            if strict_eq(i, U("property")):
                kind |= L.K_PROP
                flags |= L.TF_RULE_PROPS
                last_prop = v
            hs = L.ID_UNDEF
            if kind & L.K_PROP and isinstance(v, str):
                hs = self.d.intern(v[v.rfind("#") + 1:])
            row = self.rx_row(v) if kind & L.K_ENT_LOOSE else 0
            self.rres.append((self.d.intern(v), hs, row, kind, 0, 0))
        rec["last_prop_value"] = self.d.intern(last_prop)
        # candidate spec: a target can only match requests whose entity hits one of its
        # entity rows (resourceAttributesMatch needs entityMatch or operationMatch)
        has_op = any(strict_eq(a.get("id", MISSING), U("operation")) for a in res)
        if len(res) == 0 or has_op:
            rec["_cand"] = None  # always a candidate
        else:
            rec["_cand"] = [self.rx_row(a.get("value", MISSING)) for a in res
                            if strict_eq(a.get("id", MISSING), U("entity"))]
        if len(res) > 0 and not any(strict_eq(a.get("id", MISSING), U("property")) or
                                    strict_eq(a.get("id", MISSING), U("operation")) for a in res):
            flags |= L.TF_RES_ENT_ONLY
        if isinstance(last_prop, str):
            flags |= L.TF_LASTPROP_STR
            if "#" in last_prop:
                flags |= L.TF_LASTPROP_HASH
        rec["tflags"] = flags
        return rec


def _node(fields: dict, spec: list):
    """Pack one node record; append its candidate spec (None = always, list of rows)."""
    spec.append(fields.pop("_cand", None) if fields.get("nflags", 0) & L.NF_HAS_TARGET else
                ([] if fields.get("nflags", 0) & L.NF_NULL and spec is not None and fields.get("_rule") else None))
    fields.pop("_rule", None)
    return tuple(fields.get(n, 0) if n != "pad" else (0, 0, 0) for n in L.NODE_DT.names)


@dataclass
class _Fragment:
    """One policy set compiled on its own: node records with fragment-local child ranges and
    pool offsets (assemble() shifts them), its candidate specs and host-side objects."""
    obj: dict
    sets: np.ndarray
    pols: np.ndarray
    rules: np.ndarray
    rres: np.ndarray
    pairs: np.ndarray
    u32pool: np.ndarray
    spec: tuple
    pol_objs: list
    rule_objs: list


def _arr(x, dt):
    return np.array(x, dtype=dt) if x else np.zeros(0, dt)


def _compile_set(b: _Builder, ps) -> _Fragment:
    """Compile one policy set (accessController.ts:125-295 per-set state: policyEffect prefix,
    evaluation_cacheable prefix, child ranges) with the shared dictionary / regex rows of
    ``b`` and fresh, fragment-local pools."""
    if not isinstance(ps, dict):
        raise Unsupported("null policy set")
    saved = (b.rres, b.pairs, b.u32pool)
    b.rres, b.pairs, b.u32pool = [], [], []
    try:
        pols, rules, pol_objs, rule_objs = [], [], [], []
        spec_s, spec_p, spec_r = [], [], []
        sn = b.target(ps.get("target", MISSING))
        sn["nflags"] = L.NF_HAS_TARGET if sn else 0
        sn["child_begin"] = 0
        combin = ps.get("combinables")
        if not isinstance(combin, dict):
            raise Unsupported("policy set without combinables")
        pe_at = L.EFF_UNDEF
        set_free = L.NF_COND_FREE  # no condition rule and no invalid combining algorithm below
        for pol in combin.values():
            if pol is None or pol is MISSING:
                pols.append(_node({"nflags": L.NF_NULL, "child_begin": len(rules), "child_end": len(rules),
                                   "fe": len(rules), "pe_at": pe_at}, spec_p))
                pol_objs.append(None)
                continue
            pn = b.target(pol.get("target", MISSING))
            nf = L.NF_HAS_TARGET if pn else 0
            if truthy(pol.get("effect", MISSING)):
                nf |= L.NF_EFFECT_TRUTHY
                pe_at = effect_code(pol["effect"])   # accessController.ts:138-140
            pn.update(nflags=nf, child_begin=len(rules), effect=effect_code(pol.get("effect", MISSING)),
                      ec=b.ec_code(pol.get("evaluation_cacheable", MISSING)),
                      ca=b.ca_code(pol.get("combining_algorithm", MISSING)), pe_at=pe_at)
            rcomb = pol.get("combinables")
            if not isinstance(rcomb, dict):
                raise Unsupported("policy without combinables")
            fe = None
            pol_free = L.NF_COND_FREE
            for rule in rcomb.values():
                if rule is None or rule is MISSING:
                    rules.append(_node({"nflags": L.NF_NULL, "_rule": True}, spec_r))
                    rule_objs.append(None)
                    continue
                rn = b.target(rule.get("target", MISSING))
                rf = L.NF_HAS_TARGET if rn else 0
                cond = rule.get("condition", MISSING)
                clen = len(cond) if isinstance(cond, (str, list)) else get(cond, "length")
                if truthy(clen):
                    rf |= L.NF_HAS_CONDITION
                    pol_free = 0
                ec = b.ec_code(rule.get("evaluation_cacheable", MISSING))
                if b.ec_truthy[ec]:
                    rf |= L.NF_EC_TRUTHY
                elif fe is None:
                    fe = len(rules)  # first non-null rule with falsy evaluation_cacheable
                rn.update(nflags=rf, effect=effect_code(rule.get("effect", MISSING)), ec=ec)
                rules.append(_node(rn, spec_r))
                rule_objs.append(rule)
            pn.update(child_end=len(rules), map_size=len(rcomb), fe=len(rules) if fe is None else fe,
                      nflags=pn["nflags"] | pol_free)
            if not pol_free or pn["ca"] == L.CA_INVALID:
                set_free = 0
            pols.append(_node(pn, spec_p))
            pol_objs.append(pol)
        sn.update(child_end=len(pols), ca=b.ca_code(ps.get("combining_algorithm", MISSING)),
                  nflags=sn["nflags"] | set_free,
                  pe_at=pe_at)  # set: policyEffect after a full loop-2a scan
        sets = [_node(sn, spec_s)]
        return _Fragment(ps, _arr(sets, L.NODE_DT), _arr(pols, L.NODE_DT), _arr(rules, L.NODE_DT),
                         _arr(b.rres, L.RULE_RES_DT), _arr(b.pairs, L.PAIR_DT),
                         np.array(b.u32pool, dtype=np.uint32) if b.u32pool else np.zeros(0, np.uint32),
                         (spec_s, spec_p, spec_r), pol_objs, rule_objs)
    finally:
        b.rres, b.pairs, b.u32pool = saved


def mark_clean_below(sets, pols):
    """NF_CLEAN_BELOW on every set all of whose predecessors are clean, NF_CLEAN on every clean
    set: NF_COND_FREE (no condition rule, no invalid policy combining algorithm), a valid set
    combining algorithm and no null policy (loop 2a's TypeError).  Depends on the Map order, so it is set on the
    assembled tables (acs_compiler.cpp does the same after its last set)."""
    if not len(sets):
        return
    owner = np.repeat(np.arange(len(sets)), (sets["child_end"] - sets["child_begin"]).astype(np.int64))
    has_null = np.zeros(len(sets), bool)
    has_null[owner[(pols["nflags"] & L.NF_NULL) != 0]] = True
    clean = ((sets["nflags"] & L.NF_COND_FREE) != 0) & (sets["ca"] != L.CA_INVALID) & ~has_null
    below = np.concatenate([[True], np.logical_and.accumulate(clean)[:-1]])
    sets["nflags"] |= np.where(below, np.uint8(L.NF_CLEAN_BELOW), np.uint8(0))
    sets["nflags"] |= np.where(clean, np.uint8(L.NF_CLEAN), np.uint8(0))


def _assemble(b: _Builder, frags: list) -> CompiledStore:
    """Concatenate fragments in Map order, shifting child ranges and pool offsets."""
    ns = [len(f.pols) for f in frags]
    nr = [len(f.rules) for f in frags]
    sizes = {k: [len(getattr(f, k)) for f in frags] for k in ("rres", "pairs", "u32pool")}

    def starts(v):
        return np.concatenate([[0], np.cumsum(v, dtype=np.int64)[:-1]]).astype(np.uint32) if v else np.zeros(0, np.uint32)

    pol0, rule0 = starts(ns), starts(nr)
    res0, pair0, u320 = starts(sizes["rres"]), starts(sizes["pairs"]), starts(sizes["u32pool"])

    pools = [("subj_off", pair0), ("act_off", pair0), ("res_off", res0), ("acl_roles_off", u320)]

    def cat(key, shifts):
        if not frags:
            return np.zeros(0, L.NODE_DT)
        a = np.concatenate([getattr(f, key) for f in frags])
        owner = np.repeat(np.arange(len(frags)), [len(getattr(f, key)) for f in frags])
        for field_, base in shifts:
            a[field_] += base[owner]
        tgt = (a["nflags"] & L.NF_HAS_TARGET) != 0  # target-less nodes keep pool offsets 0
        for field_, base in pools:
            a[field_][tgt] += base[owner[tgt]]
        return a

    sets = cat("sets", [("child_begin", pol0), ("child_end", pol0)])
    pols = cat("pols", [("child_begin", rule0), ("child_end", rule0), ("fe", rule0)])
    rules = cat("rules", [])
    mark_clean_below(sets, pols)

    def pool(key, dt):
        return np.concatenate([getattr(f, key) for f in frags]) if frags else np.zeros(0, dt)

    cs = CompiledStore(
        urns=b.urns, dictionary=b.d, sets=sets, pols=pols, rules=rules, rres=pool("rres", L.RULE_RES_DT),
        pairs=pool("pairs", L.PAIR_DT), u32pool=pool("u32pool", np.uint32),
        rx_rows=list(b.rx_rows), ec_values=list(b.ec_values), id_user=b.d.intern(b.urn("user")),
        set_objs=[f.obj for f in frags], pol_objs=[o for f in frags for o in f.pol_objs],
        rule_objs=[o for f in frags for o in f.rule_objs],
        cand_spec=tuple([x for f in frags for x in f.spec[i]] for i in range(3)))
    cs.stats = {"sets": cs.n_sets, "policies": cs.n_pols, "rules": cs.n_rules, "dictionary": len(b.d),
                "rx_rows": len(b.rx_rows), "table_bytes": cs.table_bytes()}
    return cs


class IncrementalCompiler:
    """Recompiles only the policy sets that changed (store mutations
    through updatePolicySet / updatePolicy / updateRule / remove* / Map edits,
    accessController.ts:897-937, resourceManager.ts:156-1047).  Each set is compiled into a
    fragment against a shared, append-only dictionary and regex-row index, so unchanged
    fragments stay valid; compile() reuses a fragment when its key is not marked dirty and
    the Map still holds the same set object, then re-concatenates (offset shifts only).
    Interned ids of an incremental image can differ from a fresh compile's, and strings of
    removed rules stay in the dictionary; the tables are otherwise equal field for field
    (tests/test_incremental.py)."""

    def __init__(self, urns: dict, combining_algorithms: list):
        self.b = _Builder(urns, combining_algorithms)
        self.frags = {}
        self.stats = {"compiles": 0, "sets_compiled": 0, "sets_reused": 0}
        self._base = None  # append-only table sizes right after the first (full) compile

    def _sizes(self):
        return len(self.b.d), len(self.b.rx_rows), len(self.b.ec_values)

    def stale(self) -> bool:
        """The shared dictionary, regex rows and evaluation_cacheable values only grow: strings
        of replaced / removed rules stay.  True once any of them has more than doubled since
        the full compile (a fresh compiler then reclaims them; the regex matrix each batch
        computes is one cell per row, so stale rows cost every encode)."""
        if self._base is None:
            return False
        return any(now > 2 * base + 64 for now, base in zip(self._sizes(), self._base))

    def compile(self, policy_sets: dict, dirty=None) -> CompiledStore:
        """``dirty``: keys whose sets changed in place (None: every set)."""
        frags, new = [], {}
        for key, ps in policy_sets.items():
            f = self.frags.get(key)
            if f is None or f.obj is not ps or dirty is None or key in dirty:
                f = _compile_set(self.b, ps)
                self.stats["sets_compiled"] += 1
            else:
                self.stats["sets_reused"] += 1
            frags.append(f)
            new[key] = f
        self.frags = new
        self.stats["compiles"] += 1
        if self._base is None:
            self._base = self._sizes()
        return _assemble(self.b, frags)


def compile_store(policy_sets: dict, urns: dict, combining_algorithms: list) -> CompiledStore:
    """Snapshot ``policy_sets`` (ordered Map of sets, see store.py) into node tables."""
    return IncrementalCompiler(urns, combining_algorithms).compile(policy_sets)


def snapshot_json(policy_sets: dict) -> bytes:
    """The policySets Map as the JSON snapshot acs_store_compile reads: the Map's values in
    order, each set's / policy's ``combinables`` the list of its Map's values (JSON.stringify
    of Array.from(map.values()) at each level, as a Node host produces it)."""
    import json

    def clean(v):
        if isinstance(v, dict):
            return {k: clean(x) for k, x in v.items() if x is not MISSING}
        if isinstance(v, list):
            return [None if x is MISSING else clean(x) for x in v]
        return v

    def pol(p):
        if p is None or p is MISSING:
            return None
        out = clean({k: v for k, v in p.items() if k != "combinables"})
        out["combinables"] = [None if r is None or r is MISSING else clean(r) for r in p["combinables"].values()]
        return out

    sets = []
    for ps in policy_sets.values():
        if not isinstance(ps, dict):
            sets.append(None)
            continue
        out = clean({k: v for k, v in ps.items() if k not in ("combinables", "policies")})
        out["combinables"] = [pol(p) for p in ps["combinables"].values()]
        sets.append(out)
    return json.dumps(sets, ensure_ascii=False, separators=(",", ":")).encode("utf-8", "surrogatepass")


def set_texts(policy_sets: dict) -> list:
    """Each policy set's element of snapshot_json (the JSON text acs_store_builder_compile keys
    its fragments by), in Map order."""
    import json
    snap = json.loads(snapshot_json(policy_sets))
    return [json.dumps(x, ensure_ascii=False, separators=(",", ":")).encode("utf-8", "surrogatepass") for x in snap]


class NativeStoreBuilder:
    """acs_store_builder (include/acs_mi355x.h): the native compiler keeping one compiled
    fragment per policy set, so a compile after a mutation recompiles only the changed sets."""

    def __init__(self, urns: dict, combining_algorithms: list):
        import ctypes as C
        import json
        from .native import last_error, load
        self.C, self._err = C, last_error
        self.lib = lib = load()
        lib.acs_store_builder_create.restype = C.c_void_p
        lib.acs_store_builder_create.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]
        lib.acs_store_builder_compile.argtypes = [C.c_void_p, C.POINTER(C.c_char_p), C.POINTER(C.c_size_t), C.c_size_t,
                                                  C.POINTER(C.c_void_p), C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
        lib.acs_store_builder_free.argtypes = [C.c_void_p]
        lib.acs_blob_free.argtypes = [C.c_void_p]
        u, c = json.dumps(urns).encode(), json.dumps(combining_algorithms).encode()
        self.h = lib.acs_store_builder_create(u, len(u), c, len(c))
        if not self.h:
            raise Unsupported(last_error(lib))
        self.recompiled = 0

    def compile_texts(self, texts) -> bytes:
        C = self.C
        n = len(texts)
        arr = (C.c_char_p * n)(*texts)
        lens = (C.c_size_t * n)(*[len(t) for t in texts])
        out, nb, rec = C.c_void_p(), C.c_size_t(), C.c_size_t()
        if self.lib.acs_store_builder_compile(self.h, arr, lens, n, C.byref(out), C.byref(nb), C.byref(rec)) != 0:
            raise Unsupported(self._err(self.lib))
        self.recompiled = rec.value
        try:
            return C.string_at(out.value, nb.value)
        finally:
            self.lib.acs_blob_free(out)

    def stage(self, text: bytes) -> int:
        """acs_store_builder_stage: one set's text taken ahead of the next compile; returns the
        handle to pass in compile_items."""
        C = self.C
        self.lib.acs_store_builder_stage.restype = C.c_longlong
        self.lib.acs_store_builder_stage.argtypes = [C.c_void_p, C.c_char_p, C.c_size_t]
        h = self.lib.acs_store_builder_stage(self.h, text, len(text))
        if h < 0:
            raise Unsupported(self._err(self.lib))
        return h

    def compile_items(self, items) -> bytes:
        """items[k]: set k's text (bytes), ("prev", j) = the previous compile's set j, or
        ("staged", h) = a stage() handle."""
        C = self.C
        n = len(items)
        staged = 1 << (8 * C.sizeof(C.c_size_t) - 1)
        arr = (C.c_char_p * n)(*[x if isinstance(x, bytes) else None for x in items])
        lens = (C.c_size_t * n)(*[len(x) if isinstance(x, bytes) else (x[1] if x[0] == "prev" else staged | x[1])
                                  for x in items])
        out, nb, rec = C.c_void_p(), C.c_size_t(), C.c_size_t()
        if self.lib.acs_store_builder_compile(self.h, arr, lens, n, C.byref(out), C.byref(nb), C.byref(rec)) != 0:
            raise Unsupported(self._err(self.lib))
        self.recompiled = rec.value
        try:
            return C.string_at(out.value, nb.value)
        finally:
            self.lib.acs_blob_free(out)

    def compile(self, policy_sets: dict) -> bytes:
        return self.compile_texts(set_texts(policy_sets))

    def close(self):
        if self.h:
            self.lib.acs_store_builder_free(self.h)
            self.h = None


def native_store_blob(policy_sets: dict, urns: dict, combining_algorithms: list) -> bytes:
    """The store image compiled by the native compiler (acs_store_compile)."""
    import ctypes as C
    import json
    from .native import last_error, load
    lib = load()
    lib.acs_store_compile.argtypes = [C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t,
                                      C.POINTER(C.c_void_p), C.POINTER(C.c_size_t)]
    lib.acs_blob_free.argtypes = [C.c_void_p]
    snap = snapshot_json(policy_sets)
    u = json.dumps(urns).encode()
    c = json.dumps(combining_algorithms).encode()
    out, n = C.c_void_p(), C.c_size_t()
    if lib.acs_store_compile(snap, len(snap), u, len(u), c, len(c), C.byref(out), C.byref(n)) != 0:
        raise Unsupported(last_error(lib))
    try:
        return C.string_at(out.value, n.value)
    finally:
        lib.acs_blob_free(out)


# URN config names the native request codec (csrc/acs_codec.cpp) reads, in this order.
CODEC_URNS = ("entity", "property", "operation", "resourceID", "actionID", "role", "roleScopingEntity",
              "roleScopingInstance", "hierarchicalRoleScoping", "ownerEntity", "ownerInstance",
              "aclIndicatoryEntity", "aclInstance", "create", "read", "modify", "delete", "user", "skipACL",
              "maskedProperty")
CODEC_MAGIC, CODEC_VERSION = 0x43534341, 2  # "ACSC"
ABI_VERSION = 5  # include/acs_mi355x.h ACS_ABI_VERSION (store image header)


def codec_section(cs: CompiledStore) -> bytes:
    """What the native request codec needs besides the node tables (include/acs_mi355x.h,
    acs_codec_create): the interned dictionary (id -> UTF-8 string), the URN ids, the rule
    entity value of every regex-matrix row and the per-node candidate specs (candidates.py)."""
    import struct
    d = cs.dictionary
    urn_ids = [d.intern(cs.urns.get(k, MISSING)) if isinstance(cs.urns.get(k, MISSING), str) or
               cs.urns.get(k, MISSING) is MISSING else L.ID_UNDEF for k in CODEC_URNS]
    rx = [d.lookup(v) for v in cs.rx_rows]
    spec = [x for sec in cs.cand_spec for x in sec]
    kind = np.array([1 if x is None else (2 if x else 0) for x in spec], np.uint8)
    ptr = np.zeros(len(spec) + 1, np.uint32)
    idx = []
    for k, x in enumerate(spec):
        if x:
            idx.extend(x)
        ptr[k + 1] = len(idx)
    enc = [s.encode("utf-8", "surrogatepass") if isinstance(s, str) else b"" for s in d.strings]
    offs = np.zeros(len(enc) + 1, np.uint32)
    offs[1:] = np.cumsum([len(e) for e in enc]) if enc else []
    sbytes = b"".join(enc)

    def pad4(b):
        return b + b"\0" * ((-len(b)) % 4)
    hdr = struct.pack("<8I", CODEC_MAGIC, CODEC_VERSION, len(enc), len(CODEC_URNS), len(rx), len(spec), len(idx),
                      len(sbytes))
    # evaluation_cacheable values beyond undefined / null / false / true (codes 4..), as JSON
    import json
    ec = json.dumps(list(cs.ec_values[4:]), ensure_ascii=False, separators=(",", ":")).encode("utf-8", "surrogatepass")
    return b"".join([hdr, np.array(urn_ids, np.uint32).tobytes(), np.array(rx, np.uint32).tobytes(),
                     pad4(kind.tobytes()), ptr.tobytes(), np.array(idx, np.uint32).tobytes(), offs.tobytes(),
                     pad4(sbytes), struct.pack("<I", len(ec)), pad4(ec)])


def store_blob(cs: CompiledStore, codec: bool = True) -> bytes:
    """Serialise tables into the acs_compile() image (include/acs_mi355x.h: acs_blob_header),
    followed by the codec section (header reserved[0] / [1] = its byte offset / length)."""
    import struct
    parts = []
    for a in (cs.sets, cs.pols, cs.rules, cs.rres, cs.pairs, cs.u32pool):
        b = np.ascontiguousarray(a).tobytes()
        parts.append(b + b"\0" * ((-len(b)) % 16))
    body = b"".join(parts)
    sec = codec_section(cs) if codec else b""
    off = 64 + len(body) if sec else 0
    hdr = struct.pack("<16I", 0x31534341, ABI_VERSION, cs.n_sets, cs.n_pols, cs.n_rules, len(cs.rres),
                      len(cs.pairs), len(cs.u32pool), cs.id_user, off, len(sec), 0, 0, 0, 0, 0)
    return hdr + body + sec
