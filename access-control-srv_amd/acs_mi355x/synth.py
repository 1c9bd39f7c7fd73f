"""Seeded synthetic workloads for the benchmark configurations.

Stores are plain ``{policy_sets: [...]}`` documents (the shape ``populate``
loads).  Request batches are generated directly in the packed layout with
numpy (vectorised: millions of requests per second), and every request can be
re-materialised as the JSON request the reference would receive
(``decode(i)``), which is how the benchmark and the tests check a sample of a
full-size batch against the CPU oracle.

  c2: 100 sets x 2 policies x 5 rules (1k rules), flat roles, no HR/ACL data.
  c3: 200 sets x 5 policies x 10 rules (10k rules), mixed CAs, 50% of rules
      role-scoped to organizations, depth-8 4-ary org tree (21,845 orgs),
      requests carrying hierarchical_scopes subtrees of it (Euler intervals).
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np

from . import layout as L
from .compiler import CompiledStore, Overlay
from .encoder import RequestBatch
from .regex import cell

URN = {
    "role": "urn:restorecommerce:acs:names:role",
    "subjectID": "urn:oasis:names:tc:xacml:1.0:subject:subject-id",
    "entity": "urn:restorecommerce:acs:names:model:entity",
    "property": "urn:restorecommerce:acs:names:model:property",
    "resourceID": "urn:oasis:names:tc:xacml:1.0:resource:resource-id",
    "actionID": "urn:oasis:names:tc:xacml:1.0:action:action-id",
    "rse": "urn:restorecommerce:acs:names:roleScopingEntity",
    "rsi": "urn:restorecommerce:acs:names:roleScopingInstance",
    "hrs": "urn:restorecommerce:acs:names:hierarchicalRoleScoping",
    "ownerEntity": "urn:restorecommerce:acs:names:ownerIndicatoryEntity",
    "ownerInstance": "urn:restorecommerce:acs:names:ownerInstance",
    "aclEntity": "urn:restorecommerce:acs:names:aclIndicatoryEntity",
    "aclInstance": "urn:restorecommerce:acs:names:aclInstance",
}
ACTIONS = ["urn:restorecommerce:acs:names:action:read", "urn:restorecommerce:acs:names:action:modify",
           "urn:restorecommerce:acs:names:action:create", "urn:restorecommerce:acs:names:action:delete",
           "urn:restorecommerce:acs:names:action:execute"]
CAS = ["urn:oasis:names:tc:xacml:3.0:rule-combining-algorithm:deny-overrides",
       "urn:oasis:names:tc:xacml:3.0:rule-combining-algorithm:permit-overrides",
       "urn:oasis:names:tc:xacml:3.0:rule-combining-algorithm:first-applicable"]
ORG_ENTITY = "urn:restorecommerce:acs:model:organization.Organization"
N_ENT, N_ROLES, N_PROPS, N_USERS, N_RIDS = 256, 64, 8, 4096, 1024


def entity(k):
    return f"urn:restorecommerce:acs:model:ent{k}.Ent{k}"


def prop(k, p):
    return f"{entity(k)}#p{p}"


def role(k):
    return f"r{k}"


def zipf_p(n, s=1.1):
    w = 1.0 / np.arange(1, n + 1) ** s
    return w / w.sum()


def _ec(rng, r):
    x = rng.random()
    if x < 0.5:
        r["evaluation_cacheable"] = True
    elif x < 0.75:
        r["evaluation_cacheable"] = False


def _effect(rng):
    x = rng.random()
    if x < 0.001:
        return "Permit"
    return "PERMIT" if x < 0.7 else "DENY"


# ------------------------------------------------------------------ org tree (c3)
class OrgTree:
    """Complete ``fanout``-ary tree of depth ``depth`` in preorder; node k is 'org{k}'.
    Euler tour: subtree(k) = [k, k + size(level(k)))."""

    def __init__(self, fanout=4, depth=8):
        self.fanout, self.depth = fanout, depth
        self.level_sizes = [sum(fanout ** i for i in range(depth - d)) for d in range(depth)]
        self.n = n = self.level_sizes[0]
        level = np.zeros(n, np.int32)
        stack = [(0, 0)]
        while stack:  # preorder ids: the children of x (level d) start at x+1, stride size(d+1)
            x, d = stack.pop()
            level[x] = d
            if d + 1 < depth:
                stride = self.level_sizes[d + 1]
                stack.extend((x + 1 + k * stride, d + 1) for k in range(fanout))
        self.level = level
        self.size = np.array(self.level_sizes, np.int64)[level]

    def name(self, k):
        return f"org{k}"

    def subtree_json(self, k, role=None):
        """hierarchical_scopes entry for the subtree rooted at k (role on the root only).
        Memoised, and every node's dict is built once for the whole tree: a subtree is
        shared, read-only, by its parent and by every request scoped at it."""
        memo = self.__dict__.setdefault("_json_memo", {})
        if (k, role) not in memo:
            if role is not None:
                n = self.subtree_json(k)
                memo[(k, role)] = {"id": n["id"], "role": role, **({"children": n["children"]} if "children" in n else {})}
            else:
                # children first (deepest level up), so each node is built from memoised kids
                for x in sorted(self._subtree_nodes(k), key=lambda x: -int(self.level[x])):
                    if (x, None) in memo:
                        continue
                    d = int(self.level[x])
                    out = {"id": self.name(x)}
                    if d + 1 < self.depth:
                        stride = self.level_sizes[d + 1]
                        out["children"] = [memo[(x + 1 + c * stride, None)] for c in range(self.fanout)]
                    memo[(x, None)] = out
        return memo[(k, role)]

    def _subtree_nodes(self, k):
        return range(k, k + int(self.size[k]))

    def contains(self, root, x):
        return root <= x < root + self.size[root]


# ------------------------------------------------------------------ stores
def c2_store(seed=0xACC0002, n_sets=100, n_pols=2, n_rules=5):
    rng = np.random.default_rng(seed)
    pe = zipf_p(N_ENT)
    pr = zipf_p(N_ROLES)
    pa = zipf_p(len(ACTIONS))
    sets = []
    for s in range(n_sets):
        pols = []
        for p in range(n_pols):
            e = int(rng.choice(N_ENT, p=pe))
            rules = []
            for q in range(n_rules):
                t = {}
                if rng.random() < 0.9:
                    t["subjects"] = [{"id": URN["role"], "value": role(int(rng.choice(N_ROLES, p=pr)))}]
                else:
                    t["subjects"] = [{"id": URN["subjectID"], "value": f"u{int(rng.integers(N_USERS))}"}]
                res = [{"id": URN["entity"], "value": entity(e)}]
                if rng.random() < 0.3:
                    for pp in sorted(set(rng.integers(0, N_PROPS, size=int(rng.integers(1, 3))).tolist())):
                        res.append({"id": URN["property"], "value": prop(e, pp)})
                t["resources"] = res
                if rng.random() < 0.8:
                    t["actions"] = [{"id": URN["actionID"], "value": ACTIONS[int(rng.choice(len(ACTIONS), p=pa))]}]
                r = {"id": f"r{s}_{p}_{q}", "target": t, "effect": _effect(rng)}
                _ec(rng, r)
                rules.append(r)
            pol = {"id": f"p{s}_{p}", "combining_algorithm": CAS[int(rng.integers(3))], "rules": rules}
            if rng.random() < 0.8:
                pol["target"] = {"resources": [{"id": URN["entity"], "value": entity(e)}]}
            if rng.random() < 0.1:
                pol["effect"] = "PERMIT"
            pols.append(pol)
        sets.append({"id": f"s{s}", "combining_algorithm": CAS[int(rng.integers(3))], "policies": pols})
    return {"policy_sets": sets}


def c3_store(seed=0xACC0003, n_sets=200, n_pols=5, n_rules=10):
    rng = np.random.default_rng(seed)
    pe, pr, pa = zipf_p(N_ENT), zipf_p(N_ROLES), zipf_p(len(ACTIONS))
    sets = []
    for s in range(n_sets):
        pols = []
        for p in range(n_pols):
            e = int(rng.choice(N_ENT, p=pe))
            rules = []
            for q in range(n_rules):
                subs = [{"id": URN["role"], "value": role(int(rng.choice(N_ROLES, p=pr)))}]
                if rng.random() < 0.5:
                    subs.append({"id": URN["rse"], "value": ORG_ENTITY})
                    if rng.random() < 0.25:
                        subs.append({"id": URN["hrs"], "value": "false"})
                res = [{"id": URN["entity"], "value": entity(e)}]
                if rng.random() < 0.3:
                    for pp in sorted(set(rng.integers(0, N_PROPS, size=int(rng.integers(1, 3))).tolist())):
                        res.append({"id": URN["property"], "value": prop(e, pp)})
                t = {"subjects": subs, "resources": res}
                if rng.random() < 0.8:
                    t["actions"] = [{"id": URN["actionID"], "value": ACTIONS[int(rng.choice(len(ACTIONS), p=pa))]}]
                r = {"id": f"r{s}_{p}_{q}", "target": t, "effect": _effect(rng)}
                _ec(rng, r)
                rules.append(r)
            pol = {"id": f"p{s}_{p}", "combining_algorithm": CAS[int(rng.integers(3))], "rules": rules}
            if rng.random() < 0.8:
                pol["target"] = {"resources": [{"id": URN["entity"], "value": entity(e)}]}
            if rng.random() < 0.1:
                pol["effect"] = "PERMIT"
            pols.append(pol)
        sets.append({"id": f"s{s}", "combining_algorithm": CAS[int(rng.integers(3))], "policies": pols})
    return {"policy_sets": sets}


def c3_adverse_store(seed=0xACC0006, n_cond=50, early_sets=20, null_set=7):
    """c3-adverse: the c3 store made hostile to the kernel's early stops (NF_CLEAN_BELOW fails
    below the top sets): ``n_cond`` rules (0.5 %) of the first ``early_sets`` sets carry a
    `condition` (utils.ts:47-56: the request goes to the host when one is reached), and set
    ``null_set`` holds a null policy entry (accessController.ts:138: the TypeError of loop 2a),
    behind a set target of a rare role so that only its requests throw."""
    doc = c3_store()
    rng = np.random.default_rng(seed)
    sets = doc["policy_sets"]
    early = [(s, p, q) for s in range(early_sets) for p in range(len(sets[s]["policies"]))
             for q in range(len(sets[s]["policies"][p]["rules"]))]
    for k in rng.choice(len(early), size=n_cond, replace=False):
        s, p, q = early[int(k)]
        sets[s]["policies"][p]["rules"][q]["condition"] = "context.subject.id === 'u0'"
    sets[null_set]["target"] = {"subjects": [{"id": URN["role"], "value": role(50)}]}
    pols = sets[null_set]["policies"]
    pols[2] = {"id": pols[2]["id"], "$null": True}
    return doc


def c5_store(seed=0xACC0005, n_sets=1000, n_pols=10, n_rules=100):
    """c5: 1,000 sets x 10 policies x 100 rules = 1M rules, the c3 rule mix (roles, 50%
    organization-scoped with 25% of those hierarchicalRoleScoping 'false', 30% with
    properties, 80% with an action), drawn vectorised (one draw per attribute kind)."""
    rng = np.random.default_rng(seed)
    P, R = n_sets * n_pols, n_sets * n_pols * n_rules
    pol_ent = rng.choice(N_ENT, size=P, p=zipf_p(N_ENT))
    pol_ca = rng.integers(3, size=P)
    pol_tgt = rng.random(P) < 0.8
    pol_eff = rng.random(P) < 0.1
    set_ca = rng.integers(3, size=n_sets)
    r_role = rng.choice(N_ROLES, size=R, p=zipf_p(N_ROLES))
    r_rse = rng.random(R) < 0.5
    r_hrs = rng.random(R) < 0.25
    r_props = rng.random(R) < 0.3
    r_np = rng.integers(1, 3, size=R)
    r_pp = rng.integers(0, N_PROPS, size=(R, 2))
    r_act = rng.random(R) < 0.8
    r_a = rng.choice(len(ACTIONS), size=R, p=zipf_p(len(ACTIONS)))
    x = rng.random(R)
    r_eff = np.where(x < 0.001, 2, np.where(x < 0.7, 0, 1))
    y = rng.random(R)
    r_ec = np.where(y < 0.5, 1, np.where(y < 0.75, 0, -1))
    effects = ["PERMIT", "DENY", "Permit"]
    role_v = [role(k) for k in range(N_ROLES)]
    ent_v = [entity(k) for k in range(N_ENT)]
    sets, k = [], 0
    for s in range(n_sets):
        pols = []
        for p in range(n_pols):
            pi = s * n_pols + p
            e = int(pol_ent[pi])
            rules = []
            for q in range(n_rules):
                subs = [{"id": URN["role"], "value": role_v[r_role[k]]}]
                if r_rse[k]:
                    subs.append({"id": URN["rse"], "value": ORG_ENTITY})
                    if r_hrs[k]:
                        subs.append({"id": URN["hrs"], "value": "false"})
                res = [{"id": URN["entity"], "value": ent_v[e]}]
                if r_props[k]:
                    for pp in sorted(set(r_pp[k, :r_np[k]].tolist())):
                        res.append({"id": URN["property"], "value": prop(e, pp)})
                t = {"subjects": subs, "resources": res}
                if r_act[k]:
                    t["actions"] = [{"id": URN["actionID"], "value": ACTIONS[r_a[k]]}]
                r = {"id": f"r{s}_{p}_{q}", "target": t, "effect": effects[r_eff[k]]}
                if r_ec[k] >= 0:
                    r["evaluation_cacheable"] = bool(r_ec[k])
                rules.append(r)
                k += 1
            pol = {"id": f"p{s}_{p}", "combining_algorithm": CAS[pol_ca[pi]], "rules": rules}
            if pol_tgt[pi]:
                pol["target"] = {"resources": [{"id": URN["entity"], "value": ent_v[e]}]}
            if pol_eff[pi]:
                pol["effect"] = "PERMIT"
            pols.append(pol)
        sets.append({"id": f"s{s}", "combining_algorithm": CAS[set_ca[s]], "policies": pols})
    return {"policy_sets": sets}


# ------------------------------------------------------------------ requests (packed)
@dataclass
class SynthBatch:
    batch: RequestBatch
    draws: dict
    kind: str
    tree: OrgTree | None = None

    def decode(self, i, shared=None):
        """JSON request (post-unmarshall shape) for packed request i.  ``shared``: a
        SharedValues table — the request's hierarchical_scopes tree (up to 21,845 orgs at
        c3) is then the placeholder {"$shared": k} for the table's k-th value, which the C++
        oracle parses once for all the requests naming it (oracle/acs_oracle_c.COracle.raw)."""
        d = {k: v[i] for k, v in self.draws.items()}
        e, r, a, u = int(d["ent"]), int(d["role"]), int(d["act"]), int(d["user"])
        res = [{"id": URN["entity"], "value": entity(e)},
               {"id": URN["resourceID"], "value": f"res{int(d['rid'])}"}]
        for k in range(int(d["nprops"])):
            pe = int(d["prop_ent"][k])
            res.append({"id": URN["property"], "value": prop(pe, int(d["props"][k]))})
        req = {"target": {"subjects": [{"id": URN["role"], "value": role(r)},
                                       {"id": URN["subjectID"], "value": f"u{u}"}],
                          "resources": res,
                          "actions": [{"id": URN["actionID"], "value": ACTIONS[a]}]}}
        subj = {"id": f"u{u}"}
        if self.kind == "c2":
            subj["role_associations"] = [{"role": role(r), "attributes": []}]
            subj["hierarchical_scopes"] = []
            req["context"] = {"subject": subj, "resources": []}
        else:
            t = self.tree
            scope = int(d["scope"])
            subj["role_associations"] = [{"role": role(r), "attributes": [
                {"id": URN["rse"], "value": ORG_ENTITY,
                 "attributes": [{"id": URN["rsi"], "value": t.name(scope)}]}]}]
            r2 = int(d.get("role2", -1))
            scopes = [(scope, r)]
            if r2 >= 0:  # a second role association, scoped to its own org
                sc2 = int(d["scope2"])
                subj["role_associations"].append({"role": role(r2), "attributes": [
                    {"id": URN["rse"], "value": ORG_ENTITY,
                     "attributes": [{"id": URN["rsi"], "value": t.name(sc2)}]}]})
                scopes.append((sc2, r2))
            subj["hierarchical_scopes"] = []
            for sc, rr in scopes:
                tree = t.subtree_json(sc, role(rr))
                if shared is not None and "children" in tree:  # one shared children list per scope org
                    tree = dict(tree, children=shared.ref(sc, tree["children"]))
                subj["hierarchical_scopes"].append(tree)
            owner = int(d["owner"])
            meta = {"owners": [{"id": URN["ownerEntity"], "value": ORG_ENTITY,
                                "attributes": [{"id": URN["ownerInstance"], "value": t.name(owner)}]}]}
            if int(d.get("acl", -1)) >= 0:  # c3-adverse: an ACL on the resource (verifyACL.ts:37-88)
                meta["acls"] = [{"id": URN["aclEntity"], "value": ORG_ENTITY,
                                 "attributes": [{"id": URN["aclInstance"], "value": t.name(int(d["acl"]))}]}]
            req["context"] = {"subject": subj, "resources": [{"id": f"res{int(d['rid'])}", "meta": meta}]}
        return req


    def json_text(self, idx=None) -> bytes:
        """JSON array text of requests ``idx`` (default: all), built from string templates —
        millions per second's worth, for the end-to-end (JSON -> decision) measurement.  Equal,
        request for request, to ``json.dumps(decode(i))`` except that at c3 the subject names
        its HR forests by reference — ``"$hrs": [keys]``, one registered forest per role
        association, in place of the inline ``hierarchical_scopes`` trees (the per-subject
        forest cache of acs_codec, which concatenates the listed forests' roots; register them
        with ``hrs_forests``)."""
        d = self.draws
        idx = np.arange(self.batch.n) if idx is None else np.asarray(idx)
        u_ent, u_prop, u_rid = URN["entity"], URN["property"], URN["resourceID"]
        ents = [f'{{"id":"{u_ent}","value":"{entity(k)}"}}' for k in range(N_ENT)]
        props = [[f',{{"id":"{u_prop}","value":"{prop(k, p)}"}}' for p in range(N_PROPS)] for k in range(N_ENT)]
        acts = [f'"actions":[{{"id":"{URN["actionID"]}","value":"{a}"}}]' for a in ACTIONS]
        pre_s = f'{{"target":{{"subjects":[{{"id":"{URN["role"]}","value":"r'
        mid_s = f'"}},{{"id":"{URN["subjectID"]}","value":"u'
        out = []
        ent, rol, act, usr, rid, npr, pr, pe = (d["ent"], d["role"], d["act"], d["user"], d["rid"], d["nprops"],
                                                d["props"], d["prop_ent"])
        c3 = self.kind != "c2"
        if c3:
            scope, owner = d["scope"], d["owner"]
            role2 = d.get("role2", np.full(len(ent), -1))
            scope2 = d.get("scope2", np.zeros(len(ent), np.int64))
            acl = d.get("acl", np.full(len(ent), -1))
            ae, ai = URN["aclEntity"], URN["aclInstance"]
            rse, rsi, oe, oi = URN["rse"], URN["rsi"], URN["ownerEntity"], URN["ownerInstance"]
        for i in idx.tolist():
            e, r, u = int(ent[i]), int(rol[i]), int(usr[i])
            res = ents[e] + f',{{"id":"{u_rid}","value":"res{int(rid[i])}"}}' + \
                "".join(props[int(pe[i, k])][int(pr[i, k])] for k in range(int(npr[i])))
            head = f'{pre_s}{r}{mid_s}{u}"}}],"resources":[{res}],{acts[int(act[i])]}}},'
            if not c3:
                ctx = (f'"context":{{"subject":{{"id":"u{u}","role_associations":[{{"role":"r{r}","attributes":[]}}],'
                       f'"hierarchical_scopes":[]}},"resources":[]}}}}')
            else:
                sc, r2 = int(scope[i]), int(role2[i])
                ra2 = (f',{{"role":"r{r2}","attributes":[{{"id":"{rse}","value":"{ORG_ENTITY}","attributes":'
                       f'[{{"id":"{rsi}","value":"org{int(scope2[i])}"}}]}}]}}') if r2 >= 0 else ""
                ctx = (f'"context":{{"subject":{{"id":"u{u}","role_associations":[{{"role":"r{r}","attributes":['
                       f'{{"id":"{rse}","value":"{ORG_ENTITY}","attributes":[{{"id":"{rsi}","value":"org{sc}"}}]}}]}}{ra2}],'
                       f'"$hrs":{self.hrs_keys_json(i)}}},"resources":[{{"id":"res{int(rid[i])}","meta":{{"owners":['
                       f'{{"id":"{oe}","value":"{ORG_ENTITY}","attributes":[{{"id":"{oi}","value":"org{int(owner[i])}"}}]}}'
                       + (f'],"acls":[{{"id":"{ae}","value":"{ORG_ENTITY}","attributes":[{{"id":"{ai}",'
                          f'"value":"org{int(acl[i])}"}}]}}' if int(acl[i]) >= 0 else '') +
                       f']}}}}]}}}}')
            out.append(head + ctx)
        return ("[" + ",".join(out) + "]").encode()

    def hrs_keys(self, i):
        """The subject forests a c3 request names, one per role association: (scope org, role),
        and the second association's when it has one; their root arrays concatenate into the
        subject's hierarchical_scopes."""
        keys = [(int(self.draws["scope"][i]), int(self.draws["role"][i]))]
        r2 = int(self.draws["role2"][i]) if "role2" in self.draws else -1
        if r2 >= 0:
            keys.append((int(self.draws["scope2"][i]), r2))
        return keys

    def hrs_keys_json(self, i):
        return "[" + ",".join(f'"s{sc}:r{r}"' for sc, r in self.hrs_keys(i)) + "]"

    def hrs_forests(self, idx=None):
        """{key: hierarchical_scopes} of the per-association forests requests ``idx`` name (the
        forests to register: at most one per (scope org, role))."""
        out = {}
        idx = np.arange(self.batch.n) if idx is None else np.asarray(idx)
        for i in idx.tolist():
            for sc, r in self.hrs_keys(i):
                k = f"s{sc}:r{r}"
                if k not in out:
                    out[k] = [self.tree.subtree_json(sc, role(r))]
        return out


class SharedValues:
    """Values shared by many decoded requests, referenced as {"$shared": k}."""

    def __init__(self):
        self.index, self.values = {}, []

    def ref(self, key, value):
        k = self.index.get(key)
        if k is None:
            k = self.index[key] = len(self.values)
            self.values.append(value)
        return {"$shared": k}


def _vocab(cs: CompiledStore, ov: Overlay):
    I = ov.intern
    return {
        "ent": np.array([I(entity(k)) for k in range(N_ENT)], np.uint32),
        "prop": np.array([[I(prop(k, p)) for p in range(N_PROPS)] for k in range(N_ENT)], np.uint32),
        "psfx": np.array([I(f"p{p}") for p in range(N_PROPS)], np.uint32),
        "role": np.array([I(role(k)) for k in range(N_ROLES)], np.uint32),
        "user": np.array([I(f"u{k}") for k in range(N_USERS)], np.uint32),
        "rid": np.array([I(f"res{k}") for k in range(N_RIDS)], np.uint32),
        "act": np.array([I(a) for a in ACTIONS], np.uint32),
        "urn_role": I(URN["role"]), "urn_subject": I(URN["subjectID"]), "urn_action": I(URN["actionID"]),
    }


def requests(cs: CompiledStore, n: int, kind="c2", seed=0xACC1002, tree: OrgTree | None = None,
             second_role=0.0, acl=0.0, classes=True) -> SynthBatch:
    """Generate n packed requests for config ``kind`` ('c2' or 'c3') against store ``cs``.
    c3: a fraction ``second_role`` of the subjects carries a second role association (SURVEY
    §8(d): 1-2 per request), drawn like the first and distinct from it, scoped to its own random
    org of depth 0-3, with its subtree as a second hierarchical_scopes root.
    c3-adverse: a fraction ``acl`` of the context resources carries an ACL (an org inside the
    subject's scope with p = 0.5); the packed batch flags those requests RQ_HOST (it packs no
    ACL maps) — their batches come from an encoder (the native codec) instead."""
    rng = np.random.default_rng(seed)
    ov = Overlay(cs.dictionary)
    V = _vocab(cs, ov)
    ent = rng.choice(N_ENT, size=n, p=zipf_p(N_ENT)).astype(np.int32)
    rol = rng.choice(N_ROLES, size=n, p=zipf_p(N_ROLES)).astype(np.int32)
    act = rng.choice(len(ACTIONS), size=n, p=zipf_p(len(ACTIONS))).astype(np.int32)
    usr = rng.integers(0, N_USERS, size=n).astype(np.int32)
    rid = rng.integers(0, N_RIDS, size=n).astype(np.int32)
    nprops = rng.integers(0, 4, size=n).astype(np.int32)
    props = np.stack([rng.permutation(N_PROPS)[:3] for _ in range(min(n, 4096))])[np.arange(n) % min(n, 4096)]
    prop_ent = np.where(rng.random((n, 3)) < 0.9, ent[:, None], rng.choice(N_ENT, size=(n, 3))).astype(np.int32)
    draws = {"ent": ent, "role": rol, "act": act, "user": usr, "rid": rid, "nprops": nprops, "props": props,
             "prop_ent": prop_ent}

    hdr = np.zeros(n, L.REQ_HDR_DT)
    res = np.zeros((L.QMAX, n), L.REQ_RES_DT)
    subj = np.zeros((L.SMAX, n), L.PAIR_DT)
    actp = np.zeros((L.AMAX, n), L.PAIR_DT)
    roles = np.zeros((L.RMAX, n), np.uint32)

    # regex-matrix columns: one per entity value (column k <-> entity k)
    rows = cs.rx_rows
    rx = np.array([[cell(rv, entity(k)) for rv in rows] or [0] for k in range(N_ENT)], np.uint8)
    # indexOf(entityName(entity k)) over property strings of entity j
    names = [entity(k)[entity(k).rfind(":") + 1:] for k in range(N_ENT)]
    cont = np.array([[names[k] in prop(j, 0) for j in range(N_ENT)] for k in range(N_ENT)], bool)

    res["value"][0] = V["ent"][ent]
    res["kind"][0] = L.K_ENT | L.K_ENT_LOOSE
    res["col"][0] = ent
    res["slot_a"][0] = res["slot_b"][0] = L.NONE8
    res["value"][1] = V["rid"][rid]
    res["kind"][1] = L.K_RID_LOOSE
    res["slot_a"][1] = res["slot_b"][1] = L.NONE8
    for k in range(3):
        has = nprops > k
        pe = prop_ent[:, k]
        pp = props[:, k]
        res["value"][2 + k] = np.where(has, V["prop"][pe, pp], 0)
        res["kind"][2 + k] = np.where(has, L.K_PROP | L.K_HAS_HASH, 0)
        res["hash_sfx"][2 + k] = np.where(has, V["psfx"][pp], 0)
        res["contains"][2 + k] = np.where(has & cont[ent, pe], 1, 0)
        res["slot_a"][2 + k] = res["slot_b"][2 + k] = L.NONE8
    for k in range(5, L.QMAX):
        res["slot_a"][k] = res["slot_b"][k] = L.NONE8
    subj["id"][0], subj["value"][0] = V["urn_role"], V["role"][rol]
    subj["id"][1], subj["value"][1] = V["urn_subject"], V["user"][usr]
    actp["id"][0], actp["value"][0] = V["urn_action"], V["act"][act]
    roles[0] = V["role"][rol]

    flags = np.full(n, L.RQ_RA_TRUTHY | L.RQ_HRS_ITERABLE | (1 << L.RQ_ENT_SHIFT), np.uint32)  # entity at slot 0
    flags |= np.where(nprops > 0, L.RQ_ANY_PROP, 0).astype(np.uint32)
    flags |= np.where(act == 2, L.RQ_ACT_CREATE, 0).astype(np.uint32)
    flags |= np.where((act == 0) | (act == 1) | (act == 3), L.RQ_ACT_RMD, 0).astype(np.uint32)
    hdr["nres"] = 2 + nprops
    hdr["nsubj"] = 2
    hdr["nact"] = 1
    hdr["nroles"] = 1
    hdr["subject_id"] = V["user"][usr]
    r2 = np.full(n, -1, np.int32)
    if kind != "c2" and second_role > 0:
        r2 = rng.choice(N_ROLES, size=n, p=zipf_p(N_ROLES)).astype(np.int32)
        r2 = np.where(r2 == rol, (r2 + 1) % N_ROLES, r2)
        r2 = np.where(rng.random(n) < second_role, r2, -1).astype(np.int32)
        draws["role2"] = r2
    has2 = r2 >= 0
    hdr["nroles"] = np.where(has2, 2, 1)
    roles[1] = np.where(has2, V["role"][np.maximum(r2, 0)], 0)

    if kind == "c2":
        # no context resources: the first resource-id lookup finds no ACLs -> verifyACL true
        flags |= np.uint32(L.ACL_RET_TRUE << L.RQ_ACL_SHIFT)
        arena = np.zeros(2, np.uint32)
        hdr["arena_off"] = 0
    else:
        tree = tree or OrgTree()

        def draw_scope():  # a random org of depth 0..3
            lv = rng.integers(0, 4, size=n)
            sc = np.zeros(n, np.int64)
            for d in range(4):
                nodes = np.flatnonzero(tree.level == d)
                m = lv == d
                sc[m] = nodes[rng.integers(len(nodes), size=int(m.sum()))]
            return sc

        # subject scoped at a random org of depth 0..3, owner inside its subtree with p=0.6
        scope = draw_scope()
        inside = rng.random(n) < 0.6
        off = (rng.random(n) * tree.size[scope]).astype(np.int64)
        owner = np.where(inside, scope + off, rng.integers(0, tree.n, size=n))
        draws.update({"scope": scope, "owner": owner})
        scope2 = np.zeros(n, np.int64)
        if has2.any():
            scope2 = np.where(has2, draw_scope(), 0)
            draws["scope2"] = scope2
        org_id = np.array([ov.intern(tree.name(k)) for k in range(tree.n)], np.uint32)
        urn_org = ov.intern(ORG_ENTITY)
        in_sub = (owner >= scope) & (owner < scope + tree.size[scope])
        in_sub2 = has2 & (owner >= scope2) & (owner < scope2 + tree.size[scope2])
        # arena per request (acs_layout.h, the encoder's order): counts, grants, rolese, roots,
        # HR keys, 1 slot offset, the owner record.  One role: 17 words; two: 24.
        W = 24 if has2.any() else 22
        ar = np.zeros((n, W), np.uint32)
        R1, R2 = V["role"][rol], V["role"][np.maximum(r2, 0)]
        one, two = ~has2, has2
        ar[one, 0] = 1 | (1 << 8) | (1 << 16) | (1 << 24)
        ar[one, 1] = 0 | (1 << 8)
        ar[one, 2], ar[one, 3], ar[one, 4] = R1[one], urn_org, org_id[scope[one]]   # grant
        ar[one, 5], ar[one, 6] = R1[one], urn_org                                   # rolese
        ar[one, 7] = R1[one]                                                        # root raw role
        ar[one, 8] = R1[one]                                                        # hr key
        ar[one, 9] = 10                                                             # slot 0 offset
        slot1 = 10
        if not has2.any():
            two = np.zeros(0, np.int64)  # no two-role request (W = 22: the two-role columns do not exist)
        ar[two, 0] = 2 | (2 << 8) | (1 << 16) | (2 << 24)
        ar[two, 1] = 0 | (2 << 8)
        ar[two, 2], ar[two, 3], ar[two, 4] = R1[two], urn_org, org_id[scope[two]]   # grants
        ar[two, 5], ar[two, 6], ar[two, 7] = R2[two], urn_org, org_id[scope2[two]]
        ar[two, 8], ar[two, 9] = R1[two], urn_org                                   # rolese
        ar[two, 10], ar[two, 11] = R2[two], urn_org
        ar[two, 12], ar[two, 13] = R1[two], R2[two]                                 # roots
        ar[two, 14], ar[two, 15] = R1[two], R2[two]                                 # hr keys
        ar[two, 16] = 17                                                            # slot 0 offset
        for sel, base in ((one, slot1), (two, 17)) if has2.any() else ((one, slot1),):
            ar[sel, base], ar[sel, base + 1] = 0, 1                                 # owners_empty, n_owners
            ar[sel, base + 2], ar[sel, base + 3] = 1 | (1 << 8), urn_org            # is_oe | 1 attr, value
            ar[sel, base + 4], ar[sel, base + 5] = org_id[owner[sel]], L.K_OI
            ar[sel, base + 6] = in_sub[sel].astype(np.uint32) | (in_sub2[sel].astype(np.uint32) << 1)
        arena = ar.reshape(-1)
        hdr["arena_off"] = (np.arange(n, dtype=np.int64) * W).astype(np.uint32)
        res["slot_a"][1] = 0
        flags |= np.uint32(L.ACL_RET_TRUE << L.RQ_ACL_SHIFT)  # owners-only meta: no ACLs
        if acl > 0:
            has_acl = rng.random(n) < acl
            near = rng.random(n) < 0.5
            a_org = np.where(near, scope + (rng.random(n) * tree.size[scope]).astype(np.int64),
                             rng.integers(0, tree.n, size=n))
            draws["acl"] = np.where(has_acl, a_org, -1)
            flags |= np.where(has_acl, L.RQ_HOST, 0).astype(np.uint32)  # not packed here: encode the JSON
    hdr["flags"] = flags
    b = RequestBatch(n=n, hdr=hdr, res=res, subj=subj, act=actp, roles=roles, arena=arena, rx=rx,
                     rx_rows=rx.shape[1], overlay=ov)
    if classes:  # (False: the caller re-encodes the JSON, e.g. c3-adverse through the codec)
        from .encoder import attach_candidates
        attach_candidates(cs, b, [entity(k) for k in range(N_ENT)])
    return SynthBatch(batch=b, draws=draws, kind=kind, tree=tree if kind != "c2" else None)
