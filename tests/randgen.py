"""Seeded random policy stores + requests for differential tests (oracle vs evaluator).

Small vocabularies on purpose: collisions exercise entity stickiness, namespace
resets, regex substring hits (Ent1 in Ent12), property indexOf quirks, HR
owner/scope matching, ACL create/read paths, undefined/null values, odd
effect strings, invalid combining algorithms and null Map entries.
"""
import random

from oracle.acs_oracle import FULL_URNS, CORE_SPEC_URNS, CA_DENY, CA_PERMIT, CA_FIRST

U = FULL_URNS
ORG = "urn:restorecommerce:acs:model:organization.Organization"
USER = "urn:restorecommerce:acs:model:user.User"
ENTITIES = [
    "urn:restorecommerce:acs:model:location.Location",
    ORG,
    USER,
    "urn:restorecommerce:acs:model:ent1.Ent1",
    "urn:restorecommerce:acs:model:ent12.Ent12",
    "urn:other:acs:model:ent1.Ent1",
    "urn:restorecommerce:acs:model:Ent1",
    "urn:restorecommerce:acs:model:ns.sub.Ent1",
    "urn:restorecommerce:acs:model:ns.Ent",
    "urn:restorecommerce:acs:model:ent1.Ent1*",
    "urn:restorecommerce:acs:model:x.Ent(1|2)",
]
REQ_ENTITIES = ENTITIES[:9] + ["urn:restorecommerce:acs:model:ENT1.ent1", "urn:restorecommerce:acs:model:ns.Ent12"]
ROLES = ["SimpleUser", "Admin", "r2", "r3"]
ORGS = ["o0", "o1", "o2", "o3", "o4", "SuperOrg1", "Org1"]
ACTIONS = [U["read"], U["modify"], U["create"], U["delete"], "urn:restorecommerce:acs:names:action:execute"]
OPS = ["mutation.A", "mutation.B", "query.C"]
IDS = ["id0", "id1", "id2", "mutation.A"]
EFFECTS = ["PERMIT", "DENY", "PERMIT", "DENY", "Permit", "", None, "NOT_APPLICABLE"]
CAS = [CA_DENY, CA_PERMIT, CA_FIRST]


def _maybe(r, p):
    return r.random() < p


def _props(r, ent):
    base = ent[ent.rfind(":") + 1:] if r.random() < 0.85 else r.choice(ENTITIES)[-12:]
    return [f"urn:restorecommerce:acs:model:{base}#{r.choice(['id', 'name', 'desc', 'x'])}"]


def rand_target(r, urns, level):
    t = {}
    subs = []
    if _maybe(r, 0.6):
        subs.append({"id": urns.get("role", U["role"]), "value": r.choice(ROLES)})
    if _maybe(r, 0.15):
        subs.append({"id": U["subjectID"] if "subjectID" in U else "urn:oasis:names:tc:xacml:1.0:subject:subject-id",
                     "value": r.choice(["Alice", "Bob"])})
    if _maybe(r, 0.35):
        subs.append({"id": U["roleScopingEntity"], "value": r.choice([ORG, ORG, USER, ""])})
    if _maybe(r, 0.12):
        subs.append({"id": U["hierarchicalRoleScoping"], "value": r.choice(["true", "false"])})
    if _maybe(r, 0.05):
        subs.append({"id": U["skipACL"], "value": "true"})
    if subs or _maybe(r, 0.5):
        t["subjects"] = subs
    res = []
    k = r.choice([0, 1, 1, 1, 2, 3])
    for _ in range(k):
        x = r.random()
        if x < 0.55:
            res.append({"id": U["entity"], "value": r.choice(ENTITIES)})
        elif x < 0.8:
            e = r.choice(ENTITIES)
            res.append({"id": U["property"], "value": _props(r, e)[0]})
        elif x < 0.92:
            res.append({"id": U["operation"], "value": r.choice(OPS)})
        else:
            res.append({"id": U["resourceID"], "value": r.choice(IDS)})
    if res or _maybe(r, 0.5):
        t["resources"] = res
    if _maybe(r, 0.55):
        t["actions"] = [{"id": U["actionID"], "value": r.choice(ACTIONS)}]
    return t


def rand_store(r, urns):
    sets = []
    for s in range(r.randint(1, 3)):
        pols = []
        for p in range(r.randint(0, 4)):
            rules = []
            for q in range(r.randint(0, 5)):
                rule = {"id": f"R{s}{p}{q}"}
                if _maybe(r, 0.85):
                    rule["target"] = rand_target(r, urns, "rule")
                e = r.choice(EFFECTS)
                if e is not None:
                    rule["effect"] = e
                ec = r.choice([True, False, None, "absent"])
                if ec != "absent":
                    rule["evaluation_cacheable"] = ec
                if _maybe(r, 0.04):
                    rule["condition"] = "context && context.subject && context.subject.id === 'Alice'"
                rules.append(rule)
            pol = {"id": f"P{s}{p}", "combining_algorithm": r.choice(CAS + ([None] if _maybe(r, 0.05) else []))}
            if pol["combining_algorithm"] is None:
                pol["combining_algorithm"] = "urn:bogus:ca"
            if _maybe(r, 0.35):
                pol["effect"] = r.choice(["PERMIT", "DENY", "PERMIT", "Deny"])
            if _maybe(r, 0.6):
                pol["target"] = rand_target(r, urns, "policy")
            if rules or _maybe(r, 0.8):
                pol["rules"] = rules
            if _maybe(r, 0.3):
                pol["evaluation_cacheable"] = r.choice([True, False])
            pols.append(pol)
        ps = {"id": f"S{s}", "combining_algorithm": r.choice(CAS), "policies": pols}
        if _maybe(r, 0.25):
            ps["target"] = {"subjects": [{"id": urns.get("role", U["role"]), "value": r.choice(ROLES)}]}
        sets.append(ps)
    return {"policy_sets": sets}


def _hr_forest(r, roles):
    roots = []
    for _ in range(r.randint(0, 2)):
        def node(d):
            n = {"id": r.choice(ORGS)}
            if d < 2 and _maybe(r, 0.6):
                n["children"] = [node(d + 1) for _ in range(r.randint(1, 2))]
            if d > 0 and _maybe(r, 0.1):
                n["role"] = r.choice(roles)
            return n
        root = node(0)
        if _maybe(r, 0.9):
            root["role"] = r.choice(roles)
        roots.append(root)
    return roots


def rand_request(r, urns):
    req = {}
    roles = r.sample(ROLES, r.randint(0, 2))
    if _maybe(r, 0.97):
        subs = [{"id": U["role"], "value": roles[0] if roles else "SimpleUser"},
                {"id": "urn:oasis:names:tc:xacml:1.0:subject:subject-id", "value": r.choice(["Alice", "Bob"])}]
        res = []
        for _ in range(r.choice([1, 1, 2, 2, 3])):
            x = r.random()
            if x < 0.7:
                e = r.choice(REQ_ENTITIES)
                if _maybe(r, 0.03):
                    res.append({"id": U["entity"]})
                else:
                    res.append({"id": U["entity"], "value": e})
                if _maybe(r, 0.8):
                    rid = {"id": U["resourceID"]}
                    if _maybe(r, 0.9):
                        rid["value"] = r.choice(IDS)
                    res.append(rid)
                for _ in range(r.choice([0, 0, 1, 2, 3])):
                    res.append({"id": U["property"], "value": _props(r, e)[0]})
            else:
                res.append({"id": U["operation"], "value": r.choice(OPS)})
        if _maybe(r, 0.1):
            r.shuffle(res)
        acts = [{"id": U["actionID"], "value": r.choice(ACTIONS)}] if _maybe(r, 0.95) else []
        req["target"] = {"subjects": subs, "resources": res, "actions": acts}
    x = r.random()
    if x < 0.04:
        return req
    if x < 0.08:
        req["context"] = {}
        return req
    ctx = {}
    subject = {"id": r.choice(["Alice", "Bob", "o1"])}
    if _maybe(r, 0.92):
        ras = []
        for role in roles:
            ra = {"role": role, "attributes": []}
            for _ in range(r.randint(0, 2)):
                ra["attributes"].append({"id": U["roleScopingEntity"], "value": r.choice([ORG, ORG, USER]),
                                         "attributes": [{"id": U["roleScopingInstance"], "value": r.choice(ORGS)}
                                                        for _ in range(r.randint(0, 2))]})
            ras.append(ra)
        subject["role_associations"] = ras
    if _maybe(r, 0.85):
        subject["hierarchical_scopes"] = _hr_forest(r, roles or ["SimpleUser"])
    if _maybe(r, 0.95):
        ctx["subject"] = subject
    cres = []
    used = [a.get("value") for a in req.get("target", {}).get("resources", [])
            if a["id"] in (U["resourceID"], U["operation"]) and a.get("value")]
    pool = list(dict.fromkeys(used + r.sample(IDS, r.randint(0, 2)))) if _maybe(r, 0.6) else r.sample(IDS, r.randint(0, 3))
    tree_orgs = []
    for h in subject.get("hierarchical_scopes", []) or []:
        stack = [h]
        while stack:
            n = stack.pop()
            tree_orgs.append(n["id"])
            stack.extend(n.get("children", []))
    for iid in pool:
        meta = {}
        if _maybe(r, 0.85):
            meta["owners"] = []
            for _ in range(r.randint(0, 2)):
                o = {"id": U["ownerIndicatoryEntity"] if "ownerIndicatoryEntity" in U else
                     "urn:restorecommerce:acs:names:ownerIndicatoryEntity",
                     "value": r.choice([ORG, ORG, USER])}
                if _maybe(r, 0.95):
                    o["attributes"] = [{"id": U["ownerInstance"],
                                        "value": r.choice(tree_orgs) if (tree_orgs and _maybe(r, 0.6)) else r.choice(ORGS)}
                                       for _ in range(r.randint(1, 2))]
                meta["owners"].append(o)
        if _maybe(r, 0.3):
            acls = []
            for _ in range(r.randint(0, 2)):
                acls.append({"id": U["aclIndicatoryEntity"] if _maybe(r, 0.95) else "bogus",
                             "value": r.choice([ORG, USER]),
                             "attributes": [{"id": U["aclInstance"], "value": r.choice(ORGS + ["Alice"])}
                                            for _ in range(r.randint(0, 2))]})
            meta["acls"] = acls
        item = {"id": iid, "meta": meta}
        if _maybe(r, 0.2):
            item = {"instance": {"id": iid, "meta": meta}}
        cres.append(item)
    ctx["resources"] = cres
    req["context"] = ctx
    return req


def rand_case(seed):
    r = random.Random(seed)
    urns = CORE_SPEC_URNS if _maybe(r, 0.2) else FULL_URNS
    store = rand_store(r, urns)
    reqs = [rand_request(r, urns) for _ in range(12)]
    return urns, store, reqs
