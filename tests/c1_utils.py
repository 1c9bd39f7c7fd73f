"""c1 (BASELINE.json configs[0]): data/seed_data + the test/fixtures policy sets in one
store, and synthetic isAllowed requests over the fixtures' own vocabulary.

The store is the reference's DB-shaped seed load (resourceManager.ts:765-797, stitched by
acs_mi355x.store.stitch_db_documents) followed by every test fixture's policy sets, loaded
the way test/utils.ts:345-383 does, each fixture's set ids prefixed with its file name (the
fixtures reuse ids such as PS1, which would otherwise overwrite each other in the Map).  The
requests recombine the golden vectors' requests: attribute values swapped for other values
the fixtures use under the same attribute id, contexts exchanged between requests, and
attributes dropped or added — so every request is shaped like one the reference's tests
send, over values its policies actually match on.
"""
import copy
import json
import os
import random

from acs_mi355x import store as pstore
from kat_utils import GOLDEN, load_kats, load_fixture

FIXTURES = sorted(f for f in os.listdir(os.path.join(GOLDEN, "fixtures")) if f != "seed_data.json")


def c1_store():
    with open(os.path.join(GOLDEN, "fixtures", "seed_data.json")) as f:
        seed = json.load(f)
    m = pstore.stitch_db_documents(seed["policy_sets"], seed["policies"], seed["rules"])
    for name in FIXTURES:  # the fixtures reuse set ids (PS1, ...): one namespace per fixture
        for k, ps in pstore.populate(load_fixture(name)).items():
            key = f"{name[:-5]}/{k}"
            ps["id"] = key
            m[key] = ps
    return m


def _vocab(reqs):
    vals = {}
    for r in reqs:
        t = r.get("target") or {}
        for part in ("subjects", "resources", "actions"):
            for a in t.get(part) or []:
                vals.setdefault((part, a.get("id")), set()).add(json.dumps(a.get("value")))
    roles = set()
    for r in reqs:
        for ra in ((r.get("context") or {}).get("subject") or {}).get("role_associations") or []:
            roles.add(ra.get("role"))
    return {k: sorted(v) for k, v in vals.items()}, sorted(x for x in roles if isinstance(x, str))


def c1_requests(n, seed=0):
    base = [v["request"] for v in load_kats() if v["op"] == "isAllowed"]
    vals, roles = _vocab(base)
    rng = random.Random(seed)
    out = []
    for _ in range(n):
        r = copy.deepcopy(rng.choice(base))
        t = r.get("target")
        if isinstance(t, dict):
            for part in ("subjects", "resources", "actions"):
                attrs = t.get(part) or []
                for a in attrs:
                    if rng.random() < 0.3:
                        a["value"] = json.loads(rng.choice(vals[(part, a.get("id"))]))
                if attrs and rng.random() < 0.08:
                    attrs.pop(rng.randrange(len(attrs)))
                if rng.random() < 0.05:
                    k = rng.choice([k for k in vals if k[0] == part] or [None])
                    if k is not None:
                        attrs.append({"id": k[1], "attributes": [], "value": json.loads(rng.choice(vals[k]))})
        if rng.random() < 0.2:
            r["context"] = copy.deepcopy(rng.choice(base).get("context"))
        ctx = r.get("context") or {}
        subj = ctx.get("subject") if isinstance(ctx, dict) else None
        if isinstance(subj, dict) and roles and rng.random() < 0.2:
            for ra in subj.get("role_associations") or []:
                if rng.random() < 0.5:
                    ra["role"] = rng.choice(roles)
        out.append(r)
    return out
