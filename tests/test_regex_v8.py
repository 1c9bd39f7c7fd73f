"""The entity namespace / RegExp test pinned against V8 itself.

tests/golden/regex_cells.json holds ~10k (rule entity value, request entity value)
cells written by tests/golden/gen_regex_cells.js under node (V8's own RegExp engine,
restating accessController.ts:528-566 / hierarchicalScope.ts:64-101).  The product's
host-precomputed cells (acs_mi355x/regex.py), the Python oracle (oracle/jsval.py) and
the C++ oracle must equal V8 on every cell they do not send to the host; the GPU test
runs stores built from the same patterns through K1 / K2 against the pinned oracle.
"""
import json
import os
import warnings

import numpy as np
import pytest

from acs_mi355x import layout as L
from acs_mi355x.regex import cell
from oracle.acs_oracle import Oracle, FULL_URNS, DEFAULT_CAS
from oracle.jsval import OracleUnsupported, JSError

HERE = os.path.dirname(os.path.abspath(__file__))
with open(os.path.join(HERE, "golden", "regex_cells.json")) as f:
    FIX = json.load(f)
PAIRS = FIX["pairs"]
THROWS = L.RX_THROW_TYPE | L.RX_THROW_SYNTAX


def _norm(bits):
    """A throwing cell: the throw decides (the kernel tests throw bits before reset / hit)."""
    return bits & THROWS if bits & THROWS else bits & (L.RX_HIT | L.RX_RESET)


def test_fixture_shape():
    assert len(PAIRS) >= 2000
    kinds = {b for _, _, b in PAIRS}
    assert {0, L.RX_HIT, L.RX_RESET, L.RX_THROW_SYNTAX, L.RX_THROW_TYPE} <= kinds
    # the discriminating cases the fixture exists for
    want = {("urn:x:model:ent.Ent1$", "urn:x:model:ent.Ent1\n"): 0,
            ("urn:x:model:ent.Ent1$", "urn:x:model:ent.Ent1"): L.RX_HIT,
            ("urn:x:model:ent.Ent1", "urn:x:model:ent.Ent12"): L.RX_HIT,
            ("urn:x:model:ent.Ent12", "urn:x:model:ent.Ent1"): 0}
    got = {(a, b): c for a, b, c in PAIRS if (a, b) in want}
    assert got == want


def test_product_cells_equal_v8():
    host = 0
    for rv, qv, want in PAIRS:
        got = cell(rv, qv)
        if got & L.RX_HOST:
            host += 1
            continue
        assert _norm(got) == want, (rv, qv, got, want)
    assert host < 0.1 * len(PAIRS)


def test_python_oracle_equal_v8():
    o = Oracle(FULL_URNS)
    unsup = 0
    for rv, qv, want in PAIRS:
        try:
            reset, hit = o._regex_entity(rv, qv)
            got = (L.RX_RESET if reset else 0) | (L.RX_HIT if hit else 0)
        except OracleUnsupported:
            unsup += 1
            continue
        except JSError as e:
            got = L.RX_THROW_TYPE if e.kind == "TypeError" else L.RX_THROW_SYNTAX
        assert got == want, (rv, qv, got, want)
    assert unsup < 0.1 * len(PAIRS)


def test_cpp_oracle_equal_v8():
    from oracle import acs_oracle_c
    acs_oracle_c.build()
    for rv, qv, want in PAIRS:
        got = acs_oracle_c.regex_cell(rv, qv)
        if got < 0:
            continue
        assert got == want, (rv, qv, got, want)


def test_host_decisions_agree_with_v8_where_product_and_oracle_both_decide():
    """The product sends to the host every pattern the oracle cannot restate (plus non-ASCII
    values, which the oracle computes and the product leaves to the host)."""
    o = Oracle(FULL_URNS)
    for rv, qv, _ in PAIRS:
        p_host = bool(cell(rv, qv) & L.RX_HOST)
        try:
            o._regex_entity(rv, qv)
            o_host = False
        except OracleUnsupported:
            o_host = True
        except JSError:
            o_host = False
        if o_host:
            assert p_host, (rv, qv)
        elif p_host:
            assert not (rv.isascii() and qv.isascii()), (rv, qv)


# ---------------------------------------------------------------- stores from the patterns
ORG = "urn:restorecommerce:acs:model:organization.Organization"


def regex_store_cases():
    """[(doc, requests)]: one store per rule pattern — a set whose first policy holds a rule
    per namespace prefix of that pattern (plain role targets: resourceAttributesMatch's
    RegExp retry, accessController.ts:214-219, decides) and whose second policy holds the
    same rules role-scoped to organizations (checkHierarchicalScope's entity scan,
    hierarchicalScope.ts:64-101, runs the cell again with `==`).  The requests carry every
    fixture request value, half of them with an owned context resource."""
    urn = FULL_URNS
    by_pat = {}
    for rv in dict.fromkeys(rv for rv, _, _ in PAIRS if rv is not None):
        by_pat.setdefault(rv[rv.rfind(":") + 1:].split(".")[-1], []).append(rv)
    # the curated patterns (each under all 4 namespace prefixes); the fuzzed ones are cell tests
    by_pat = {k: v for k, v in by_pat.items() if len(v) >= 4}
    reqv = sorted({qv for _, qv, _ in PAIRS if qv is not None})
    reqs = []
    for k, qv in enumerate(reqv):
        for scoped in (False, True):
            r = {"target": {"subjects": [{"id": urn["role"], "value": "u"}],
                            "resources": [{"id": urn["entity"], "value": qv}],
                            "actions": [{"id": urn["actionID"], "value": urn["read"]}]},
                 "context": {"subject": {"id": "a", "role_associations": [{"role": "u", "attributes": [
                     {"id": urn["roleScopingEntity"], "value": ORG,
                      "attributes": [{"id": urn["roleScopingInstance"], "value": "o1"}]}]}],
                     "hierarchical_scopes": [{"id": "o1", "role": "u", "children": [{"id": "o2"}]}]},
                     "resources": []}}
            if scoped:
                r["target"]["resources"].append({"id": urn["resourceID"], "value": f"x{k}"})
                r["context"]["resources"] = [{"id": f"x{k}", "meta": {"owners": [
                    {"id": urn["ownerEntity"], "value": ORG,
                     "attributes": [{"id": urn["ownerInstance"], "value": ["o1", "o2", "o9"][k % 3]}]}]}}]
            reqs.append(r)
    cases = []
    for j, (pat, rvs) in enumerate(sorted(by_pat.items())):
        def rule(i, rv, scoped):
            subs = [{"id": urn["role"], "value": "u"}]
            if scoped:
                subs.append({"id": urn["roleScopingEntity"], "value": ORG})
            return {"id": f"r{i}{'s' if scoped else ''}", "effect": ["PERMIT", "DENY"][(i + j) % 2],
                    "target": {"subjects": subs, "resources": [{"id": urn["entity"], "value": rv}],
                               "actions": [{"id": urn["actionID"], "value": urn["read"]}]}}
        pols = [{"id": f"p{sc}", "combining_algorithm": DEFAULT_CAS[(j + sc) % 3]["urn"],
                 "rules": [rule(i, rv, bool(sc)) for i, rv in enumerate(rvs)]} for sc in (0, 1)]
        doc = {"policy_sets": [{"id": "s", "combining_algorithm": DEFAULT_CAS[j % 3]["urn"], "policies": pols}]}
        cases.append((doc, reqs))
    return cases


def _check_cases(run):
    """run(cs, batch) -> decision records; every non-host outcome equals the oracle's."""
    from acs_mi355x import compiler, encoder, store
    from diff_utils import gpu_outcome, oracle_outcome
    decided, kinds = 0, set()
    for doc, reqs in regex_store_cases():
        o = Oracle(FULL_URNS)
        o.load(doc)
        cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
        b = encoder.Encoder(cs).encode(reqs)
        dec = run(cs, b)
        for i, req in enumerate(reqs):
            got = gpu_outcome(cs, dec[i])
            if got[0] == "HOST":
                continue
            with warnings.catch_warnings():
                warnings.simplefilter("ignore")
                try:
                    want = oracle_outcome(o, req)
                except OracleUnsupported:
                    continue
            assert got == want, (doc["policy_sets"][0]["policies"][0]["rules"][0]["target"], i, got, want)
            decided += 1
            kinds.add(got[:2])
    return decided, kinds


def test_regex_stores_host_core():
    """The pattern stores through the CPU build of the evaluator core (no GPU)."""
    import host_core
    decided, kinds = _check_cases(host_core.is_allowed)
    assert decided >= 2000
    assert {("OK", "PERMIT"), ("OK", "DENY"), ("ERR", "SyntaxError")} <= kinds


@pytest.mark.gpu
def test_regex_stores_gpu():
    """K1 on stores built from the V8-pinned patterns matches the pinned oracle, and K2's
    reverse queries match the oracle's whatIsAllowed on a sample."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from acs_mi355x import compiler, native, results
    from diff_utils import norm_rq

    def run(cs, b):
        t = native.Tables(compiler.store_blob(cs), 0)
        try:
            return t.is_allowed(b)
        finally:
            t.close()
    decided, kinds = _check_cases(run)
    assert decided >= 2000
    assert {("OK", "PERMIT"), ("OK", "DENY"), ("ERR", "SyntaxError")} <= kinds
    from acs_mi355x import encoder, store
    for doc, reqs in regex_store_cases()[::7]:
        o = Oracle(FULL_URNS)
        o.load(doc)
        cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
        b = encoder.Encoder(cs).encode(reqs)
        t = native.Tables(compiler.store_blob(cs), 0)
        bits, obl, obl_n, out = t.what_is_allowed(b)
        t.close()
        for i, req in enumerate(reqs):
            try:
                w = ("OK", norm_rq(o.what_is_allowed(req)))
            except JSError as e:
                w = ("ERR", e.kind)
            except OracleUnsupported:
                continue
            try:
                g = ("OK", norm_rq(results.reverse_query(cs, b.overlay, bits[i], obl[i][:obl_n[i]], out[i])))
            except results.HostPathRequired:
                continue
            except results.EvaluationError as e:
                g = ("ERR", e.kind)
            assert g == w, i
