"""The C++ oracle (oracle/acs_oracle.cpp) against the golden vectors of the reference's
test suite and against the Python oracle on randomised and synthetic workloads."""
import numpy as np
import pytest

import randgen
from diff_utils import oracle_outcome
from kat_utils import load_kats, load_fixture, urns_for
from oracle import acs_oracle_c
from oracle.acs_oracle import DEFAULT_CAS, FULL_URNS, Oracle
from oracle.jsval import OracleUnsupported
from acs_mi355x import compiler, store, synth

KATS = load_kats()


@pytest.fixture(scope="module", autouse=True)
def built():
    acs_oracle_c.build()


def test_kats_is_allowed():
    by_fx = {}
    for v in KATS:
        if v["op"] == "isAllowed":
            by_fx.setdefault((v["fixture"], v["urns"]), []).append(v)
    checked = 0
    for (fx, _), vecs in by_fx.items():
        o = acs_oracle_c.COracle(urns_for(vecs[0]), DEFAULT_CAS, load_fixture(fx))
        for v, got in zip(vecs, o.outcomes([v["request"] for v in vecs])):
            if got[0] == "UNSUPPORTED":  # rule conditions need JS eval (Python oracle + node)
                assert fx == "conditions.yml", v["spec"]
                continue
            assert got[0] == "OK" and got[1] == v["expect"]["decision"], (v["spec"], got)
            if "status" in v["expect"]:
                assert got[3] == v["expect"]["status"]
            checked += 1
    assert checked >= 70


@pytest.mark.parametrize("seed", range(0, 600, 20))
def test_random_vs_python_oracle(seed):
    agree = 0
    for s in range(seed, seed + 20):
        urns, doc, reqs = randgen.rand_case(s)
        po = Oracle(urns=urns)
        po.load(doc)
        co = acs_oracle_c.COracle(urns, DEFAULT_CAS, doc)
        for req, got in zip(reqs, co.outcomes(reqs, threads=2)):
            try:
                want = oracle_outcome(po, req)
            except OracleUnsupported:
                continue
            if got[0] == "UNSUPPORTED":
                continue
            assert got == want, (s, req)
            agree += 1
    assert agree > 100


@pytest.mark.parametrize("kind", ["c2", "c3"])
def test_synthetic_vs_python_oracle(kind):
    doc = synth.c2_store() if kind == "c2" else synth.c3_store()
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 20_000, kind)
    idx = np.random.default_rng(1).choice(sb.batch.n, size=60, replace=False)
    reqs = [sb.decode(int(i)) for i in idx]
    po = Oracle(FULL_URNS)
    po.load(doc)
    co = acs_oracle_c.COracle(FULL_URNS, DEFAULT_CAS, doc)
    got = co.outcomes(reqs, threads=4)
    assert got == [oracle_outcome(po, r) for r in reqs]


# ---------------------------------------------------------------- whatIsAllowed
def _wia_python(po, req):
    from diff_utils import norm_rq
    from oracle.jsval import JSError
    try:
        return norm_rq(po.what_is_allowed(req))
    except JSError as e:
        return ("ERR", e.kind)


def test_kats_what_is_allowed():
    """The C++ whatIsAllowed (rule sets + maskedProperty pushes) meets every whatIsAllowed
    golden vector of the reference's specs and equals the Python oracle on them."""
    from diff_utils import compact_reverse_query
    from kat_utils import check_asserts
    by_fx = {}
    for v in KATS:
        if v["op"] == "whatIsAllowed":
            by_fx.setdefault((v["fixture"], v["urns"]), []).append(v)
    checked = 0
    for (fx, _), vecs in by_fx.items():
        doc = load_fixture(fx)
        urns = urns_for(vecs[0])
        cs = compiler.compile_store(store.populate(doc), urns, DEFAULT_CAS)
        co = acs_oracle_c.COracle(urns, DEFAULT_CAS, doc)
        po = Oracle(urns=urns)
        po.load(doc)
        res, _ = co.what_is_allowed([v["request"] for v in vecs])
        for v, c in zip(vecs, res):
            got = compact_reverse_query(cs, c)
            assert got is not None, v["spec"]
            assert check_asserts(got, v["expect"]["asserts"]) == [], v["spec"]
            assert got == _wia_python(po, v["request"]), v["spec"]
            checked += 1
    assert checked >= 19


@pytest.mark.parametrize("seed", range(0, 600, 30))
def test_random_what_is_allowed_vs_python_oracle(seed):
    from diff_utils import compact_reverse_query
    from acs_mi355x.jsops import Unsupported
    agree = 0
    for s in range(seed, seed + 30):
        urns, doc, reqs = randgen.rand_case(s)
        try:
            cs = compiler.compile_store(store.populate(doc), urns, DEFAULT_CAS)
        except Unsupported:
            continue
        po = Oracle(urns=urns)
        po.load(doc)
        co = acs_oracle_c.COracle(urns, DEFAULT_CAS, doc)
        res, _ = co.what_is_allowed(reqs, threads=2)
        for req, c in zip(reqs, res):
            got = compact_reverse_query(cs, c)
            if got is None:
                continue
            try:
                want = _wia_python(po, req)
            except OracleUnsupported:
                continue
            assert got == want, (s, req)
            agree += 1
    assert agree > 150
