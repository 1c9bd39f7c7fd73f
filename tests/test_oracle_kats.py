"""Pin the CPU oracle against every isAllowed/whatIsAllowed assertion of the
reference's own test suite (tests/golden/kats.json, made by extract_kats.py)."""
import shutil

import pytest

from kat_utils import load_kats, oracle_for, check_asserts
from oracle.acs_oracle import NodeConditionEvaluator

KATS = load_kats()


@pytest.fixture(scope="module")
def cond():
    if shutil.which("node") is None:
        pytest.skip("node not available for rule conditions")
    ev = NodeConditionEvaluator()
    yield ev
    ev.close()


@pytest.mark.parametrize("vec", [v for v in KATS if v["op"] == "isAllowed"], ids=lambda v: v["spec"])
def test_is_allowed_kat(vec, cond):
    o = oracle_for(vec, cond)
    res = o.is_allowed(vec["request"])
    assert res["decision"] == vec["expect"]["decision"], vec["name"]
    if "status" in vec["expect"]:
        assert res["operation_status"]["code"] == vec["expect"]["status"]


@pytest.mark.parametrize("vec", [v for v in KATS if v["op"] == "whatIsAllowed"], ids=lambda v: v["spec"])
def test_what_is_allowed_kat(vec):
    o = oracle_for(vec)
    res = o.what_is_allowed(vec["request"])
    assert check_asserts(res, vec["expect"]["asserts"]) == [], vec["name"]


def test_kat_count():
    assert len([v for v in KATS if v["op"] == "isAllowed"]) >= 80
    assert len([v for v in KATS if v["op"] == "whatIsAllowed"]) >= 20
