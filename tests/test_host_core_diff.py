"""Randomised differential test: evaluator core (CPU build) vs the oracle."""
import pytest

import host_core
import randgen
from diff_utils import oracle_outcome, gpu_outcome, build, norm_rq
from oracle.jsval import OracleUnsupported, JSError
from acs_mi355x import encoder, results


@pytest.mark.parametrize("seed", range(600))
def test_is_allowed_diff(seed):
    urns, doc, reqs = randgen.rand_case(seed)
    o, cs = build(urns, doc)
    b = encoder.Encoder(cs).encode(reqs)
    dec = host_core.is_allowed(cs, b)
    for i, req in enumerate(reqs):
        got = gpu_outcome(cs, dec[i])
        if got[0] == "HOST":
            continue
        try:
            want = oracle_outcome(o, req)
        except OracleUnsupported:
            continue
        assert got == want, (seed, i, b.host_reasons.get(i))


@pytest.mark.parametrize("seed", range(150))
def test_what_is_allowed_diff(seed):
    urns, doc, reqs = randgen.rand_case(seed)
    o, cs = build(urns, doc)
    b = encoder.Encoder(cs).encode(reqs)
    bits, obl, obl_n, out = host_core.what_is_allowed(cs, b)
    for i, req in enumerate(reqs):
        try:
            want = ("OK", norm_rq(o.what_is_allowed(req)))
        except JSError as e:
            want = ("ERR", e.kind)
        except OracleUnsupported:
            continue
        try:
            got = ("OK", norm_rq(results.reverse_query(cs, b.overlay, bits[i], obl[i][:obl_n[i]], out[i])))
        except results.HostPathRequired:
            continue
        except results.EvaluationError as e:
            got = ("ERR", e.kind)
        assert got == want, (seed, i)
