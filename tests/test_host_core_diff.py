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


def test_what_is_allowed_overflow_pass_host():
    """Obligation-only pass (CPU build of the core): requests whose log exceeded OBL_MAX get
    their whole maskedProperty log, K2's truncated log is its prefix, and the reverse query
    built from it equals the oracle's; cap 70 exercises the exact-count re-run."""
    import numpy as np
    from acs_mi355x import compiler, store, synth, layout as L
    from oracle.acs_oracle import Oracle, FULL_URNS, DEFAULT_CAS
    doc = synth.c3_store()
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 2_000, "c3")
    t = host_core.Tables(compiler.store_blob(cs))
    bits, obl, obl_n, out = t.what_is_allowed(sb.batch)
    over = np.flatnonzero((out["flags"] & L.OF_OBL_OVERFLOW) != 0)
    assert len(over) > 0
    logs = t.resolve_overflow(sb.batch, out.copy(), cap=70)
    assert sorted(logs) == over.tolist()
    assert max(len(v) for v in logs.values()) > 70
    for i in over:
        assert len(logs[i]) > L.OBL_MAX and np.array_equal(logs[i][:L.OBL_MAX], obl[i])
    o = Oracle(FULL_URNS)
    o.load(doc)
    rec = out.copy()
    rec["flags"][over] &= np.uint8(~L.OF_OBL_OVERFLOW & 0xFF)
    for i in over[:4]:
        got = norm_rq(results.reverse_query(cs, sb.batch.overlay, bits[i], logs[i], rec[i]))
        assert got == norm_rq(o.what_is_allowed(sb.decode(int(i)))), int(i)
