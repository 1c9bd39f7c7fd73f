"""c1: the seed_data + fixtures store with 10k fixture-vocabulary requests (BASELINE.json
configs[0]) — the product against the oracle, on the CPU build of the core and on the GPU."""
import json

import numpy as np
import pytest

import host_core
from c1_utils import c1_requests, c1_store
from diff_utils import gpu_outcome, oracle_from_store, oracle_outcome
from oracle.acs_oracle import DEFAULT_CAS, FULL_URNS
from oracle.jsval import OracleUnsupported
from acs_mi355x import compiler, encoder
from acs_mi355x.codec import NativeCodec

N = 10_000


def test_seed_data_loads_into_the_store():
    m = c1_store()
    assert "global_policy_set_id" in m
    ps = m["global_policy_set_id"]
    assert list(ps["combinables"]) == ["super_admin_policy_id"]
    assert list(ps["combinables"]["super_admin_policy_id"]["combinables"]) == ["super_admin_rule_id"]
    cs = compiler.compile_store(m, FULL_URNS, DEFAULT_CAS)
    assert cs.n_sets == len(m) and cs.n_rules > 50
    # the seed alone: its SuperAdmin rule permits anything for its role
    m = {"global_policy_set_id": ps}
    cs = compiler.compile_store(m, FULL_URNS, DEFAULT_CAS)
    req = {"target": {"subjects": [{"id": FULL_URNS["role"], "value": "superadministrator-r-id"}],
                      "resources": [{"id": FULL_URNS["entity"], "value": "urn:x:y.Z"}],
                      "actions": [{"id": FULL_URNS["actionID"], "value": FULL_URNS["read"]}]},
           "context": {"subject": {"id": "root", "role_associations": [{"role": "superadministrator-r-id"}],
                                   "hierarchical_scopes": []}, "resources": []}}
    o = oracle_from_store(FULL_URNS, m)
    assert oracle_outcome(o, req)[:2] == ("OK", "PERMIT")
    d = host_core.is_allowed(cs, encoder.Encoder(cs).encode([req]))
    assert gpu_outcome(cs, d[0]) == oracle_outcome(o, req)


def _compare(cs, o, reqs, dec):
    checked = host = 0
    mix = {}
    for i, req in enumerate(reqs):
        got = gpu_outcome(cs, dec[i])
        if got[0] == "HOST":
            host += 1
            continue
        try:
            want = oracle_outcome(o, req)
        except OracleUnsupported:
            continue
        assert got == want, (i, json.dumps(req)[:400])
        mix[got[1]] = mix.get(got[1], 0) + 1
        checked += 1
    return checked, host, mix


def test_c1_cpu_core_matches_oracle():
    m = c1_store()
    cs = compiler.compile_store(m, FULL_URNS, DEFAULT_CAS)
    reqs = c1_requests(N, seed=1)
    b = encoder.Encoder(cs).encode(reqs)
    dec = host_core.is_allowed(cs, b)
    # the native codec packs the same JSON to the same decisions
    nb = NativeCodec(compiler.store_blob(cs)).encode(json.dumps(reqs).encode(), threads=4)
    assert np.array_equal(host_core.is_allowed(cs, nb).view(np.uint64), dec.view(np.uint64))
    checked, host, mix = _compare(cs, oracle_from_store(FULL_URNS, m), reqs, dec)
    assert checked >= 0.9 * N and host <= 0.05 * N
    assert len(mix) >= 3  # PERMIT / DENY / INDETERMINATE (and errors) all occur


@pytest.mark.gpu
def test_c1_gpu_matches_oracle():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from acs_mi355x import native
    m = c1_store()
    cs = compiler.compile_store(m, FULL_URNS, DEFAULT_CAS)
    reqs = c1_requests(N, seed=2)
    blob = compiler.store_blob(cs)
    t = native.Tables(blob, 0)
    nb = NativeCodec(blob).encode(json.dumps(reqs).encode(), threads=4)
    dec = t.is_allowed(nb)
    assert np.array_equal(dec.view(np.uint64), t.is_allowed(encoder.Encoder(cs).encode(reqs)).view(np.uint64))
    t.close()
    checked, host, _ = _compare(cs, oracle_from_store(FULL_URNS, m), reqs, dec)
    assert checked >= 0.9 * N
