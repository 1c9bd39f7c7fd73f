"""c3-adverse (SURVEY §8(d) robustness): the c3 store with condition rules in its early sets, a
null policy entry behind a rare set target, and ACL-bearing context resources on 10 % of the
requests — every early stop of the kernel (NF_CLEAN_BELOW, the loop cuts) is disabled below the
top sets.  The product (host core here, K1 on the GPU) against the oracles:
  * a request that reaches a condition rule goes to the host (OF_HOST_COND) exactly when the
    C++ oracle, walking the sets forward, meets that condition first (it reports UNSUPPORTED:
    conditions need JS eval, utils.ts:47-56);
  * a request reaching the null policy rejects with the TypeError of accessController.ts:138;
  * every other outcome (ACL paths included, verifyACL.ts:37-251) is identical.
Parity is pinned by the oracles as elsewhere; no reference fixture holds this workload."""
import numpy as np
import pytest

from diff_utils import gpu_outcome
from oracle import acs_oracle_c
from oracle.acs_oracle import DEFAULT_CAS, FULL_URNS
from acs_mi355x import compiler, encoder, store, synth, layout as L
from acs_mi355x.codec import NativeCodec
import host_core


@pytest.fixture(scope="module")
def adverse():
    acs_oracle_c.build()
    doc = synth.c3_adverse_store()
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 3000, "c3", seed=41, tree=synth.OrgTree(fanout=3, depth=5), acl=0.1)
    return doc, cs, sb


def compare(cs, doc, sb, dec, idx):
    co = acs_oracle_c.COracle(FULL_URNS, DEFAULT_CAS, doc)
    reqs = [sb.decode(int(i)) for i in idx]
    counts = {"ok": 0, "host_cond": 0, "err": 0}
    for i, want in zip(idx, co.outcomes(reqs, threads=4)):
        got = gpu_outcome(cs, dec[i])
        if want[0] == "UNSUPPORTED":  # the oracle met a rule condition
            assert dec[i]["flags"] & L.OF_HOST_COND, (int(i), got)
            counts["host_cond"] += 1
            continue
        assert not dec[i]["flags"] & L.OF_HOST_COND, (int(i), want)
        assert got == want, (int(i), got, want)
        counts["err" if want[0] == "ERR" else "ok"] += 1
    co.close()
    return counts


def test_adverse_store_flags(adverse):
    """No set below the null policy / the condition sets is clean; the top sets are."""
    _, cs, _ = adverse
    clean = (cs.sets["nflags"] & L.NF_CLEAN_BELOW) != 0
    assert not clean[8:].any() and clean[:1].all()
    assert ((cs.pols["nflags"] & L.NF_NULL) != 0).sum() == 1
    assert 45 <= ((cs.rules["nflags"] & L.NF_HAS_CONDITION) != 0).sum() <= 50  # minus any in the null policy


def test_adverse_host_core_vs_oracle(adverse):
    doc, cs, sb = adverse
    b = encoder.Encoder(cs).encode([sb.decode(i) for i in range(sb.batch.n)])
    acl = int((sb.draws["acl"] >= 0).sum())
    assert acl > 200 and not b.host_reasons
    dec = host_core.is_allowed(cs, b)
    c = compare(cs, doc, sb, dec, np.arange(b.n))
    assert c["host_cond"] > 0 and c["ok"] > 2000, c
    # the native codec's batch of the same JSON text decides identically
    codec = NativeCodec(compiler.store_blob(cs))
    for k, v in sb.hrs_forests().items():
        codec.set_subject_scopes(k, v)
    nb = codec.encode(sb.json_text(), threads=3)
    assert np.array_equal(host_core.is_allowed(cs, nb).view(np.uint64), dec.view(np.uint64))


def test_adverse_event_index_changes_no_record(adverse, monkeypatch):
    """The event index (acs_eval.h set_may_raise: below the deciding set, skip a set none of whose
    condition rules is a candidate and that holds no null policy / invalid algorithm) gives the
    records of the walk without it, over every filter form (class rows, role factor, none)."""
    from acs_mi355x import candidates
    _, cs, sb = adverse
    reqs = [sb.decode(i) for i in range(sb.batch.n)]
    for level in (None, "entity+action", "entity"):
        monkeypatch.setattr(candidates, "FORCE_LEVEL", level)
        b = encoder.Encoder(cs).encode(reqs)
        with_ix = host_core.is_allowed(cs, b).view(np.uint64)
        monkeypatch.setenv("ACS_HOST_NO_EV_INDEX", "1")
        without = host_core.is_allowed(cs, b).view(np.uint64)
        monkeypatch.delenv("ACS_HOST_NO_EV_INDEX")
        assert np.array_equal(with_ix, without), level
    b.cand = None
    b.role_key = b.role_bits = None
    b.lines["cls2"] = 0
    with_ix = host_core.is_allowed(cs, b).view(np.uint64)
    monkeypatch.setenv("ACS_HOST_NO_EV_INDEX", "1")
    assert np.array_equal(with_ix, host_core.is_allowed(cs, b).view(np.uint64))


def test_acl_none_changes_no_record(adverse):
    """ACL_NONE (the encoders' rule-independent verifyACL veto, acs_layout.h): both encoders mark
    the same requests, some of them, and turning the state back to ACL_CONTINUE (verifyACL per
    rule, every rule evaluated) gives the same records."""
    _, cs, sb = adverse
    reqs = [sb.decode(i) for i in range(sb.batch.n)]
    pb = encoder.Encoder(cs).encode(reqs)
    codec = NativeCodec(compiler.store_blob(cs))
    for k, v in sb.hrs_forests().items():
        codec.set_subject_scopes(k, v)
    nb = codec.encode(sb.json_text(), threads=3)
    st_p = (pb.hdr["flags"] >> L.RQ_ACL_SHIFT) & 3
    st_n = (nb.lines["h"]["flags"] >> L.RQ_ACL_SHIFT) & 3
    assert np.array_equal(st_p, st_n)
    none = st_p == L.ACL_NONE
    assert none.sum() > 50, int(none.sum())
    assert pb.hints == nb.hints == L.HINT_ACL_NONE  # K1 instantiates the ACL_NONE skips
    want = host_core.is_allowed(cs, pb).view(np.uint64).copy()
    pb.hdr["flags"] = np.where(none, pb.hdr["flags"] & ~np.uint32(3 << L.RQ_ACL_SHIFT), pb.hdr["flags"])
    pb.lines["h"]["flags"] = pb.hdr["flags"]
    assert np.array_equal(host_core.is_allowed(cs, pb).view(np.uint64), want)


@pytest.mark.gpu
def test_adverse_gpu(adverse):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from acs_mi355x import native
    from acs_mi355x.device import DeviceBatch, is_allowed_device, decisions_from_tensor
    doc, cs, sb = adverse
    codec = NativeCodec(compiler.store_blob(cs))
    for k, v in sb.hrs_forests().items():
        codec.set_subject_scopes(k, v)
    nb = codec.encode(sb.json_text(), threads=4)
    t = native.Tables(compiler.store_blob(cs), 0)
    db = DeviceBatch(nb, 0)
    assert db.struct.hints == L.HINT_ACL_NONE
    dec = decisions_from_tensor(is_allowed_device(t, db))
    assert np.array_equal(np.ascontiguousarray(dec).view(np.uint64), host_core.is_allowed(cs, nb).view(np.uint64))
    db.struct.hints = 0  # the plain K1 (no ACL_NONE skips) decides the same
    plain = decisions_from_tensor(is_allowed_device(t, db))
    assert np.array_equal(np.ascontiguousarray(plain).view(np.uint64), np.ascontiguousarray(dec).view(np.uint64))
    c = compare(cs, doc, sb, dec, np.arange(nb.n))
    assert c["host_cond"] > 0 and c["ok"] > 2000, c
    t.close()
