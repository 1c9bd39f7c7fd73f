"""GPU parity tests: the HIP path (through the C ABI) against the CPU oracles.

* every golden vector (isAllowed + whatIsAllowed) of the reference test suite,
* randomised stores/requests that exercise the reference's quirks,
* c2 / c3 synthetic configurations: the WHOLE batch vs the C++ oracle (and a sample vs
  the Python oracle); c4 whatIsAllowed vs the Python oracle; c5 (1M rules) and the
  large-store filter modes on oracle samples, plus the CPU build of the same core as a
  full-batch consistency check,
* rule sharding (2/3/8 shards, c3 and c5 scale) vs an unsharded evaluation,
* edge shapes: empty batch, ragged sizes, maximum attribute counts, device API.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

from kat_utils import load_kats, load_fixture, urns_for, check_asserts  # noqa: E402
import randgen  # noqa: E402
import host_core  # noqa: E402
from diff_utils import oracle_outcome, gpu_outcome, build, norm_rq  # noqa: E402
from oracle.acs_oracle import Oracle, FULL_URNS, DEFAULT_CAS  # noqa: E402
from oracle.jsval import OracleUnsupported, JSError  # noqa: E402
from acs_mi355x import store, compiler, encoder, results, native, shard, synth, layout as L  # noqa: E402
from acs_mi355x.device import DeviceBatch, is_allowed_device, decisions_from_tensor  # noqa: E402

KATS = load_kats()


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    native.load()


def gpu_tables(cs):
    return native.Tables(compiler.store_blob(cs), 0)


def test_kats_is_allowed_gpu():
    by_fx = {}
    for v in KATS:
        by_fx.setdefault((v["fixture"], v["urns"]), []).append(v)
    checked = 0
    for (fx, u), vecs in by_fx.items():
        cs = compiler.compile_store(store.populate(load_fixture(fx)), urns_for(vecs[0]), DEFAULT_CAS)
        t = gpu_tables(cs)
        ia = [v for v in vecs if v["op"] == "isAllowed"]
        if ia:
            b = encoder.Encoder(cs).encode([v["request"] for v in ia])
            dec = t.is_allowed(b)
            for v, d in zip(ia, dec):
                oc = results.outcome(cs, d)
                if oc[0] == "HOST" and fx == "conditions.yml":
                    continue
                assert oc[0] == "OK" and oc[1] == v["expect"]["decision"], (v["spec"], oc)
                checked += 1
        wa = [v for v in vecs if v["op"] == "whatIsAllowed"]
        if wa:
            b = encoder.Encoder(cs).encode([v["request"] for v in wa])
            bits, obl, obl_n, out = t.what_is_allowed(b)
            for k, v in enumerate(wa):
                rq = results.reverse_query(cs, b.overlay, bits[k], obl[k][:obl_n[k]], out[k])
                assert check_asserts(rq, v["expect"]["asserts"]) == [], v["spec"]
                checked += 1
        t.close()
    assert checked >= 100


@pytest.mark.parametrize("seed", range(0, 400, 4))
def test_random_diff_gpu(seed):
    for s in range(seed, seed + 4):
        urns, doc, reqs = randgen.rand_case(s)
        o, cs = build(urns, doc)
        b = encoder.Encoder(cs).encode(reqs)
        t = gpu_tables(cs)
        dec = t.is_allowed(b)
        bits, obl, obl_n, out = t.what_is_allowed(b)
        t.close()
        for i, req in enumerate(reqs):
            got = gpu_outcome(cs, dec[i])
            if got[0] != "HOST":
                try:
                    assert got == oracle_outcome(o, req), (s, i)
                except OracleUnsupported:
                    pass
            try:
                want = ("OK", norm_rq(o.what_is_allowed(req)))
            except JSError as e:
                want = ("ERR", e.kind)
            except OracleUnsupported:
                continue
            try:
                g = ("OK", norm_rq(results.reverse_query(cs, b.overlay, bits[i], obl[i][:obl_n[i]], out[i])))
            except results.HostPathRequired:
                continue
            except results.EvaluationError as e:
                g = ("ERR", e.kind)
            assert g == want, (s, i)


def _synth(kind, n):
    doc = synth.c2_store() if kind == "c2" else synth.c3_store()
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    return doc, cs, synth.requests(cs, n, kind)


def coracle_check(doc, cs, sb, dec, idx, chunk=10_000):
    """The requests idx of a synthetic batch, decoded to the reference's JSON shape, re-decided
    by the C++ oracle (16 threads; HR trees shared via placeholders): every outcome must
    equal the GPU's record.  Returns the number compared."""
    from oracle import acs_oracle_c
    co = acs_oracle_c.COracle(FULL_URNS, DEFAULT_CAS, doc)
    checked = 0
    try:
        for k in range(0, len(idx), chunk):
            part = idx[k:k + chunk]
            sh = synth.SharedValues()
            out, _ = co.raw([sb.decode(int(i), sh) for i in part], 16, shared=sh.values)
            for i, r in zip(part, out):
                want = acs_oracle_c.outcome(r)
                assert want[0] != "UNSUPPORTED", int(i)
                assert gpu_outcome(cs, dec[i]) == want, int(i)
                checked += 1
    finally:
        co.close()
    return checked


@pytest.mark.parametrize("kind,n,sample", [("c2", 300_000, 200), ("c3", 60_000, 40)])
def test_synthetic_config_gpu(kind, n, sample):
    doc, cs, sb = _synth(kind, n)
    t = gpu_tables(cs)
    dec = t.is_allowed(sb.batch)
    # the whole batch vs the C++ oracle (the reference's algorithm over the JSON requests)
    assert coracle_check(doc, cs, sb, dec, np.arange(n)) == n
    # full batch: identical records to the CPU build of the same core
    ref = host_core.is_allowed(cs, sb.batch)
    assert np.array_equal(dec.view(np.uint64), ref.view(np.uint64))
    # sample vs the Python oracle on the decoded JSON requests
    o = Oracle(FULL_URNS)
    o.load(doc)
    idx = np.random.default_rng(7).choice(n, size=sample, replace=False)
    for i in idx:
        assert gpu_outcome(cs, dec[i]) == oracle_outcome(o, sb.decode(int(i))), int(i)
    # decision mix is non-trivial
    codes = np.bincount(dec["decision"], minlength=7)
    assert codes[L.DEC_PERMIT] > 0 and codes[L.DEC_DENY] > 0
    t.close()


@pytest.mark.parametrize("level", [None, "composed"])
def test_c3_two_role_associations_gpu(level, monkeypatch):
    """c3 as SURVEY §8(d) specifies it: 1-2 org-scoped role associations per request (half with
    two, each with its own HR subtree root).  With composed class rows (two per-role rows the
    kernel ORs, ReqLine.cls2) as with joint rows, the WHOLE batch equals the C++ oracle
    (hierarchicalScope.ts:155-245 over several grants, accessController.ts:793-823), through the
    host-buffer and the device-resident entry points, with the encoder's coherence order and
    with the device sort; whatIsAllowed rows and obligation logs equal the CPU build's."""
    from acs_mi355x import candidates
    if level:
        monkeypatch.setattr(candidates, "FORCE_LEVEL", level)
    doc = synth.c3_store()
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    n = 60_000
    sb = synth.requests(cs, n, "c3", second_role=0.5)
    two = sb.batch.hdr["nroles"] == 2
    assert 0.4 < two.mean() < 0.6
    if level:
        assert (sb.batch.lines["cls2"] != 0).mean() > 0.3
    t = gpu_tables(cs)
    dec = t.is_allowed(sb.batch)
    ref = host_core.is_allowed(cs, sb.batch)
    assert np.array_equal(dec.view(np.uint64), ref.view(np.uint64))
    db = DeviceBatch(sb.batch, 0, compact=True)
    dev = decisions_from_tensor(is_allowed_device(t, db))
    assert np.array_equal(dev.view(np.uint64), ref.view(np.uint64))
    perm, sb.batch.perm = sb.batch.perm, None  # the device's own coherence sort
    dev2 = decisions_from_tensor(is_allowed_device(t, DeviceBatch(sb.batch, 0, compact=True)))
    sb.batch.perm = perm
    assert np.array_equal(dev2.view(np.uint64), ref.view(np.uint64))
    assert coracle_check(doc, cs, sb, dec, np.arange(n)) == n
    codes = np.bincount(dec["decision"][two], minlength=7)
    assert codes[L.DEC_PERMIT] > 0 and codes[L.DEC_DENY] > 0
    m = 6000  # whatIsAllowed on a slice of the same requests
    sub = synth.requests(cs, m, "c3", second_role=0.5)
    bits, obl, obl_n, out = t.what_is_allowed(sub.batch)
    rbits, robl, robl_n, rout = host_core.what_is_allowed(cs, sub.batch)
    assert np.array_equal(bits, rbits) and np.array_equal(obl_n, robl_n)
    assert np.array_equal(out.view(np.uint64), rout.view(np.uint64))
    for i in range(m):
        assert np.array_equal(obl[i, :min(obl_n[i], L.OBL_MAX)], robl[i, :min(robl_n[i], L.OBL_MAX)]), i
    t.close()


def test_large_store_class_list_gpu():
    """Rows longer than the LDS union (W > 1024 words): waves of up to 4 classes use row
    pointers, mixed waves the LDS class list — both bit-identical to the CPU build."""
    doc = synth.c5_store(n_sets=60)  # 60 sets x 10 x 100 = 60k rules, W ~ 1.9k words
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 30_000, "c3", tree=synth.OrgTree(fanout=4, depth=5))
    assert sb.batch.cand.shape[1] > 1024
    t = gpu_tables(cs)
    dec = t.is_allowed(sb.batch)
    t.close()
    ref = host_core.is_allowed(cs, sb.batch)
    assert np.array_equal(dec.view(np.uint64), ref.view(np.uint64))
    codes = np.bincount(dec["decision"], minlength=7)
    assert codes[L.DEC_PERMIT] > 0 and codes[L.DEC_DENY] > 0
    idx = np.random.default_rng(11).choice(sb.batch.n, size=300, replace=False)
    assert coracle_check(doc, cs, sb, dec, idx) == 300


@pytest.mark.parametrize("kind", ["c3", "c5_small"])
def test_role_factor_gpu(kind, monkeypatch):
    """Class rows keyed by (entity, action) AND-ed with the role factor (the large-store
    filter): in the LDS union (c3, W <= 1024) and in the row-pointer / LDS-list modes
    (c5_small, W > 1024) the records equal the CPU build's."""
    from acs_mi355x import candidates
    monkeypatch.setattr(candidates, "FORCE_LEVEL", "entity+action")
    doc = synth.c3_store() if kind == "c3" else synth.c5_store(n_sets=60)
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 40_000, "c3", tree=synth.OrgTree(fanout=4, depth=5))
    assert sb.batch.role_key is not None
    t = gpu_tables(cs)
    dec = t.is_allowed(sb.batch)
    db = DeviceBatch(sb.batch, 0)
    dev = decisions_from_tensor(is_allowed_device(t, db))
    t.close()
    ref = host_core.is_allowed(cs, sb.batch)
    assert np.array_equal(dec.view(np.uint64), ref.view(np.uint64))
    assert np.array_equal(dev.view(np.uint64), ref.view(np.uint64))
    idx = np.random.default_rng(12).choice(sb.batch.n, size=300, replace=False)
    assert coracle_check(doc, cs, sb, dev, idx) == 300


def test_what_is_allowed_c4_gpu():
    """c4-shaped whatIsAllowed (c3 store, 1-2 role associations): the whole batch equals the CPU
    build of the core, and 1,500 queries (every overflowed one after the obligation pass, and a
    random sample of the rest: BASELINE.md's >= 1 % many times over) equal the C++ oracle's
    whatIsAllowed — rule sets bit-exact, maskedProperty pushes in order."""
    from oracle import acs_oracle_c
    from diff_utils import gpu_reverse_query_compact
    doc, cs, sb = _synth("c3", 8_000)
    t = gpu_tables(cs)
    bits, obl, obl_n, out = t.what_is_allowed(sb.batch)
    rbits, robl, robl_n, rout = host_core.what_is_allowed(cs, sb.batch)
    assert np.array_equal(bits, rbits) and np.array_equal(obl_n, robl_n)
    over = np.flatnonzero((out["flags"] & L.OF_OBL_OVERFLOW) != 0)
    logs = t.resolve_overflow(sb.batch, out)  # clears OF_OBL_OVERFLOW on the resolved records
    assert sorted(logs) == over.tolist()
    rng = np.random.default_rng(3)
    rest = np.setdiff1d(np.arange(sb.batch.n), over)
    idx = np.concatenate([over, rng.choice(rest, size=1500 - len(over), replace=False)])
    co = acs_oracle_c.COracle(FULL_URNS, DEFAULT_CAS, doc)
    checked = 0
    try:
        for k in range(0, len(idx), 500):
            part = idx[k:k + 500]
            sh = synth.SharedValues()
            res, _ = co.what_is_allowed([sb.decode(int(i), sh) for i in part], 16, shared=sh.values)
            for i, want in zip(part, res):
                log = logs[i] if i in logs else obl[i][:obl_n[i]]
                got = gpu_reverse_query_compact(cs, sb.batch.overlay, bits[i], log, out[i])
                assert want["k"] != 2 and got is not None, int(i)
                assert got == want, int(i)
                checked += 1
    finally:
        co.close()
    assert checked == 1500
    t.close()


@pytest.mark.parametrize("cap", [1024, 70])
def test_what_is_allowed_overflow_pass_gpu(cap):
    """Requests with > OBL_MAX maskedProperty pushes: the obligation-only pass returns the
    whole log (its first OBL_MAX entries are K2's log), and the reverse query built from it
    equals the oracle's (rule sets and obligations).  cap=70 forces the exact-count re-run."""
    doc, cs, sb = _synth("c3", 8_000)
    t = gpu_tables(cs)
    bits, obl, obl_n, out = t.what_is_allowed(sb.batch)
    over = np.flatnonzero((out["flags"] & L.OF_OBL_OVERFLOW) != 0)
    assert len(over) > 0
    logs = t.resolve_overflow(sb.batch, out, cap=cap)
    assert sorted(logs) == over.tolist()
    assert not (out["flags"] & L.OF_OBL_OVERFLOW).any()
    for i in over:
        assert len(logs[i]) > L.OBL_MAX and np.array_equal(logs[i][:L.OBL_MAX], obl[i])
    if cap < 1024:  # some logs needed the exact-count re-run
        assert max(len(v) for v in logs.values()) > cap
    # the device form on the same indices agrees with the host form, for 1 and 5 set ranges
    import ctypes as C
    db = DeviceBatch(sb.batch, 0)
    didx = torch.from_numpy(over.astype(np.int32)).cuda()
    m, big = len(over), max(len(v) for v in logs.values())
    for chunks in (1, 5):
        dobl = torch.zeros((chunks, m, big, 2), dtype=torch.int32, device="cuda")
        dn = torch.zeros((chunks, m), dtype=torch.int32, device="cuda")
        rc = t.lib.acs_what_is_allowed_obl_device(t.h, C.byref(db.struct), didx.data_ptr(), m, chunks, big,
                                                   dobl.data_ptr(), dn.data_ptr(), None)
        assert rc == 0, native.last_error(t.lib)
        torch.cuda.synchronize()
        joined = native.join_chunk_logs(dobl.cpu().numpy().view(np.uint32), dn.cpu().numpy().view(np.uint32), big)
        for k, i in enumerate(over):
            assert np.array_equal(joined[k], logs[i])
    o = Oracle(FULL_URNS)
    o.load(doc)
    for i in np.random.default_rng(5).choice(over, size=min(6, len(over)), replace=False):
        got = norm_rq(results.reverse_query(cs, sb.batch.overlay, bits[i], logs[i], out[i]))
        assert got == norm_rq(o.what_is_allowed(sb.decode(int(i)))), int(i)
    # out-of-range indices: rejected by the host form, marked by the device form
    with pytest.raises(RuntimeError):
        t.what_is_allowed_obl(sb.batch, np.array([sb.batch.n], np.uint32), 8)
    bad = torch.tensor([sb.batch.n, int(over[0])], dtype=torch.int32, device="cuda")
    bn = torch.zeros((1, 2), dtype=torch.int32, device="cuda")
    bo = torch.zeros((1, 2, big, 2), dtype=torch.int32, device="cuda")
    assert t.lib.acs_what_is_allowed_obl_device(t.h, C.byref(db.struct), bad.data_ptr(), 2, 1, big, bo.data_ptr(),
                                                 bn.data_ptr(), None) == 0
    torch.cuda.synchronize()
    bn = bn.cpu().numpy().view(np.uint32)
    assert bn[0, 0] == 0xFFFFFFFF and bn[0, 1] == len(logs[int(over[0])])
    t.close()


@pytest.mark.parametrize("compact", [True, False])
def test_overflow_resolution_on_device_gpu(compact):
    """The device path's overflow bookkeeping (acs_overflow_index_device /
    acs_overflow_repass_device, no torch kernels): the index list is the overflowed
    requests, every one once, in a deterministic order; cap=70 forces the exact-count
    re-pass, whose list and cap equal a numpy restatement; the joined logs equal the host
    form's."""
    import ctypes as C
    from acs_mi355x.device import resolve_overflow_device, overflow_logs, what_is_allowed_device
    doc, cs, sb = _synth("c3", 8_000)
    t = gpu_tables(cs)
    _, _, _, out = t.what_is_allowed(sb.batch)
    want = t.resolve_overflow(sb.batch, out.copy(), cap=1024)
    db = DeviceBatch(sb.batch, 0, compact=compact)
    bufs = what_is_allowed_device(t, db)
    passes = resolve_overflow_device(t, db, bufs, cap=70, chunks=4)
    assert len(passes) >= 2
    idx0 = passes[0][0].cpu().numpy()
    assert sorted(idx0.tolist()) == sorted(want)
    again = resolve_overflow_device(t, db, bufs, cap=70, chunks=4)
    assert np.array_equal(again[0][0].cpu().numpy(), idx0)  # deterministic order
    for (idx, cap, obl, obl_n), nxt in zip(passes, passes[1:] + [None]):
        n = obl_n.cpu().numpy().view(np.uint32).astype(np.int64)
        more = (n > cap).any(axis=0)
        exp = idx.cpu().numpy()[more]
        if nxt is None:
            assert not more.any()
        else:
            assert np.array_equal(nxt[0].cpu().numpy(), exp) and nxt[1] == int(n[:, more].max())
    logs = overflow_logs(passes)
    assert sorted(logs) == sorted(want)
    for i, lg in want.items():
        assert np.array_equal(logs[i], lg), i
    # none overflowed: an empty list and no pass
    clean = bufs[3].clone()
    clean[:, 2] &= ~L.OF_OBL_OVERFLOW
    assert resolve_overflow_device(t, db, (bufs[0], bufs[1], bufs[2], clean)) == []
    m = C.c_size_t(7)
    idx = torch.empty(sb.batch.n, dtype=torch.int32, device="cuda")
    assert t.lib.acs_overflow_index_device(t.h, C.byref(db.struct), clean.data_ptr(), idx.data_ptr(), C.byref(m),
                                           None) == 0 and m.value == 0
    t.close()


def _shard_reduce_gpu(urns, full_map, world, make_batch):
    """Evaluate `world` policy-set shards one after another on this GPU and reduce their
    keys with MAX, as the RCCL all-reduce of the rule-sharded bench does across GPUs."""
    keys = []
    for r in range(world):
        a, b = shard.partition(full_map, world)[r]
        cs = compiler.compile_store(shard.slice_store(full_map, a, b), urns, DEFAULT_CAS)
        t = gpu_tables(cs)
        dec = is_allowed_device(t, DeviceBatch(make_batch(cs), 0))
        keys.append(shard.keys_device(t, dec, shard.base(full_map, a)))
        torch.cuda.synchronize()
        t.close()
    red = torch.stack(keys).max(dim=0).values
    return decisions_from_tensor(shard.decode_device(native.load(), red))


@pytest.mark.parametrize("world", [2, 3, 8])
def test_rule_shard_c3_gpu(world):
    doc, cs, sb = _synth("c3", 60_000)
    full = store.populate(doc)
    t = gpu_tables(cs)
    want = decisions_from_tensor(is_allowed_device(t, DeviceBatch(sb.batch, 0)))
    t.close()
    got = _shard_reduce_gpu(FULL_URNS, full, world, lambda c: synth.requests(c, 60_000, "c3").batch)
    assert np.array_equal(got.view(np.uint64), want.view(np.uint64))


def test_rule_shard_random_gpu():
    terminal = 0
    for seed in range(60):
        urns, doc, reqs = randgen.rand_case(seed)
        o, cs = build(urns, doc)
        want = gpu_tables(cs).is_allowed(encoder.Encoder(cs).encode(reqs))
        got = _shard_reduce_gpu(urns, store.populate(doc), 2, lambda c: encoder.Encoder(c).encode(reqs))
        assert np.array_equal(got.view(np.uint64), want.view(np.uint64)), seed
        terminal += int(((want["flags"] & (L.OF_ERR | L.OF_HOST_COND)) != 0).sum())
    assert terminal > 0


def test_device_api_and_ragged_sizes():
    doc, cs, sb = _synth("c2", 70_001)  # not a multiple of the 256-lane block
    t = gpu_tables(cs)
    db = DeviceBatch(sb.batch, 0)
    out = is_allowed_device(t, db)
    torch.cuda.synchronize()
    dec = decisions_from_tensor(out)
    ref = t.is_allowed(sb.batch)
    assert np.array_equal(dec.view(np.uint64), ref.view(np.uint64))
    empty = encoder.Encoder(cs).encode([])
    assert t.is_allowed(empty).shape == (0,)
    t.close()


def test_max_attribute_counts():
    urns, doc, _ = randgen.rand_case(11)
    o, cs = build(urns, doc)
    ent = randgen.ENTITIES
    req = {"target": {"subjects": [{"id": randgen.U["role"], "value": "SimpleUser"}] * L.SMAX,
                      "resources": [{"id": randgen.U["entity"], "value": ent[k % len(ent)]} for k in range(L.QMAX)],
                      "actions": [{"id": randgen.U["actionID"], "value": randgen.ACTIONS[0]}] * L.AMAX},
           "context": {"subject": {"id": "Alice", "role_associations": [{"role": "SimpleUser"}] * L.RMAX,
                                   "hierarchical_scopes": []}, "resources": []}}
    over = {"target": dict(req["target"], resources=req["target"]["resources"] * 2), "context": req["context"]}
    b = encoder.Encoder(cs).encode([req, over])
    t = gpu_tables(cs)
    dec = t.is_allowed(b)
    t.close()
    got = gpu_outcome(cs, dec[0])
    if got[0] != "HOST":
        assert got == oracle_outcome(o, req)
    assert results.outcome(cs, dec[1])[0] == "HOST"  # beyond packed capacity -> host, never wrong
