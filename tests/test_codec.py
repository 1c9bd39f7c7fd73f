"""The native request codec (csrc/acs_codec.cpp) against the Python encoder + the oracle.

For the same JSON requests the codec's batch must carry the same request-only facts as
encoder.py's (flags, counts, attribute kinds, context slots, indexOf masks, regex-matrix
columns and cells; ids compared as the strings they intern) and, evaluated by the CPU
build of the evaluator core, give bit-identical decision records and reverse queries —
which the oracle pins (tests/test_host_core_diff.py).  Also: regex cells vs V8, the HR
forest cache (inline text, per-subject registration, eviction), multi-threaded encoding.
"""
import ctypes
import json

import numpy as np
import pytest

import host_core
import randgen
from diff_utils import build, gpu_outcome, oracle_outcome, norm_rq
from kat_utils import load_kats, load_fixture, urns_for
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS, Oracle
from oracle.jsval import OracleUnsupported
from acs_mi355x import compiler, encoder, native, results, store, synth, layout as L
from acs_mi355x.codec import NativeCodec
from acs_mi355x.jsops import MISSING


def _s(ov, i):
    v = ov.string(int(i))
    return ("m",) if v is MISSING else (("n",) if v is None else ("s", v))


def compare_batches(pb, nb, check_cols=True):
    """Request-only facts of the Python batch `pb` and the codec batch `nb`."""
    assert pb.n == nb.n
    n = pb.n
    ph, nh = pb.hdr, nb.hdr
    assert np.array_equal(ph["flags"] & 0xFFFF, nh["flags"] & 0xFFFF)
    for f in ("nres", "nsubj", "nact", "nroles"):
        assert np.array_equal(ph[f], nh[f]), f
    host = (ph["flags"] & L.RQ_HOST) != 0
    assert sorted(pb.host_reasons) == sorted(nb.host_reasons)
    for i in range(n):
        if host[i]:
            continue
        assert _s(pb.overlay, ph["subject_id"][i]) == _s(nb.overlay, nh["subject_id"][i]), i
        for j in range(ph["nres"][i]):
            p, q = pb.res[j, i], nb.res[j, i]
            for f in ("contains", "kind", "slot_a", "slot_b"):
                assert p[f] == q[f], (i, j, f)
            if check_cols:
                assert p["col"] == q["col"], (i, j)
            assert _s(pb.overlay, p["value"]) == _s(nb.overlay, q["value"]), (i, j)
            assert _s(pb.overlay, p["hash_sfx"]) == _s(nb.overlay, q["hash_sfx"]), (i, j)
        for arr, cnt in ((("subj", "nsubj")), (("act", "nact"))):
            for j in range(ph[cnt][i]):
                a, b = getattr(pb, arr)[j, i], getattr(nb, arr)[j, i]
                assert _s(pb.overlay, a["id"]) == _s(nb.overlay, b["id"])
                assert _s(pb.overlay, a["value"]) == _s(nb.overlay, b["value"])
        for j in range(ph["nroles"][i]):
            assert _s(pb.overlay, pb.roles[j, i]) == _s(nb.overlay, nb.roles[j, i])
        # context arena: same length per request (contents hold batch-local ids)
    if check_cols:
        assert pb.rx.shape == nb.rx.shape and np.array_equal(pb.rx, nb.rx)
    # packed request lines + extension records: both encoders emit exactly those of their own rows
    for x in (pb, nb):
        assert x.lines is not None
        assert x.lines.tobytes() == encoder.pack_lines(x).tobytes()
        assert x.ext.tobytes() == encoder.pack_ext(x).tobytes()


def decisions_equal(cs, pb, nb):
    """The Python batch (SoA and compact) and the codec batch (its own compact form and its
    expanded SoA rows) decide identically on the CPU build of the core."""
    a, b = host_core.is_allowed(cs, pb), host_core.is_allowed(cs, nb, compact=True)
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64))
    assert np.array_equal(a.view(np.uint64), host_core.is_allowed(cs, pb, compact=True).view(np.uint64))
    assert np.array_equal(a.view(np.uint64), host_core.is_allowed(cs, nb).view(np.uint64))
    return b


@pytest.mark.parametrize("seed", range(0, 600, 25))
def test_codec_random_stores(seed):
    for s in range(seed, seed + 25):
        urns, doc, reqs = randgen.rand_case(s)
        o, cs = build(urns, doc)
        pb = encoder.Encoder(cs).encode(reqs)
        codec = NativeCodec(compiler.store_blob(cs))
        nb = codec.encode(reqs)
        compare_batches(pb, nb)
        dec = decisions_equal(cs, pb, nb)
        for i, req in enumerate(reqs):
            got = gpu_outcome(cs, dec[i])
            if got[0] == "HOST":
                continue
            try:
                assert got == oracle_outcome(o, req), (s, i)
            except OracleUnsupported:
                pass
        # whatIsAllowed: same reverse queries (obligation ids through each batch's strings)
        pw, nw = host_core.what_is_allowed(cs, pb), host_core.what_is_allowed(cs, nb)
        assert np.array_equal(pw[0], nw[0]) and np.array_equal(pw[2], nw[2])
        for i in range(len(reqs)):
            try:
                a = norm_rq(results.reverse_query(cs, pb.overlay, pw[0][i], pw[1][i][:pw[2][i]], pw[3][i]))
            except (results.HostPathRequired, results.EvaluationError) as e:
                a = type(e).__name__
            try:
                b = norm_rq(results.reverse_query(cs, nb.overlay, nw[0][i], nw[1][i][:nw[2][i]], nw[3][i]))
            except (results.HostPathRequired, results.EvaluationError) as e:
                b = type(e).__name__
            assert a == b, (s, i)
        nb.close()
        codec.close()


def test_codec_kats():
    by_fx = {}
    for v in load_kats():
        by_fx.setdefault((v["fixture"], v["urns"]), []).append(v)
    checked = 0
    for (fx, _), vecs in by_fx.items():
        cs = compiler.compile_store(store.populate(load_fixture(fx)), urns_for(vecs[0]), DEFAULT_CAS)
        reqs = [v["request"] for v in vecs]
        pb = encoder.Encoder(cs).encode(reqs)
        nb = NativeCodec(compiler.store_blob(cs)).encode(reqs)
        compare_batches(pb, nb)
        dec = decisions_equal(cs, pb, nb)
        for v, d in zip(vecs, dec):
            if v["op"] == "isAllowed":
                oc = results.outcome(cs, d)
                if oc[0] == "OK":
                    assert oc[1] == v["expect"]["decision"], v["spec"]
                    checked += 1
    assert checked >= 70


@pytest.mark.parametrize("kind,threads,second", [("c2", 1, 0.0), ("c2", 4, 0.0), ("c3", 3, 0.0), ("c3", 2, 0.5)])
def test_codec_synthetic_threads(kind, threads, second):
    """The synthetic packer (incl. c3r2's second org-scoped role association and HR root) and
    both encoders give the same decisions for the same JSON requests."""
    doc = synth.c2_store() if kind == "c2" else synth.c3_store()
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 1500 if kind == "c2" else 400, kind, seed=77, second_role=second)
    reqs = [sb.decode(i) for i in range(sb.batch.n)]
    pb = encoder.Encoder(cs).encode(reqs)
    codec = NativeCodec(compiler.store_blob(cs))
    nb = codec.encode(reqs, threads=threads)
    compare_batches(pb, nb)
    decisions_equal(cs, pb, nb)
    # the synthetic packer and both encoders agree on the decisions
    assert np.array_equal(host_core.is_allowed(cs, sb.batch).view(np.uint64),
                          host_core.is_allowed(cs, nb).view(np.uint64))
    if kind == "c3" and not second:  # one flatten per distinct forest (threads may race on a first sight)
        st = nb.stats()
        distinct = len(set(zip(sb.draws["scope"].tolist(), sb.draws["role"].tolist())))
        assert st["hr_cache_hits"] + st["hr_cache_misses"] == sb.batch.n
        assert st["hr_cache_misses"] <= distinct * threads
        st2 = codec.encode(reqs, threads=threads).stats()
        assert st2["hr_cache_misses"] == 0 and st2["hr_cache_hits"] == sb.batch.n


def test_codec_classes_independent_of_threads():
    """The class work runs over the worker pool (per-thread key sets merged by hash partition,
    codec load over the pool): the same batch encoded on 1, 3 and 8 threads gets the same class
    of every request, the same class rows in the same order and the same coherence order, and
    a batch no larger than one whose level-0 keys were given up gets the same rows again."""
    cs = compiler.compile_store(store.populate(synth.c3_store()), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 30000, "c3", seed=5, second_role=0.5)
    text = sb.json_text()
    outs = []
    for th in (1, 3, 8):
        codec = NativeCodec(compiler.store_blob(cs))
        for k, v in sb.hrs_forests().items():
            codec.set_subject_scopes(k, v)
        b = codec.encode(text, threads=th)
        outs.append((b.lines["h"]["flags"].copy(), b.lines["cls2"].copy(), b.cand.copy(),
                     None if b.perm is None else b.perm.copy()))
        b2 = codec.encode(text, threads=th)  # second batch: the level-0 attempt may be skipped
        assert np.array_equal(b2.cand, b.cand) and np.array_equal(b2.lines["cls2"], b.lines["cls2"])
        b2.close()
        b.close()
        codec.close()
    for o in outs[1:]:
        assert np.array_equal(outs[0][0], o[0]) and np.array_equal(outs[0][1], o[1])
        assert np.array_equal(outs[0][2], o[2])
        assert (outs[0][3] is None) == (o[3] is None) and (o[3] is None or np.array_equal(outs[0][3], o[3]))


def test_codec_subject_scope_registry():
    """A request naming a registered forest ("$hrs") decides exactly as one carrying the
    forest inline; eviction sends it to the host; replacing the forest changes it."""
    doc = synth.c3_store()
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 160, "c3", seed=5)
    inline = [sb.decode(i) for i in range(sb.batch.n)]
    codec = NativeCodec(compiler.store_blob(cs))
    by_ref = []
    for r in inline:
        r = json.loads(json.dumps(r))
        subj = r["context"]["subject"]
        key = json.dumps(subj["hierarchical_scopes"], sort_keys=True)
        codec.set_subject_scopes(key, subj.pop("hierarchical_scopes"))
        subj["$hrs"] = key
        by_ref.append(r)
    a = host_core.is_allowed(cs, codec.encode(inline, threads=2))
    b = host_core.is_allowed(cs, codec.encode(by_ref, threads=2))
    assert np.array_equal(a.view(np.uint64), b.view(np.uint64))
    k0 = by_ref[0]["context"]["subject"]["$hrs"]
    assert codec.evict_subject(k0) and not codec.evict_subject(k0)
    nb = codec.encode(by_ref[:1])
    assert nb.hdr["flags"][0] & L.RQ_HOST and "not in the codec cache" in nb.host_reasons[0]


def test_codec_regex_cells_v8():
    """Every non-host cell the codec computes equals V8's (the rows of a store whose rule
    entity values are the fixture's patterns, the columns its request values)."""
    with open(__file__.replace("test_codec.py", "golden/regex_cells.json")) as f:
        pairs = json.load(f)["pairs"]
    rules = sorted({p[0] for p in pairs if p[0] is not None})[:600]
    rset = set(rules)
    urn = FULL_URNS
    doc = {"policy_sets": [{"id": "s", "combining_algorithm": DEFAULT_CAS[0]["urn"], "policies": [
        {"id": "p", "combining_algorithm": DEFAULT_CAS[0]["urn"], "rules": [
            {"id": f"r{k}", "effect": "PERMIT", "target": {"resources": [{"id": urn["entity"], "value": v}]}}
            for k, v in enumerate(rules)]}]}]}
    cs = compiler.compile_store(store.populate(doc), urn, DEFAULT_CAS)
    reqv = sorted({p[1] for p in pairs if p[1] is not None})
    reqs = [{"target": {"resources": [{"id": urn["entity"], "value": q}]}} for q in reqv]
    nb = NativeCodec(compiler.store_blob(cs)).encode(reqs)
    row = {v: r for r, v in enumerate(cs.rx_rows)}
    col = {nb.overlay.string(nb.res[0, i]["value"]): nb.res[0, i]["col"] for i in range(nb.n)}
    checked = 0
    for rv, qv, want in pairs:
        if rv not in rset or qv is None:
            continue
        got = int(nb.rx[col[qv], row[rv]])
        if got & L.RX_HOST:
            continue
        if got & (L.RX_THROW_TYPE | L.RX_THROW_SYNTAX):
            got &= L.RX_THROW_TYPE | L.RX_THROW_SYNTAX
        assert got == want, (rv, qv, got, want)
        checked += 1
    assert checked > 5000


def test_codec_rejects_malformed_array():
    cs = compiler.compile_store(store.populate(synth.c2_store()), FULL_URNS, DEFAULT_CAS)
    codec = NativeCodec(compiler.store_blob(cs))
    for bad in (b"", b"{}", b"[1,", b"[{\"target\": }]", b"[] x"):
        with pytest.raises(RuntimeError):
            codec.encode(bad)
    assert codec.encode(b"[]").n == 0
    nb = codec.encode(b'[1, "x", null, {"target": 5}]')
    assert (nb.hdr["flags"] & L.RQ_HOST).all() or (nb.hdr["flags"][2] & L.RQ_NO_TARGET)


# ---------------------------------------------------------------- the native store compiler
def _both(m, urns):
    from acs_mi355x.jsops import Unsupported
    try:
        a = compiler.store_blob(compiler.compile_store(m, urns, DEFAULT_CAS))
    except Unsupported:
        a = "Unsupported"
    try:
        b = compiler.native_store_blob(m, urns, DEFAULT_CAS)
    except Unsupported:
        b = "Unsupported"
    return a, b


@pytest.mark.parametrize("seed", range(0, 600, 100))
def test_native_compiler_random_stores_byte_identical(seed):
    for s in range(seed, seed + 100):
        urns, doc, _ = randgen.rand_case(s)
        a, b = _both(store.populate(doc), urns)
        assert a == b, s


def test_native_compiler_fixtures_and_configs_byte_identical():
    fx = sorted({(v["fixture"], v["urns"]) for v in load_kats()})
    for name, u in fx:
        v = next(x for x in load_kats() if x["fixture"] == name and x["urns"] == u)
        a, b = _both(store.populate(load_fixture(name)), urns_for(v))
        assert a == b and a != "Unsupported", name
    for doc in (synth.c2_store(), synth.c3_store()):
        a, b = _both(store.populate(doc), FULL_URNS)
        assert a == b


def _request_rows(b):
    """Per request: (its class rows — the class row and its second class row (composed rows) —
    and its role-factor rows (None: no role filtering)), each as a set: which of two rows is
    first is the batch's row order."""
    cls = (b.hdr["flags"] >> np.uint32(16)).astype(np.int64)
    cls2 = b.lines["cls2"].astype(np.int64)
    out = []
    for i in range(b.n):
        c = b.cand[cls[i]].tobytes() if b.cand is not None and cls[i] < b.cand.shape[0] else None
        c2 = b.cand[cls2[i] - 1].tobytes() if cls2[i] else None
        r = None
        if b.role_key is not None:  # row | (1 + second row) << 16
            k = int(b.role_key[i])
            r1, r2 = k & 0xFFFF, (k >> 16) - 1
            if r1 < b.role_bits.shape[0] and r2 < b.role_bits.shape[0]:
                r = frozenset(b.role_bits[x].tobytes() for x in (r1, r2) if x >= 0)
        out.append((frozenset(x for x in (c, c2) if x is not None), r))
    return out


@pytest.mark.parametrize("level", [0, 1, 2, 3])
def test_codec_class_rows_match_python_at_every_level(level, monkeypatch):
    """The codec's class rows (with the useful sections) and role-factor rows equal the Python
    candidates' for every request, at each key level (level 1 composes per-role rows, levels 2
    and 3 carry a role factor)."""
    from acs_mi355x import candidates
    names = list(candidates.LEVELS)
    cases = [(FULL_URNS, store.populate(synth.c3_store(n_sets=40)), None)]
    for s in range(0, 60, 6):
        urns, doc, reqs = randgen.rand_case(s)
        cases.append((urns, store.populate(doc), reqs))
    checked = 0
    for urns, m, reqs in cases:
        try:
            cs = compiler.compile_store(m, urns, DEFAULT_CAS)
        except Exception:
            continue
        if reqs is None:
            sb = synth.requests(cs, 3000, "c3", seed=11, tree=synth.OrgTree(fanout=3, depth=5), second_role=0.5)
            reqs = [sb.decode(i) for i in range(sb.batch.n)]
        monkeypatch.setattr(candidates, "FORCE_LEVEL", names[level])
        pb = encoder.Encoder(cs).encode(reqs)
        codec = NativeCodec(compiler.store_blob(cs))
        native.load().acs_internal_codec_force_level(ctypes.c_void_p(codec.h), level)  # test hook
        nb = codec.encode(reqs, threads=2)
        assert (pb.cand_wp, pb.cand_wsu, pb.cand_wpu, pb.cand_wr) == (nb.cand_wp, nb.cand_wsu, nb.cand_wpu, nb.cand_wr)
        assert (pb.role_key is None) == (nb.role_key is None)
        assert _request_rows(pb) == _request_rows(nb)
        checked += 1
    assert checked >= 8


def test_parallel_delimiter_matches_serial():
    """The three-pass parallel delimiter of the request array (acs_codec.cpp split_items: quote
    parity, per-chunk depth minima, top-level commas) gives the serial delimiter's items on a
    > 4 MB array whose strings hold quotes, escapes, brackets and "},{" sequences, chunk
    boundaries falling anywhere."""
    import random
    doc = synth.c2_store()
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 400, "c2", seed=13)
    base = [sb.decode(i) for i in range(sb.batch.n)]
    rng = random.Random(5)
    nasty = ['a"b', 'x\\\\"},{"y', '[[{', '}]', '\\\\', 'q\\\\\\\\"', '},{', ',,,', 'tab\\there', 'ü"ñ']
    reqs, size = [], 0
    while size < (5 << 20):
        r = json.loads(json.dumps(rng.choice(base)))
        r["target"]["subjects"].append({"id": "urn:x", "value": rng.choice(nasty) * rng.randint(1, 4)})
        if rng.random() < 0.3:
            r["note"] = {"deep": [[{"s": rng.choice(nasty)}]], "t": rng.choice(nasty)}
        reqs.append(r)
        size += len(json.dumps(r)) + 2
    codec = NativeCodec(compiler.store_blob(cs))
    # batch-local string ids depend on the encoding thread: compare what does not
    shape = lambda b: np.stack([b.lines["h"][f].astype(np.int64) for f in ("flags", "nres", "nsubj", "nact", "nroles")])  # noqa: E731
    for text in (json.dumps(reqs), json.dumps(reqs, indent=1), json.dumps(reqs, ensure_ascii=False)):
        one = codec.encode(text, threads=1)
        want = host_core.is_allowed(cs, one, compact=True).view(np.uint64)
        for t in (3, 7):
            many = codec.encode(text, threads=t)
            assert many.n == one.n == len(reqs)
            assert np.array_equal(shape(many), shape(one))
            assert many.host_reasons == one.host_reasons
            assert np.array_equal(host_core.is_allowed(cs, many, compact=True).view(np.uint64), want)


def test_codec_hrs_key_lists_compose_registered_forests():
    """"$hrs": [k1, k2] names one registered forest per role association; the codec decides
    such requests exactly as with the concatenated hierarchical_scopes inline (and as the
    synthetic packer), for one- and two-association subjects."""
    doc = synth.c3_store(n_sets=40)
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 3000, "c3", seed=9, tree=synth.OrgTree(fanout=3, depth=5), second_role=0.5)
    codec = NativeCodec(compiler.store_blob(cs))
    forests = sb.hrs_forests()
    assert len(forests) < sb.batch.n  # one per (scope, role), shared
    for k, v in forests.items():
        codec.set_subject_scopes(k, v)
    by_ref = codec.encode(sb.json_text(), threads=3)
    assert not by_ref.host_reasons
    inline = codec.encode([sb.decode(i) for i in range(sb.batch.n)], threads=3)
    want = host_core.is_allowed(cs, inline, compact=True).view(np.uint64)
    assert np.array_equal(host_core.is_allowed(cs, by_ref, compact=True).view(np.uint64), want)
    assert np.array_equal(host_core.is_allowed(cs, sb.batch).view(np.uint64), want)
    # a list naming an unregistered forest goes to the host
    bad = codec.encode(sb.json_text([0]).replace(b'"$hrs":[', b'"$hrs":["nope",'))
    assert bad.hdr["flags"][0] & L.RQ_HOST
