"""Rule sharding inside the library (acs_compile_sharded, SURVEY §8(e) configs[4] variant ii in
one process): the store cut into contiguous runs of whole policy sets, one device each; every
device evaluates the whole batch with the batch's class rows cut to its nodes, and the primary
MAX-reduces the 64-bit shard keys into the records of an unsharded evaluation.

CPU: the library's own cut (acs_internal_shard_blob: sub-images with rebased child ranges and a
per-run NF_CLEAN_BELOW) and row slicing (acs_internal_slice_rows, the slice_rows_kernel's code)
run through the CPU build of the evaluator core shard by shard, keys MAX-reduced and decoded,
equal the unsharded records — random stores (errors, conditions, null policies, HR, ACL) and
the c3 / c3-adverse workloads, 1 to 5 shards.  GPU: acs_compile_sharded on device 0 two and
three times equals a single handle, for isAllowed and for whatIsAllowed (rows, logs, and the
obligation-only pass).  whatIsAllowed on the host core's shards joined by the library equals the
unsharded outputs (random stores, c4-shaped queries, 1 to 5 shards)."""
import ctypes as C

import numpy as np
import pytest

import host_core
import randgen
from diff_utils import build
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS
from acs_mi355x import compiler, encoder, native, store, synth
from acs_mi355x.codec import NativeCodec


class ShardC(C.Structure):
    _fields_ = [("set_base", C.c_uint32), ("pol_base", C.c_uint32), ("rule_base", C.c_uint32)]


def _lib():
    lib = native.load()
    lib.acs_internal_shard_blob.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_int, C.POINTER(C.c_void_p),
                                            C.POINTER(C.c_size_t), C.POINTER(ShardC)]
    lib.acs_internal_slice_rows.argtypes = [C.c_void_p, C.c_uint32, C.POINTER(ShardC), C.c_uint32, C.c_uint32,
                                            C.c_uint32, C.c_void_p, C.c_void_p, C.c_void_p]
    lib.acs_blob_free.argtypes = [C.c_void_p]
    return lib


def shard_blob(blob, parts, k):
    lib = _lib()
    out, n, base = C.c_void_p(), C.c_size_t(), ShardC()
    assert lib.acs_internal_shard_blob(blob, len(blob), parts, k, C.byref(out), C.byref(n), C.byref(base)) == 0, \
        native.last_error()
    try:
        return C.string_at(out.value, n.value), base
    finally:
        lib.acs_blob_free(out)


def sharded_records_host(blob, batch, parts, compact):
    """acs_compile_sharded's evaluation restated over the host core."""
    lib = _lib()
    h = np.frombuffer(blob[:64], np.uint32)
    g_pols = int(h[3])
    s = host_core._struct(batch, compact)
    n = int(s.n)
    best = np.zeros(n, np.uint64)
    for k in range(parts):
        sub, base = shard_blob(blob, parts, k)
        sh = np.frombuffer(sub[:64], np.uint32)
        ns, npol, nr = int(sh[2]), int(sh[3]), int(sh[4])
        d = native.ReqBatchC.from_buffer_copy(s)
        keep = []
        if s.cand:
            lay = np.zeros(6, np.uint32)
            assert lib.acs_internal_slice_rows(C.byref(s), g_pols, C.byref(base), ns, npol, nr, None, None,
                                               lay.ctypes.data) == 0
            words = int(lay[0])
            rows = np.zeros(int(s.cand_rows) * words + 1, np.uint32)
            roles = np.zeros(max(int(s.role_rows), 1) * words + 1, np.uint32)
            assert lib.acs_internal_slice_rows(C.byref(s), g_pols, C.byref(base), ns, npol, nr, rows.ctypes.data,
                                               roles.ctypes.data, lay.ctypes.data) == 0
            keep += [rows, roles]
            d.cand = rows.ctypes.data
            d.cand_words, d.cand_wp, d.cand_wr, d.cand_wsu, d.cand_wpu, d.cand_wv = (int(x) for x in lay)
            if s.role_key:
                d.role_rows_bits = roles.ctypes.data
        dec = np.zeros(n, host_core.L.DECISION_DT)
        assert host_core.lib().acs_host_is_allowed(sub, len(sub), C.byref(d), dec.ctypes.data) == 0
        keys = np.zeros(n, np.int64)
        hb = host_core.ShardC(base.set_base, base.pol_base, base.rule_base)
        assert host_core.lib().acs_host_shard_keys(sub, len(sub), dec.ctypes.data, n, C.byref(hb),
                                                   keys.ctypes.data) == 0
        best = np.maximum(best, keys.view(np.uint64))
    return host_core.shard_decode(best.view(np.int64))


def _u64(d):
    return np.ascontiguousarray(d).view(np.uint64)


class WiaPartC(C.Structure):
    _fields_ = [("base", ShardC), ("n_sets", C.c_uint32), ("n_pols", C.c_uint32), ("n_rules", C.c_uint32),
                ("bits", C.c_void_p), ("obl", C.c_void_p), ("obl_n", C.c_void_p), ("out", C.c_void_p)]


def _shard_batch(lib, s, g_pols, base, ns, npol, nr, keep):
    """The batch struct s with its class rows cut to one shard's nodes (acs_internal_slice_rows)."""
    d = native.ReqBatchC.from_buffer_copy(s)
    if s.cand:
        lay = np.zeros(6, np.uint32)
        assert lib.acs_internal_slice_rows(C.byref(s), g_pols, C.byref(base), ns, npol, nr, None, None,
                                           lay.ctypes.data) == 0
        words = int(lay[0])
        rows = np.zeros(int(s.cand_rows) * words + 1, np.uint32)
        roles = np.zeros(max(int(s.role_rows), 1) * words + 1, np.uint32)
        assert lib.acs_internal_slice_rows(C.byref(s), g_pols, C.byref(base), ns, npol, nr, rows.ctypes.data,
                                           roles.ctypes.data, lay.ctypes.data) == 0
        keep += [rows, roles]
        d.cand = rows.ctypes.data
        d.cand_words, d.cand_wp, d.cand_wr, d.cand_wsu, d.cand_wpu, d.cand_wv = (int(x) for x in lay)
        if s.role_key:
            d.role_rows_bits = roles.ctypes.data
    return d


def sharded_what_is_allowed_host(blob, batch, parts, compact, overflow_idx=None, cap=70, chunks=5):
    """acs_compile_sharded's whatIsAllowed restated over the host core: each shard's K2 outputs on its
    sub-image, joined by the library's acs_internal_wia_join; with overflow_idx, also the
    obligation-only pass per shard joined by acs_internal_wia_obl_join."""
    from acs_mi355x import layout as L
    from acs_mi355x.results import bits_layout
    lib = _lib()
    vp = C.c_void_p
    lib.acs_internal_wia_join.argtypes = [C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, C.POINTER(WiaPartC),
                                          C.c_size_t, C.c_size_t, vp, vp, vp, vp]
    lib.acs_internal_wia_join.restype = None
    lib.acs_internal_wia_obl_join.argtypes = [C.c_int, C.POINTER(vp), C.POINTER(vp), C.c_size_t, C.c_uint32,
                                              C.c_uint32, vp, vp]
    lib.acs_internal_wia_obl_join.restype = None
    hc = host_core.lib()
    hc.acs_host_what_is_allowed_obl_shard.argtypes = [vp, C.c_size_t, C.POINTER(native.ReqBatchC), vp, C.c_size_t,
                                                      C.c_uint32, C.c_uint32, vp, vp, C.c_uint32, C.c_uint32]
    h = np.frombuffer(blob[:64], np.uint32)
    g_sets, g_pols, g_rules = int(h[2]), int(h[3]), int(h[4])
    s = host_core._struct(batch, compact)
    n = int(s.n)
    keep, P, obl_parts = [], (WiaPartC * parts)(), []
    for k in range(parts):
        sub, base = shard_blob(blob, parts, k)
        sh = np.frombuffer(sub[:64], np.uint32)
        ns, npol, nr = int(sh[2]), int(sh[3]), int(sh[4])
        d = _shard_batch(lib, s, g_pols, base, ns, npol, nr, keep)
        words = max(bits_layout(ns, npol, nr)[2], 1)
        bits = np.zeros((n, words), np.uint32)
        obl = np.zeros((n, L.OBL_MAX, 2), np.uint32)
        obl_n = np.zeros(n, np.uint32)
        out = np.zeros(n, L.DECISION_DT)
        assert hc.acs_host_what_is_allowed(sub, len(sub), C.byref(d), bits.ctypes.data, obl.ctypes.data,
                                           obl_n.ctypes.data, out.ctypes.data) == 0
        keep += [bits, obl, obl_n, out]
        P[k] = WiaPartC(base, ns, npol, nr, bits.ctypes.data, obl.ctypes.data, obl_n.ctypes.data, out.ctypes.data)
        if overflow_idx is not None and len(overflow_idx):
            idx = np.ascontiguousarray(overflow_idx, np.uint32)
            po = np.zeros((chunks, len(idx), cap, 2), np.uint32)
            pn = np.zeros((chunks, len(idx)), np.uint32)
            assert hc.acs_host_what_is_allowed_obl_shard(sub, len(sub), C.byref(d), idx.ctypes.data, len(idx), chunks,
                                                         cap, po.ctypes.data, pn.ctypes.data, g_sets,
                                                         base.set_base) == 0
            obl_parts.append((po, pn))
    words = bits_layout(g_sets, g_pols, g_rules)[2]
    bits = np.zeros((n, max(words, 1)), np.uint32)
    obl = np.zeros((n, L.OBL_MAX, 2), np.uint32)
    obl_n = np.zeros(n, np.uint32)
    out = np.zeros(n, L.DECISION_DT)
    lib.acs_internal_wia_join(g_sets, g_pols, g_rules, parts, P, 0, n, bits.ctypes.data, obl.ctypes.data,
                              obl_n.ctypes.data, out.ctypes.data)
    res = (bits, obl, obl_n, out)
    if obl_parts:
        m = len(overflow_idx)
        jo = np.zeros((chunks, m, cap, 2), np.uint32)
        jn = np.zeros((chunks, m), np.uint32)
        po = (vp * parts)(*[x[0].ctypes.data for x in obl_parts])
        pn = (vp * parts)(*[x[1].ctypes.data for x in obl_parts])
        lib.acs_internal_wia_obl_join(parts, po, pn, m, chunks, cap, jo.ctypes.data, jn.ctypes.data)
        res = res + (jo, jn)
    return res


def _same_wia(got, want, ctx):
    """whatIsAllowed outputs equal as the ABI defines them (log entries past a request's count are
    unspecified)."""
    bits, obl, obl_n, out = got[:4]
    wbits, wobl, wobl_n, wout = want[:4]
    assert np.array_equal(_u64(out), _u64(wout)), ctx
    assert np.array_equal(obl_n, wobl_n), ctx
    assert np.array_equal(bits, wbits), ctx
    for i in np.flatnonzero(obl_n):
        assert np.array_equal(obl[i, :obl_n[i]], wobl[i, :obl_n[i]]), (ctx, int(i))


def test_sharded_random_stores_host():
    checked = 0
    for seed in range(0, 90, 3):
        urns, doc, reqs = randgen.rand_case(seed)
        try:
            _, cs = build(urns, doc)
        except Exception:
            continue
        b = encoder.Encoder(cs).encode(reqs)
        blob = compiler.store_blob(cs)
        want = host_core.is_allowed(cs, b)
        for parts in (1, 2, 3, 5):
            got = sharded_records_host(blob, b, parts, compact=False)
            assert np.array_equal(_u64(got), _u64(want)), (seed, parts)
        checked += 1
    assert checked >= 20


@pytest.mark.parametrize("kind", ["c3", "c3adv"])
def test_sharded_codec_batches_host(kind):
    """Native codec batches (class rows with useful and verdict sections, composed second
    class rows, HR / ACL arena records) cut to 2 and 4 runs of sets."""
    import bench
    cs = compiler.compile_store(store.populate(bench.make_store(kind)), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 3000, "c3", seed=5, second_role=0.5, acl=0.1 if kind == "c3adv" else 0.0,
                        classes=False)
    blob = compiler.store_blob(cs)
    codec = NativeCodec(blob)
    for k, v in sb.hrs_forests().items():
        codec.set_subject_scopes(k, v)
    b = codec.encode(sb.json_text(), threads=3)
    want = host_core.is_allowed(cs, b, compact=True)
    for parts in (2, 4):
        got = sharded_records_host(blob, b, parts, compact=True)
        assert np.array_equal(_u64(got), _u64(want)), parts
    b.close()
    codec.close()


def test_sharded_what_is_allowed_random_stores_host():
    """whatIsAllowed on a rule-sharded store (set-sharded bitsets concatenate,
    obligations merged in set order) through the host core and the library's join: equal to the
    unsharded outputs — errors (the first throwing set decides), host requests, obligations — over
    random stores, 1 to 5 shards."""
    checked = 0
    for seed in range(0, 120, 3):
        urns, doc, reqs = randgen.rand_case(seed)
        try:
            _, cs = build(urns, doc)
        except Exception:
            continue
        b = encoder.Encoder(cs).encode(reqs)
        blob = compiler.store_blob(cs)
        want = host_core.what_is_allowed(cs, b)
        for parts in (1, 2, 3, 5):
            _same_wia(sharded_what_is_allowed_host(blob, b, parts, compact=False), want, (seed, parts))
        checked += 1
    assert checked >= 25


def test_sharded_what_is_allowed_c4_host():
    """c4-shaped queries (c3 store, 1-2 role associations) on 2 and 4 shards: the joined rows and
    logs equal the unsharded ones, and the obligation-only pass over the shards (global set ranges
    clipped per shard, parts joined in shard order) returns the unsharded pass's logs."""
    from acs_mi355x import layout as L
    cs = compiler.compile_store(store.populate(synth.c3_store()), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 1500, "c3", seed=8, second_role=0.5)
    blob = compiler.store_blob(cs)
    want = host_core.what_is_allowed(cs, sb.batch)
    over = np.flatnonzero((want[3]["flags"] & L.OF_OBL_OVERFLOW) != 0)
    assert len(over) > 0
    one = host_core.Tables(blob)
    wobl, wn = one.what_is_allowed_obl(sb.batch, over, 70, chunks=5)
    for parts in (2, 4):
        got = sharded_what_is_allowed_host(blob, sb.batch, parts, compact=False, overflow_idx=over, cap=70, chunks=5)
        _same_wia(got, want, parts)
        jo, jn = got[4], got[5]
        assert np.array_equal(jn, wn), parts
        for c in range(5):
            for j in range(len(over)):
                if wn[c, j] <= 70:
                    assert np.array_equal(jo[c, j, :wn[c, j]], wobl[c, j, :wn[c, j]]), (parts, c, j)


@pytest.mark.gpu
def test_sharded_handle_gpu():
    """acs_compile_sharded over device 0 two and three times == one handle (c3 20k requests
    through the codec, and a c3-adverse batch with conditions, a null policy and ACLs)."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import bench
    for kind in ("c3", "c3adv"):
        cs = compiler.compile_store(store.populate(bench.make_store(kind)), FULL_URNS, DEFAULT_CAS)
        sb = synth.requests(cs, 20_000, "c3", seed=7, second_role=0.5, acl=0.1 if kind == "c3adv" else 0.0,
                            classes=False)
        blob = compiler.store_blob(cs)
        codec = NativeCodec(blob)
        for k, v in sb.hrs_forests().items():
            codec.set_subject_scopes(k, v)
        b = codec.encode(sb.json_text(), threads=4)
        one = native.Tables(blob, 0)
        want = one.is_allowed(b)
        if kind == "c3":
            wia_one = one.what_is_allowed(b)
            logs_one = one.resolve_overflow(b, wia_one[3].copy())
        for parts in (2, 3):
            t = native.Tables(blob, devices=[0] * parts, sharded=True)
            assert t.devices() == [0] * parts
            assert np.array_equal(_u64(t.is_allowed(b)), _u64(want)), (kind, parts)
            # the decision pipeline on the sharded handle: JSON chunks encoded while the previous
            # chunk is evaluated on every shard and reduced
            from acs_mi355x.codec import Pipeline
            pl = Pipeline(t, codec, threads=4, chunk=7000)
            got, pst = pl.is_allowed(sb.json_text(), sb.batch.n)
            pl.close()
            assert pst["chunks"] == 3 and np.array_equal(_u64(got), _u64(want)), (kind, parts, "pipeline")
            if kind == "c3":  # whatIsAllowed: shard rows joined, logs merged in set order
                got = t.what_is_allowed(b)
                _same_wia(got, wia_one, (kind, parts))
                over = np.flatnonzero((got[3]["flags"] & 0x20) != 0)
                assert len(over) > 0
                assert t.resolve_overflow(b, got[3].copy()).keys() == logs_one.keys()
                for i, lg in t.resolve_overflow(b, got[3].copy(), cap=70).items():
                    assert np.array_equal(lg, logs_one[i]), (parts, i)
            t.close()
        one.close()
        b.close()
        codec.close()
