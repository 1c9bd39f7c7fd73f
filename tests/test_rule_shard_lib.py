"""Rule sharding inside the library (acs_compile_sharded, SURVEY §8(e) configs[4] variant ii in
one process): the store cut into contiguous runs of whole policy sets, one device each; every
device evaluates the whole batch with the batch's class rows cut to its nodes, and the primary
MAX-reduces the 64-bit shard keys into the records of an unsharded evaluation.

CPU: the library's own cut (acs_internal_shard_blob: sub-images with rebased child ranges and a
per-run NF_CLEAN_BELOW) and row slicing (acs_internal_slice_rows, the slice_rows_kernel's code)
run through the CPU build of the evaluator core shard by shard, keys MAX-reduced and decoded,
equal the unsharded records — random stores (errors, conditions, null policies, HR, ACL) and
the c3 / c3-adverse workloads, 1 to 5 shards.  GPU: acs_compile_sharded on device 0 two and
three times equals a single handle."""
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
        for parts in (2, 3):
            t = native.Tables(blob, devices=[0] * parts, sharded=True)
            assert t.devices() == [0] * parts
            assert np.array_equal(_u64(t.is_allowed(b)), _u64(want)), (kind, parts)
            with pytest.raises(RuntimeError):
                t.what_is_allowed(b)  # the cross-shard reduction covers isAllowed only
            t.close()
        one.close()
        b.close()
        codec.close()
