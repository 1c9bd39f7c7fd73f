"""The multi-device handle (acs_compile_multi): a compact host batch split into contiguous
request shards, each device receiving only its shard's request lines, extension records and
arena words (acs_internal_shard_plan) with the batch's absolute offsets kept valid by
basing the shard's pointers one slice-start below the copies, and the records gathered in
request order.

CPU: the same split (plan + slice copies + rebased pointers) run through the CPU build of
the evaluator core shard by shard equals the whole batch.  GPU: a handle replicated on
device 0 twice (two images, two streams) equals a single handle, through acs_is_allowed,
acs_what_is_allowed and the pipeline."""
import ctypes as C

import numpy as np
import pytest

import host_core
import randgen
from diff_utils import build
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS
from acs_mi355x import compiler, encoder, native, store, synth
from acs_mi355x.codec import NativeCodec


def _u64(d):
    return np.ascontiguousarray(d).view(np.uint64)


def _plan_lib():
    lib = native.load()
    lib.acs_internal_check_batch2.argtypes = [C.c_void_p, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                              C.c_void_p]
    lib.acs_internal_shard_plan.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p, C.c_void_p]
    lib.acs_internal_shard_plan.restype = None
    return lib


def split_is_allowed_host(cs, batch, cuts, what=False):
    """acs_is_allowed's (what: acs_what_is_allowed's) multi-device split restated over the host
    core: shards [cuts[k], cuts[k+1]) each evaluated from copies of only its slices; what
    returns (bits, obl, obl_n, out) gathered in request order."""
    lib = _plan_lib()
    s = native.host_struct(batch, True)
    n = int(s.n)
    arena_end = np.zeros(n, np.uint32)
    assert lib.acs_internal_check_batch2(C.byref(s), cs.n_sets, cs.n_pols, cs.n_rules, 0,
                                         arena_end.ctypes.data) == 0, native.last_error()
    arena = np.ctypeslib.as_array((C.c_uint32 * max(int(s.arena_words), 1)).from_address(s.arena))
    ext = (np.ctypeslib.as_array((C.c_uint32 * int(s.ext_words)).from_address(s.ext)) if s.ext_words
           else np.zeros(0, np.uint32))
    out = np.zeros(n, host_core.L.DECISION_DT)
    blob = compiler.store_blob(cs)
    if what:
        from acs_mi355x.results import bits_layout
        words = max(bits_layout(cs.n_sets, cs.n_pols, cs.n_rules)[2], 1)
        bits = np.zeros((n, words), np.uint32)
        obl = np.zeros((n, host_core.L.OBL_MAX, 2), np.uint32)
        obl_n = np.zeros(n, np.uint32)
    for lo, hi in zip(cuts[:-1], cuts[1:]):
        if hi == lo:
            continue
        plan = np.zeros(4, np.uint64)
        lib.acs_internal_shard_plan(C.byref(s), lo, hi, arena_end.ctypes.data, plan.ctypes.data)
        a0, a1, e0, e1 = (int(x) for x in plan)
        # the "device" copies: the shard's lines and its slices only
        lines = np.array(np.ctypeslib.as_array((C.c_uint8 * (n * 128)).from_address(s.lines))[lo * 128:hi * 128])
        ar = np.array(arena[a0:a1]) if a1 > a0 else np.zeros(1, np.uint32)
        ex = np.array(ext[e0:e1]) if e1 > e0 else np.zeros(1, np.uint32)
        d = native.ReqBatchC.from_buffer_copy(s)
        d.n = hi - lo
        d.lines = lines.ctypes.data
        d.arena = ar.ctypes.data - 4 * a0
        d.ext = (ex.ctypes.data - 4 * e0) if s.ext else None
        if s.role_key:
            rk = np.array(np.ctypeslib.as_array((C.c_uint32 * n).from_address(s.role_key))[lo:hi])
            d.role_key = rk.ctypes.data
        sub = np.zeros(hi - lo, host_core.L.DECISION_DT)
        if what:
            sb_, so, sn = np.zeros((hi - lo, words), np.uint32), np.zeros((hi - lo, host_core.L.OBL_MAX, 2), np.uint32), \
                np.zeros(hi - lo, np.uint32)
            assert host_core.lib().acs_host_what_is_allowed(blob, len(blob), C.byref(d), sb_.ctypes.data, so.ctypes.data,
                                                            sn.ctypes.data, sub.ctypes.data) == 0
            bits[lo:hi], obl[lo:hi], obl_n[lo:hi] = sb_, so, sn
        else:
            assert host_core.lib().acs_host_is_allowed(blob, len(blob), C.byref(d), sub.ctypes.data) == 0
        out[lo:hi] = sub
        # the plan covers every request's arena words
        for i in range(lo, hi):
            off = int(batch.lines["h"]["arena_off"][i])
            assert arena_end[i] == off or (a0 <= off and arena_end[i] <= a1)
    return (bits, obl, obl_n, out) if what else out


def _same_wia(a, b):
    bits, obl, obl_n, out = a
    bits2, obl2, obl_n2, out2 = b
    assert np.array_equal(bits, bits2) and np.array_equal(obl_n, obl_n2) and np.array_equal(_u64(out), _u64(out2))
    for i in range(len(obl_n)):
        k = min(int(obl_n[i]), obl.shape[1])
        assert np.array_equal(obl[i, :k], obl2[i, :k]), i


def _cuts(n, parts, rng):
    inner = sorted(rng.choice(np.arange(1, n), size=min(parts - 1, n - 1), replace=False).tolist()) if n > 1 else []
    return [0] + inner + [n]


def test_split_gather_random_stores_host():
    """Random stores with wide requests (extension records, arena records): any contiguous
    split gives the whole batch's records."""
    rng = np.random.default_rng(3)
    checked = 0
    for seed in range(0, 120, 3):
        urns, doc, reqs = randgen.rand_case(seed)
        try:
            _, cs = build(urns, doc)
        except Exception:
            continue
        b = encoder.Encoder(cs).encode(reqs)
        if b.n < 2:
            continue
        whole = host_core.is_allowed(cs, b, compact=True)
        for parts in (2, 3, b.n):
            got = split_is_allowed_host(cs, b, _cuts(b.n, parts, rng))
            assert np.array_equal(_u64(got), _u64(whole)), (seed, parts)
        checked += 1
    assert checked >= 25


@pytest.mark.parametrize("kind", ["c2", "c3"])
def test_split_gather_codec_batch_host(kind):
    """Native codec batches (page-locked compact blocks, class rows, HR-scope arena records)
    split in 2 and 5 equal the whole batch."""
    doc = synth.c3_store() if kind == "c3" else synth.c2_store()
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    n = 3000
    sb = synth.requests(cs, n, kind, seed=9)
    idx = np.arange(n)
    codec = NativeCodec(compiler.store_blob(cs))
    if kind == "c3":
        for k, v in sb.hrs_forests(idx).items():
            codec.set_subject_scopes(k, v)
    b = codec.encode(sb.json_text(idx), threads=4)
    whole = host_core.is_allowed(cs, b, compact=True)
    wia = host_core.what_is_allowed(cs, b, compact=True)
    for parts in (2, 5):
        cuts = [n * k // parts for k in range(parts + 1)]
        assert np.array_equal(_u64(split_is_allowed_host(cs, b, cuts)), _u64(whole)), parts
        _same_wia(split_is_allowed_host(cs, b, cuts, what=True), wia)  # acs_what_is_allowed's split
    b.close()
    codec.close()


@pytest.mark.gpu
def test_two_replicas_on_one_device_gpu():
    """devices=[0, 0]: two images on device 0 (the replica peer-copied from the primary),
    a 20k c3 batch split between them == one handle; the pipeline over the replicated handle
    (chunks alternate between the devices) == too."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from acs_mi355x.codec import Pipeline
    cs = compiler.compile_store(store.populate(synth.c3_store()), FULL_URNS, DEFAULT_CAS)
    n = 20_000
    sb = synth.requests(cs, n, "c3", seed=21)
    idx = np.arange(n)
    text = sb.json_text(idx)
    blob = compiler.store_blob(cs)
    one = native.Tables(blob, 0)
    two = native.Tables(blob, devices=[0, 0])
    assert two.devices() == [0, 0]
    codec = NativeCodec(blob)
    for k, v in sb.hrs_forests(idx).items():
        codec.set_subject_scopes(k, v)
    b = codec.encode(text, threads=4)
    want = one.is_allowed(b)
    assert np.array_equal(_u64(two.is_allowed(b)), _u64(want))
    _same_wia(two.what_is_allowed(b), one.what_is_allowed(b))  # whatIsAllowed split over the replicas
    assert np.array_equal(_u64(two.is_allowed(sb.batch, compact=True)), _u64(want))
    p = Pipeline(two, codec, threads=4, chunk=3000)
    got, st = p.is_allowed(text, n)
    assert st["chunks"] == 7
    assert np.array_equal(_u64(got), _u64(want))
    p.close()
    b.close()
    two.close()
    one.close()


@pytest.mark.gpu
def test_eight_devices_replicated_and_sharded_update_gpu():
    """Eight replicas and eight rule shards on device 0 == one handle for isAllowed and
    whatIsAllowed; then acs_compile_update on both (SURVEY §8(e) with a store change): the last
    set's rule effects flipped (same shape: the replicas take the primary's changed blocks device to device,
    each shard a delta of its previous image) and a rule added (new shape: full images), each
    equal to a fresh single-device compile of the changed store."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import copy
    doc = synth.c3_store()
    sb = synth.requests(compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS), 20_000, "c3",
                        seed=41, second_role=0.5)

    def batch_for(d):
        cs = compiler.compile_store(store.populate(d), FULL_URNS, DEFAULT_CAS)
        blob = compiler.store_blob(cs)
        codec = NativeCodec(blob)
        for k, v in sb.hrs_forests().items():
            codec.set_subject_scopes(k, v)
        return blob, codec, codec.encode(sb.json_text(), threads=4)

    blob, codec, b = batch_for(doc)
    one = native.Tables(blob, 0)
    want, wia = one.is_allowed(b), one.what_is_allowed(b)
    rep = native.Tables(blob, devices=[0] * 8)
    sh = native.Tables(blob, devices=[0] * 8, sharded=True)
    for t, name in ((rep, "replicated"), (sh, "sharded")):
        assert t.devices() == [0] * 8
        assert np.array_equal(_u64(t.is_allowed(b)), _u64(want)), name
        _same_wia(t.what_is_allowed(b), wia)
    full = rep.upload_bytes
    flip = copy.deepcopy(doc)  # every rule of the last set (the walk's first) flipped: same shape
    for pol in flip["policy_sets"][-1]["policies"]:
        for r in pol["rules"]:
            r["effect"] = "DENY" if r["effect"] == "PERMIT" else "PERMIT"
    grow = copy.deepcopy(doc)
    grow["policy_sets"][20]["policies"][0]["rules"].append(dict(copy.deepcopy(r), id="added_rule"))
    for changed, same_shape in ((flip, True), (grow, False)):
        blob2, codec2, b2 = batch_for(changed)
        fresh = native.Tables(blob2, 0)
        want2, wia2 = fresh.is_allowed(b2), fresh.what_is_allowed(b2)
        for t, name in ((rep, "replicated"), (sh, "sharded")):
            u = t.updated(blob2)
            assert u.devices() == [0] * 8, name
            assert np.array_equal(_u64(u.is_allowed(b2)), _u64(want2)), (name, same_shape)
            _same_wia(u.what_is_allowed(b2), wia2)
            if same_shape:
                assert u.upload_bytes < full // 4, (name, u.upload_bytes, full)
            u.close()
        fresh.close()
        b2.close()
        codec2.close()
    blob2, codec2, b2 = batch_for(flip)  # the flipped rule changes some records (not a no-op update)
    fresh = native.Tables(blob2, 0)
    assert not np.array_equal(_u64(fresh.is_allowed(b2)), _u64(want))
    fresh.close()
    b2.close()
    codec2.close()
    for t in (rep, sh, one):
        t.close()
    b.close()
    codec.close()
