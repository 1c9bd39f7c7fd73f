"""Host-side structural checks of the library (csrc/acs_validate.cpp), CPU only.

Every image / batch our compilers and encoders produce passes; corrupting any offset the
kernels follow (child ranges, pool offsets, arena offsets and records, regex-matrix
coordinates, context slots, candidate layout) is refused with an error before any device
work — acs_compile rejects a malformed image before it allocates anything.
"""
import ctypes as C

import numpy as np
import pytest

import randgen
from acs_mi355x import compiler, encoder, layout as L, native, store, synth
from acs_mi355x.codec import NativeCodec
from acs_mi355x.jsops import Unsupported
from kat_utils import load_kats, load_fixture, urns_for
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS


@pytest.fixture(scope="module")
def lib():
    lib = native.load()
    lib.acs_internal_check_blob.argtypes = [C.c_void_p, C.c_size_t, C.POINTER(C.c_uint32)]
    lib.acs_internal_check_batch.argtypes = [C.POINTER(native.ReqBatchC), C.c_uint32, C.c_uint32, C.c_uint32,
                                             C.c_uint32]
    return lib


def _rows(cs):
    k = (cs.rres["kind"] & L.K_ENT_LOOSE) != 0
    return int(cs.rres["row"][k].max()) + 1 if k.any() else 0


def _check(lib, cs, b):
    s = native.batch_struct(b)
    return lib.acs_internal_check_batch(C.byref(s), cs.n_sets, cs.n_pols, cs.n_rules, _rows(cs))


def _cases():
    out = []
    by_fx = {}
    for v in load_kats():
        by_fx.setdefault((v["fixture"], v["urns"]), []).append(v)
    for (fx, _), vecs in by_fx.items():
        cs = compiler.compile_store(store.populate(load_fixture(fx)), urns_for(vecs[0]), DEFAULT_CAS)
        out.append((cs, [v["request"] for v in vecs]))
    for s in range(0, 120, 3):
        urns, doc, reqs = randgen.rand_case(s)
        try:
            out.append((compiler.compile_store(store.populate(doc), urns, DEFAULT_CAS), reqs))
        except Unsupported:
            pass
    return out


def test_valid_images_and_batches_pass(lib):
    for cs, reqs in _cases():
        blob = compiler.store_blob(cs)
        rows = C.c_uint32(99)
        assert lib.acs_internal_check_blob(blob, len(blob), C.byref(rows)) == 0
        assert rows.value == _rows(cs)
        assert _check(lib, cs, encoder.Encoder(cs).encode(reqs)) == 0, native.last_error(lib)
        nb = NativeCodec(blob).encode(reqs)
        assert _check(lib, cs, nb) == 0, native.last_error(lib)
    for kind in ("c2", "c3"):
        cs = compiler.compile_store(store.populate(synth.c2_store() if kind == "c2" else synth.c3_store()),
                                    FULL_URNS, DEFAULT_CAS)
        sb = synth.requests(cs, 3000, kind, seed=3)
        assert _check(lib, cs, sb.batch) == 0, native.last_error(lib)


def _mut(b, field, fn):
    """A copy of batch b's arrays with one of them modified."""
    class B:
        pass
    c = B()
    for k in ("n", "hdr", "res", "subj", "act", "roles", "arena", "rx", "cand", "cand_wp", "cand_wr",
              "role_key", "role_bits", "lines"):
        v = getattr(b, k, None)
        setattr(c, k, v.copy() if isinstance(v, np.ndarray) else v)
    fn(getattr(c, field), c)
    return c


def test_corrupt_batches_refused(lib):
    cs = compiler.compile_store(store.populate(synth.c3_store()), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 500, "c3", seed=4)
    b = sb.batch
    assert _check(lib, cs, b) == 0
    # a request with context slots and an arena carrying slot records / instance lists
    arena_words = b.arena.view(np.uint32)
    offs = b.hdr["arena_off"].astype(np.int64)
    with_slots = next(i for i in range(b.n) if (arena_words[offs[i]] >> 16) & 0xFF)
    ent = (b.res["kind"] & L.K_ENT_LOOSE) != 0
    safe = ent & ((b.res["pad"] & L.RES_RX_SAFE) != 0)
    safe_col = int(b.res["col"][tuple(np.argwhere(safe)[0])])

    bad = {
        "arena offset": _mut(b, "hdr", lambda a, c: a["arena_off"].__setitem__(7, len(arena_words) - 1)),
        "counts": _mut(b, "hdr", lambda a, c: a["nres"].__setitem__(3, L.QMAX + 1)),
        "arena header": _mut(b, "arena", lambda a, c: a.__setitem__(offs[5], a[offs[5]] | (200 << 16))),
        "slot record": _mut(b, "arena", lambda a, c: a.__setitem__(
            offs[with_slots] + _slotoff_word(a, offs[with_slots]), 10 ** 9)),
        "regex column": _mut(b, "res", lambda a, c: a["col"].__setitem__(
            tuple(np.argwhere(ent)[0]), b.rx.shape[0])),
        "context slot": _mut(b, "res", lambda a, c: a["slot_a"].__setitem__((0, with_slots), 200)),
        "candidate layout": _mut(b, "cand", lambda a, c: setattr(c, "cand_wr", c.cand_wp)),
        "regex rows": _mut(b, "rx", lambda a, c: setattr(c, "rx", a[:, :max(_rows(cs) - 1, 0)].copy())),
        "request line": _mut(b, "lines", lambda a, c: a["h"]["arena_off"].__setitem__(7, a["h"]["arena_off"][7] + 1)),
        "request line attribute": _mut(b, "lines", lambda a, c: a["res"]["col"].__setitem__((2, 0), 7)),
        # a column an RES_RX_SAFE attribute names must hold no throwing / host cell
        "rx safe": _mut(b, "rx", lambda a, c: a.__setitem__((safe_col, 0), a[safe_col, 0] | 4)),
    }
    assert b.lines is not None
    for what, c in bad.items():
        c.n = b.n
        assert _check(lib, cs, c) != 0, what
        assert "malformed batch" in native.last_error(lib), what


def _slotoff_word(a, o):
    c0 = int(a[o])
    ng, nre, nro = c0 & 0xFF, (c0 >> 8) & 0xFF, c0 >> 24
    nh = (int(a[o + 1]) >> 8) & 0xFF
    return 2 + 3 * ng + 2 * nre + nro + nh


def test_corrupt_images_refused_before_device_work(lib):
    cs = compiler.compile_store(store.populate(synth.c2_store()), FULL_URNS, DEFAULT_CAS)
    blob = bytearray(compiler.store_blob(cs))
    hdr = np.frombuffer(bytes(blob[:64]), np.uint32)
    n_sets, n_pols = int(hdr[2]), int(hdr[3])
    rec = L.NODE_DT.itemsize
    set0, pol0 = 64, 64 + ((n_sets * rec + 15) & ~15)

    def poke(off, field, value):
        b = bytearray(blob)
        arr = np.frombuffer(b, L.NODE_DT, count=1, offset=off).copy()
        arr[field] = value
        b[off:off + rec] = arr.tobytes()
        return bytes(b)

    bads = [poke(set0, "child_end", n_pols + 1), poke(pol0, "child_begin", 10 ** 6),
            poke(pol0 + rec, "res_off", 10 ** 8), poke(set0, "subj_n", 60000)]
    lib.acs_compile.restype = C.c_void_p
    for blob_bad in bads:
        rows = C.c_uint32()
        assert lib.acs_internal_check_blob(blob_bad, len(blob_bad), C.byref(rows)) != 0
        assert not lib.acs_compile(blob_bad, len(blob_bad), 0)
        assert "malformed image" in native.last_error(lib)


def test_acl_none_claim_checked_against_arena(lib):
    """ACL_NONE (K1 skips ACL-gated rules and ACL-inert sets for it) is recomputed from
    the request's arena — ACL instance lists, grants, role-scoping pairs — and a request whose
    ACLs could let a rule pass is refused; every ACL_NONE the codec writes passes."""
    lib.acs_internal_check_acl_none.argtypes = [C.POINTER(native.ReqBatchC), C.c_uint32]
    cs = compiler.compile_store(store.populate(synth.c3_adverse_store()), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 4000, "c3", seed=11, acl=0.5, classes=False)
    codec = NativeCodec(compiler.store_blob(cs))
    for k, v in sb.hrs_forests().items():
        codec.set_subject_scopes(k, v)
    nb = codec.encode(sb.json_text(), threads=2)
    s = native.batch_struct(nb, compact=True)
    assert lib.acs_internal_check_acl_none(C.byref(s), cs.id_user) == 0, native.last_error(lib)
    lines = nb.lines
    state = (lines["h"]["flags"] >> np.uint32(L.RQ_ACL_SHIFT)) & np.uint32(3)
    assert (state == L.ACL_NONE).sum() > 0
    # ACL_CONTINUE requests with ACL entities: claiming ACL_NONE for them is refused for those whose
    # ACLs can pass (an instance that is a grant's of the same entity, or the subject's)
    cont = np.flatnonzero((state == L.ACL_CONTINUE) & ((lines["ar1"] & np.uint32(0xFF)) != 0)
                          & ((lines["h"]["flags"] & np.uint32(L.RQ_ACT_RMD | L.RQ_ACT_CREATE)) != 0))
    assert len(cont) > 0
    refused = 0
    for i in cont[:40]:
        keep = lines["h"]["flags"][i]
        lines["h"]["flags"][i] = (keep & ~np.uint32(3 << L.RQ_ACL_SHIFT)) | np.uint32(L.ACL_NONE << L.RQ_ACL_SHIFT)
        s = native.batch_struct(nb, compact=True)
        if lib.acs_internal_check_acl_none(C.byref(s), cs.id_user) != 0:
            assert "ACL_NONE" in native.last_error(lib)
            refused += 1
        lines["h"]["flags"][i] = keep
    assert refused > 0
    codec.close()
