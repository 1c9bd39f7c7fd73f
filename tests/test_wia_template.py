"""whatIsAllowed templates (csrc/acs_eval.h: wia_template_set, what_is_allowed_tpl), CPU build of
the core: a request decided from its class template(s) plus its work rules gets exactly the
outputs of the full walk (inclusion rows, maskedProperty logs in push order, records) — random
stores (errors, conditions, multi-entity requests, regex cells, properties), and c4-shaped batches
with 1-2 role associations (composed class rows) from both encoders; most c4 requests are
templated."""
import ctypes as C

import numpy as np
import pytest

import host_core
import randgen
from diff_utils import build
from acs_mi355x import compiler, encoder, native, store, synth, layout as L
from acs_mi355x.codec import NativeCodec
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS


def _lib():
    lib = host_core.lib()
    vp = C.c_void_p
    lib.acs_host_wia_templates.argtypes = [vp, C.c_size_t, C.POINTER(native.ReqBatchC), vp, C.POINTER(C.c_uint32)]
    lib.acs_host_what_is_allowed_tpl.argtypes = [vp, C.c_size_t, C.POINTER(native.ReqBatchC), vp, vp, vp, vp, vp,
                                                 C.POINTER(C.c_size_t)]
    return lib


def templated_wia(cs, batch, compact):
    """(bits, obl, obl_n, out, templated requests, templates) through the template path."""
    from acs_mi355x.results import bits_layout
    lib = _lib()
    blob = compiler.store_blob(cs)
    s = host_core._struct(batch, compact)
    stride = C.c_uint32()
    assert lib.acs_host_wia_templates(blob, len(blob), C.byref(s), None, C.byref(stride)) == 0
    rows = int(s.cand_rows) if s.cand else 0
    tpl = np.zeros((max(rows, 1), stride.value), np.uint32)
    if s.cand and s.cand_wv:
        assert lib.acs_host_wia_templates(blob, len(blob), C.byref(s), tpl.ctypes.data, C.byref(stride)) == 0
    words = bits_layout(cs.n_sets, cs.n_pols, cs.n_rules)[2]
    n = batch.n
    bits = np.zeros((n, max(words, 1)), np.uint32)
    obl = np.zeros((n, L.OBL_MAX, 2), np.uint32)
    obl_n = np.zeros(n, np.uint32)
    out = np.zeros(n, L.DECISION_DT)
    k = C.c_size_t()
    assert lib.acs_host_what_is_allowed_tpl(blob, len(blob), C.byref(s), tpl.ctypes.data, bits.ctypes.data,
                                            obl.ctypes.data, obl_n.ctypes.data, out.ctypes.data, C.byref(k)) == 0
    return bits, obl, obl_n, out, k.value, tpl


def _same(got, want, ctx):
    bits, obl, obl_n, out = got[:4]
    wbits, wobl, wobl_n, wout = want
    assert np.array_equal(np.ascontiguousarray(out).view(np.uint64), np.ascontiguousarray(wout).view(np.uint64)), ctx
    assert np.array_equal(obl_n, wobl_n), ctx
    assert np.array_equal(bits, wbits), ctx
    for i in np.flatnonzero(obl_n):
        assert np.array_equal(obl[i, :obl_n[i]], wobl[i, :obl_n[i]]), (ctx, int(i))


def test_templates_equal_full_walk_random_stores():
    checked = templated = 0
    for seed in range(0, 240, 2):
        urns, doc, reqs = randgen.rand_case(seed)
        try:
            _, cs = build(urns, doc)
        except Exception:
            continue
        b = encoder.Encoder(cs).encode(reqs)
        got = templated_wia(cs, b, compact=False)
        _same(got, host_core.what_is_allowed(cs, b), seed)
        templated += got[4]
        checked += 1
    assert checked >= 60 and templated > 0


@pytest.mark.parametrize("second", [0.0, 0.5])
def test_templates_c4_both_encoders(second):
    cs = compiler.compile_store(store.populate(synth.c3_store()), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 3000, "c3", seed=21, second_role=second)
    got = templated_wia(cs, sb.batch, compact=False)
    _same(got, host_core.what_is_allowed(cs, sb.batch), ("synth", second))
    assert got[4] > 0.9 * sb.batch.n  # c4: nearly every request decided from templates
    codec = NativeCodec(compiler.store_blob(cs))
    for k, v in sb.hrs_forests().items():
        codec.set_subject_scopes(k, v)
    nb = codec.encode(sb.json_text(), threads=2)
    got = templated_wia(cs, nb, compact=True)
    _same(got, host_core.what_is_allowed(cs, nb, compact=True), ("codec", second))
    assert got[4] > 0.9 * nb.n
    nb.close()
    codec.close()


@pytest.mark.gpu
@pytest.mark.parametrize("second", [0.0, 0.5])
def test_templates_gpu_equal_full_walk(second):
    """K2 with the template pass (the product path for c4-shaped batches) equals the CPU build's
    full walk: rows, logs and records, synthetic (SoA + lines) and codec (compact) batches."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from acs_mi355x.device import DeviceBatch, what_is_allowed_device
    cs = compiler.compile_store(store.populate(synth.c3_store()), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 20_000, "c3", seed=23, second_role=second)
    t = native.Tables(compiler.store_blob(cs), 0)
    got = [x.cpu().numpy() for x in what_is_allowed_device(t, DeviceBatch(sb.batch, 0, compact=True))]
    want = host_core.what_is_allowed(cs, sb.batch)
    _same((got[0].view(np.uint32), got[1].view(np.uint32), got[2].view(np.uint32),
           got[3].reshape(-1).view(L.DECISION_DT)), want, ("device", second))
    _same(t.what_is_allowed(sb.batch), want, ("host buffers", second))
    codec = NativeCodec(compiler.store_blob(cs))
    for k, v in sb.hrs_forests().items():
        codec.set_subject_scopes(k, v)
    nb = codec.encode(sb.json_text(), threads=4)
    _same(t.what_is_allowed(nb), host_core.what_is_allowed(cs, nb, compact=True), ("codec", second))
    nb.close()
    codec.close()
    t.close()


@pytest.mark.gpu
def test_templates_gpu_stray_set_bits():
    """A caller's class rows with bits set past n_sets in the last word of the candidate-set
    section (padding, not sets): the template pass drops them (wia_template_kernel), so K2 with
    templates still equals the CPU build's full walk on the clean rows."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from acs_mi355x.device import DeviceBatch, what_is_allowed_device
    cs = compiler.compile_store(store.populate(synth.c3_store()), FULL_URNS, DEFAULT_CAS)
    assert cs.n_sets % 32, "the store must leave padding bits in its last set word"
    sb = synth.requests(cs, 8_000, "c3", seed=29, second_role=0.5)
    want = host_core.what_is_allowed(cs, sb.batch)
    pad = np.uint32((0xFFFFFFFF << (cs.n_sets & 31)) & 0xFFFFFFFF)
    sb.batch.cand[:, cs.n_sets // 32] |= pad
    t = native.Tables(compiler.store_blob(cs), 0)
    got = [x.cpu().numpy() for x in what_is_allowed_device(t, DeviceBatch(sb.batch, 0, compact=True))]
    _same((got[0].view(np.uint32), got[1].view(np.uint32), got[2].view(np.uint32),
           got[3].reshape(-1).view(L.DECISION_DT)), want, "stray set bits")
    t.close()


def _many_work_rules_store():
    """c3 store plus a last policy set whose one policy holds 400 property rules (10 entities x 40
    properties, no subjects, PERMIT / DENY alternating): a class of one of those entities reaches 40
    work rules there, more than K2 stages in one batch (23 at c3's row length, acs_kernels.hip
    what_is_allowed_tpl_staged)."""
    doc = synth.c3_store()
    ent = "urn:restorecommerce:acs:names:model:entity"
    prop = "urn:restorecommerce:acs:names:model:property"
    rules = []
    for e in range(10):
        for k in range(40):
            v = f"urn:restorecommerce:acs:model:ent{e}.Ent{e}"
            rules.append({"id": f"rw_{e}_{k}", "target": {"resources": [{"id": ent, "value": v},
                                                                        {"id": prop, "value": f"{v}#p{k}"}]},
                          "effect": "PERMIT" if k % 2 == 0 else "DENY", "evaluation_cacheable": False})
    doc["policy_sets"].append({"id": "s_work", "combining_algorithm":
                               "urn:oasis:names:tc:xacml:3.0:rule-combining-algorithm:deny-overrides",
                               "policies": [{"id": "p_work", "combining_algorithm":
                                             "urn:oasis:names:tc:xacml:3.0:rule-combining-algorithm:deny-overrides",
                                             "rules": rules}]})
    return doc


def test_templates_many_work_rules():
    """CPU build: the store with 40 work rules per class in one policy — templates equal the full
    walk."""
    cs = compiler.compile_store(store.populate(_many_work_rules_store()), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 3_000, "c3", seed=41, second_role=0.5)
    got = templated_wia(cs, sb.batch, compact=True)
    want = host_core.what_is_allowed(cs, sb.batch)
    _same(got[:4], want, "many work rules")
    assert got[4] > 0.5 * sb.batch.n


@pytest.mark.gpu
def test_templates_gpu_many_work_rules():
    """K2 with several staged batches of work rules per wave (40 work rules per class in one
    policy, more than one LDS batch holds) equals the CPU build's full walk: rows, logs and
    records."""
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from acs_mi355x.device import DeviceBatch, what_is_allowed_device
    cs = compiler.compile_store(store.populate(_many_work_rules_store()), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 20_000, "c3", seed=43, second_role=0.5)
    t = native.Tables(compiler.store_blob(cs), 0)
    got = [x.cpu().numpy() for x in what_is_allowed_device(t, DeviceBatch(sb.batch, 0, compact=True))]
    want = host_core.what_is_allowed(cs, sb.batch)
    _same((got[0].view(np.uint32), got[1].view(np.uint32), got[2].view(np.uint32),
           got[3].reshape(-1).view(L.DECISION_DT)), want, "many work rules, device")
    _same(t.what_is_allowed(sb.batch), want, "many work rules, host buffers")
    t.close()
