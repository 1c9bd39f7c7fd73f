"""The compact batch form (acs_layout.h: request lines + extension records, no SoA rows) on
the GPU, through the C ABI: every kernel decides it exactly as the SoA form, from device
buffers and from host buffers; the native codec's batches (compact, page-locked) and the
decision pipeline (acs_pipeline: chunked encode overlapped with device work) give the
records of the SoA path and the oracle."""
import json

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

import randgen  # noqa: E402
from diff_utils import gpu_outcome, oracle_outcome, build  # noqa: E402
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS  # noqa: E402
from oracle.jsval import OracleUnsupported  # noqa: E402
from acs_mi355x import compiler, encoder, native, store, synth, layout as L  # noqa: E402
from acs_mi355x.codec import NativeCodec, Pipeline  # noqa: E402
from acs_mi355x.device import (DeviceBatch, is_allowed_device, what_is_allowed_device,  # noqa: E402
                               decisions_from_tensor)


@pytest.fixture(scope="module", autouse=True)
def gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    native.load()


def _u64(d):
    return np.ascontiguousarray(d).view(np.uint64)


def test_compact_equals_soa_random_stores_gpu():
    """Random stores with wide requests (tails past the line: attributes 4.., subjects 2..,
    actions 1.., roles 2..): K1 / K2 on the compact form == the SoA form, device and host."""
    checked = tails = 0
    for s in range(0, 160, 2):
        urns, doc, reqs = randgen.rand_case(s)
        try:
            o, cs = build(urns, doc)
        except Exception:
            continue
        b = encoder.Encoder(cs).encode(reqs)
        tails += int((b.lines["ext"] != 0).sum())
        t = native.Tables(compiler.store_blob(cs), 0)
        soa = decisions_from_tensor(is_allowed_device(t, DeviceBatch(b, 0, compact=False)))
        cmp_ = decisions_from_tensor(is_allowed_device(t, DeviceBatch(b, 0, compact=True)))
        assert np.array_equal(_u64(soa), _u64(cmp_)), s
        assert np.array_equal(_u64(t.is_allowed(b, compact=True)), _u64(soa)), s
        w_soa = [x.cpu().numpy() for x in what_is_allowed_device(t, DeviceBatch(b, 0, compact=False))]
        w_cmp = [x.cpu().numpy() for x in what_is_allowed_device(t, DeviceBatch(b, 0, compact=True))]
        assert np.array_equal(w_soa[0], w_cmp[0]) and np.array_equal(w_soa[2], w_cmp[2]), s
        assert np.array_equal(w_soa[3], w_cmp[3]), s
        t.close()
        checked += 1
    assert checked >= 60 and tails > 0


@pytest.mark.parametrize("kind", ["c2", "c3"])
def test_codec_batches_and_pipeline_gpu(kind):
    """JSON -> native codec (compact, page-locked) -> acs_is_allowed, and the same text
    through acs_pipeline in small chunks (many overlapped chunks), equal the packed synthetic
    batch's records and the oracle on a sample."""
    doc = synth.c2_store() if kind == "c2" else synth.c3_store()
    cs = compiler.compile_store(store.populate(doc), FULL_URNS, DEFAULT_CAS)
    n = 50_000 if kind == "c2" else 20_000
    sb = synth.requests(cs, n, kind, seed=5)
    idx = np.arange(n)
    text = sb.json_text(idx)
    t = native.Tables(compiler.store_blob(cs), 0)
    want = t.is_allowed(sb.batch)
    codec = NativeCodec(compiler.store_blob(cs))
    if kind != "c2":
        for k, v in sb.hrs_forests(idx).items():
            codec.set_subject_scopes(k, v)
    b = codec.encode(text, threads=4)
    assert np.array_equal(_u64(t.is_allowed(b)), _u64(want))
    st2 = codec.encode(text, threads=4).stats()
    assert st2["classes_new"] == 0  # every class row came from the codec's cache
    for chunk in (4096, 7777):
        p = Pipeline(t, codec, threads=4, chunk=chunk)
        got, st = p.is_allowed(text, n)
        p.close()
        assert len(got) == n and st["chunks"] == -(-n // chunk)
        assert np.array_equal(_u64(got), _u64(want)), chunk
    o, _ = build(FULL_URNS, doc)
    rng = np.random.default_rng(1)
    for i in rng.choice(n, 300, replace=False):
        try:
            assert gpu_outcome(cs, want[i]) == oracle_outcome(o, sb.decode(int(i))), i
        except OracleUnsupported:
            pass
    b.close()
    codec.close()
    t.close()


def test_pipeline_errors_and_host_requests_gpu():
    """A malformed array is an error; too small an output reports the count; requests the
    packed form cannot carry come back flagged for the host path."""
    cs = compiler.compile_store(store.populate(synth.c2_store()), FULL_URNS, DEFAULT_CAS)
    t = native.Tables(compiler.store_blob(cs), 0)
    codec = NativeCodec(compiler.store_blob(cs))
    p = Pipeline(t, codec, threads=2, chunk=3)
    with pytest.raises(RuntimeError):
        p.is_allowed(b"[1,", 4)
    with pytest.raises(RuntimeError):
        p.is_allowed(b"[{}, {}, {}]", 2)
    reqs = [{"target": {"subjects": [], "resources": [], "actions": []},
             "context": {"subject": {"token": "t"}}}, {}, {"target": None}]
    got, st = p.is_allowed(json.dumps(reqs).encode(), 3)
    assert (got["flags"][0] & L.OF_HOST_REQ) and st["host_requests"] == 1
    assert got["flags"][2] & L.OF_NO_TARGET
    want = codec.encode(json.dumps(reqs).encode()).host_reasons
    assert p.host_reasons == want and list(want) == [0] and want[0]
    got, _ = p.is_allowed(b"[]", 0)
    assert len(got) == 0
    p.close()
    codec.close()
    t.close()


def test_pipeline_error_mid_run_then_single_request_gpu():
    """Round-3 advisor / round-4 verdict: an item that only fails in the codec (malformed JSON inside
    a well-delimited array) in the SECOND chunk — with the first chunk already in flight — fails
    the call; the pipeline drains (pipeline_reset), and the next call, one request, gets exactly
    its own record, not a stale record of the failed run."""
    cs = compiler.compile_store(store.populate(synth.c2_store()), FULL_URNS, DEFAULT_CAS)
    t = native.Tables(compiler.store_blob(cs), 0)
    codec = NativeCodec(compiler.store_blob(cs))
    sb = synth.requests(cs, 64, "c2", seed=9)
    items = [sb.json_text(np.array([i])).decode()[1:-1] for i in range(8)]
    want = t.is_allowed(codec.encode(("[" + ",".join(items) + "]").encode()))
    p = Pipeline(t, codec, threads=2, chunk=3)
    bad = items[:4] + ['{"target": {"subjects": [}, "context": {}}'] + items[5:]
    with pytest.raises(RuntimeError):
        p.is_allowed(("[" + ",".join(bad) + "]").encode(), len(bad))
    for k in (7, 2, 0):
        got, st = p.is_allowed(("[" + items[k] + "]").encode(), 1)
        assert len(got) == 1 and st["chunks"] == 1
        assert _u64(got)[0] == _u64(want)[k], k
    got, _ = p.is_allowed(("[" + ",".join(items) + "]").encode(), len(items))  # the whole run still works
    assert np.array_equal(_u64(got), _u64(want))
    p.close()
    codec.close()
    t.close()


def test_chunked_host_path_gpu(monkeypatch):
    """acs_is_allowed on one device in overlapped chunks (ACS_OPT_CHUNK: each chunk uploaded as a
    shard, the class / role rows once per call, two streams) equals one upload and one launch:
    a c3 batch with composed rows and the encoder's coherence order in 9 and 16 chunks (a batch is
    cut only into 8 chunks or more), a
    role-factor batch, and random stores' wide requests (extension records, arena tails) in
    chunks of a few requests."""
    cs = compiler.compile_store(store.populate(synth.c3_store()), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 600_000, "c3", seed=31, second_role=0.5)
    t = native.Tables(compiler.store_blob(cs), 0)
    t.set_chunk(0)
    want = t.is_allowed(sb.batch, compact=True)
    dev = decisions_from_tensor(is_allowed_device(t, DeviceBatch(sb.batch, 0, compact=True)))
    assert np.array_equal(_u64(want), _u64(dev))
    for c in (65_000, 30_000):
        t.set_chunk(c)
        assert np.array_equal(_u64(t.is_allowed(sb.batch, compact=True)), _u64(want)), c
    t.close()
    from acs_mi355x import candidates
    monkeypatch.setattr(candidates, "FORCE_LEVEL", "entity+action")
    rb = synth.requests(cs, 40_000, "c3", seed=32, tree=synth.OrgTree(fanout=4, depth=5))
    assert rb.batch.role_key is not None
    t = native.Tables(compiler.store_blob(cs), 0)
    t.set_chunk(0)
    want = t.is_allowed(rb.batch, compact=True)
    t.set_chunk(4000)
    assert np.array_equal(_u64(t.is_allowed(rb.batch, compact=True)), _u64(want))
    t.close()
    monkeypatch.undo()
    checked = 0
    for s in range(1, 80, 3):
        urns, doc, reqs = randgen.rand_case(s)
        try:
            _, rcs = build(urns, doc)
        except Exception:
            continue
        b = encoder.Encoder(rcs).encode(reqs)
        if b.n < 8:
            continue
        t = native.Tables(compiler.store_blob(rcs), 0)
        t.set_chunk(0)
        want = t.is_allowed(b, compact=True)
        t.set_chunk(max(1, b.n // 9))
        assert np.array_equal(_u64(t.is_allowed(b, compact=True)), _u64(want)), s
        t.close()
        checked += 1
    assert checked >= 10
