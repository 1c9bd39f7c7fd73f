"""napi/gpuCodec.js — the JS drop-in a TypeScript host loads — driven from Node.

CPU: the JS snapshot of a policySets Map (Maps rebuilt from the store's JSON), compiled by
acs_store_compile through the addon, is byte-identical to the Python compiler's image for
every golden fixture, 200 randomised stores and the c2 / c3 configurations; the addon's
encode() flags the same requests for the host as the Python binding.

GPU: JSON requests -> GpuAccessController.isAllowedBatch / whatIsAllowedBatch -> the
reference's Response / ReverseQuery objects equal the Python product's decoding of the
same requests (and the golden vectors' expectations, and the oracle on randomised stores);
the per-subject HR-scope registry, eviction, host routing and refresh.
"""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from acs_mi355x import build, compiler, encoder, results, store, synth
from acs_mi355x.codec import NativeCodec
from acs_mi355x.jsops import Unsupported
from kat_utils import load_kats, load_fixture, urns_for, check_asserts
from diff_utils import norm_rq, oracle_outcome, gpu_outcome
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS, Oracle
from oracle.jsval import OracleUnsupported
import randgen

NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None or not (os.path.exists("/usr/include/node/node_api.h")
                                                     or os.path.exists(build.NAPI_OUT)),
                                reason="no node / N-API addon")
RUNNER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "js", "gpu_codec_run.js")


def _addon():
    if os.path.exists("/usr/include/node/node_api.h"):
        build.build_napi()
    assert os.path.exists(build.NAPI_OUT)


def _case(policy_sets, urns, ia, wa=(), **kw):
    return {"snapshot": json.loads(compiler.snapshot_json(policy_sets)), "urns": urns, "cas": DEFAULT_CAS,
            "isAllowed": list(ia), "whatIsAllowed": list(wa), **kw}


def _run(tmp, cases, mode, timeout=600):
    _addon()
    tmp.joinpath("cases.json").write_text(json.dumps(cases))
    r = subprocess.run([NODE, RUNNER, str(tmp), mode], capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, (r.returncode, r.stderr[-4000:])
    out = json.loads(tmp.joinpath("out.json").read_text())
    if mode == "decide":  # every case also ran through the pipeline on a two-replica handle
        for k, res in enumerate(out):
            assert "compileError" in res or (res["pipelineSame"] and res["devices"] == [0, 0]), k
    return out


def _kat_groups():
    by_fx = {}
    for v in load_kats():
        by_fx.setdefault((v["fixture"], v["urns"]), []).append(v)
    return by_fx


# ---------------------------------------------------------------------------- CPU
def test_js_snapshot_compile_byte_identical(tmp_path):
    stores = []
    for (fx, _), vecs in _kat_groups().items():
        stores.append((store.populate(load_fixture(fx)), urns_for(vecs[0]), [v["request"] for v in vecs]))
    for s in range(200):
        urns, doc, reqs = randgen.rand_case(s)
        stores.append((store.populate(doc), urns, reqs))
    for doc in (synth.c2_store(), synth.c3_store()):
        stores.append((store.populate(doc), FULL_URNS, []))
    out = _run(tmp_path, [_case(m, u, reqs) for m, u, reqs in stores], "compile")
    compiled = 0
    for k, ((m, u, reqs), got) in enumerate(zip(stores, out)):
        try:
            want = compiler.store_blob(compiler.compile_store(m, u, DEFAULT_CAS))
        except Unsupported:
            assert "compileError" in got, k
            continue
        assert "compileError" not in got, (k, got)
        assert tmp_path.joinpath(f"blob_{k}.bin").read_bytes() == want, k
        nb = NativeCodec(want).encode(reqs, threads=2)
        assert got["info"]["n"] == len(reqs)
        assert sorted(int(i) for i in got["info"]["host"]) == sorted(nb.host_reasons), k
        compiled += 1
    assert compiled >= 150


# ---------------------------------------------------------------------------- GPU
def _gpu():
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from acs_mi355x import native
    native.load()
    return native


def _strip(x):
    """Node's encoding of one result, host reasons dropped (the two encoders word them differently)."""
    if isinstance(x, dict) and "$error" in x:
        return {"$error": x["$error"]}
    return x


def _py_results(native, cs, ia, wa):
    """The Python product's decoding of the same requests (encoder.py + C ABI + results.py)."""
    t = native.Tables(compiler.store_blob(cs), 0)
    out_ia, out_wa = [], []
    if ia:
        b = encoder.Encoder(cs).encode(ia)
        dec = t.is_allowed(b)
        for i in range(len(ia)):
            try:
                out_ia.append(norm_rq(results.decision_record(cs, dec[i], b.host_reasons.get(i))))
            except results.HostPathRequired:
                out_ia.append({"$error": "HostPathRequired"})
            except results.EvaluationError as e:
                out_ia.append({"$error": e.kind})
    if wa:
        b = encoder.Encoder(cs).encode(wa)
        bits, obl, obl_n, out = t.what_is_allowed(b)
        long_logs = t.resolve_overflow(b, out)  # as the controller (and gpuCodec.js) do
        for i in range(len(wa)):
            log = long_logs[i] if i in long_logs else obl[i][:obl_n[i]]
            try:
                out_wa.append(norm_rq(results.reverse_query(cs, b.overlay, bits[i], log, out[i],
                                                            b.host_reasons.get(i))))
            except results.HostPathRequired:
                out_wa.append({"$error": "HostPathRequired"})
            except results.EvaluationError as e:
                out_wa.append({"$error": e.kind})
    t.close()
    return out_ia, out_wa


@pytest.mark.gpu
def test_js_controller_kats_gpu(tmp_path):
    native = _gpu()
    groups = list(_kat_groups().items())
    cases = []
    for (fx, _), vecs in groups:
        m = store.populate(load_fixture(fx))
        cases.append(_case(m, urns_for(vecs[0]), [v["request"] for v in vecs if v["op"] == "isAllowed"],
                           [v["request"] for v in vecs if v["op"] == "whatIsAllowed"]))
    out = _run(tmp_path, cases, "decide")
    checked = 0
    for ((fx, _), vecs), case, got in zip(groups, cases, out):
        cs = compiler.compile_store(store.populate(load_fixture(fx)), urns_for(vecs[0]), DEFAULT_CAS)
        want_ia, want_wa = _py_results(native, cs, case["isAllowed"], case["whatIsAllowed"])
        assert [_strip(x) for x in got["isAllowed"]] == want_ia, fx
        assert [_strip(x) for x in got["whatIsAllowed"]] == want_wa, fx
        ia = [v for v in vecs if v["op"] == "isAllowed"]
        for v, r in zip(ia, got["isAllowed"]):
            if "$error" in r:
                assert fx == "conditions.yml" and r["$error"] == "HostPathRequired", (v["spec"], r)
                continue
            assert r["decision"] == v["expect"]["decision"], v["spec"]
            checked += 1
        wa = [v for v in vecs if v["op"] == "whatIsAllowed"]
        for v, r in zip(wa, got["whatIsAllowed"]):
            assert check_asserts(r, v["expect"]["asserts"]) == [], v["spec"]
            checked += 1
    assert checked >= 100


@pytest.mark.gpu
def test_js_controller_random_stores_gpu(tmp_path):
    native = _gpu()
    seeds, cases = [], []
    for s in range(0, 240, 2):
        urns, doc, reqs = randgen.rand_case(s)
        try:
            compiler.compile_store(store.populate(doc), urns, DEFAULT_CAS)
        except Unsupported:
            continue
        seeds.append((s, urns, doc, reqs))
        cases.append(_case(store.populate(doc), urns, reqs, reqs))
    out = _run(tmp_path, cases, "decide")
    vs_oracle = 0
    for (s, urns, doc, reqs), case, got in zip(seeds, cases, out):
        cs = compiler.compile_store(store.populate(doc), urns, DEFAULT_CAS)
        want_ia, want_wa = _py_results(native, cs, reqs, reqs)
        assert [_strip(x) for x in got["isAllowed"]] == want_ia, s
        assert [_strip(x) for x in got["whatIsAllowed"]] == want_wa, s
        o = Oracle(urns=urns)
        o.load(doc)
        for req, r in zip(reqs, got["isAllowed"]):
            if r.get("$error") == "HostPathRequired":
                continue
            try:
                want = oracle_outcome(o, req)
            except OracleUnsupported:
                continue
            if "$error" in r:
                assert want == ("ERR", r["$error"]), (s, r, want)
            else:
                ec = r.get("evaluation_cacheable", "undefined")
                assert want == ("OK", r["decision"], ec, r["operation_status"]["code"]), (s, r, want)
            vs_oracle += 1
    assert len(seeds) >= 80 and vs_oracle >= 500


@pytest.mark.gpu
def test_js_controller_synthetic_gpu(tmp_path):
    """c2: 20k JSON requests through Node = the C ABI's decisions on the packed batch; c3 with
    the per-subject HR-scope registry ($hrs), eviction to the host evaluator, and refresh."""
    native = _gpu()
    cs2 = compiler.compile_store(store.populate(synth.c2_store()), FULL_URNS, DEFAULT_CAS)
    sb2 = synth.requests(cs2, 20_000, "c2", seed=31)
    reqs2 = [sb2.decode(i) for i in range(sb2.batch.n)]
    cs3 = compiler.compile_store(store.populate(synth.c3_store()), FULL_URNS, DEFAULT_CAS)
    sb3 = synth.requests(cs3, 600, "c3", seed=32)
    inline = [json.loads(json.dumps(sb3.decode(i))) for i in range(sb3.batch.n)]
    by_ref, scopes = [], {}
    for r in inline:
        r = json.loads(json.dumps(r))
        subj = r["context"]["subject"]
        f = json.dumps(subj.pop("hierarchical_scopes"), sort_keys=True)
        key = next((k for k, v in scopes.items() if v == f), None) or f"subject-{len(scopes)}"
        scopes[key] = f
        subj["$hrs"] = key
        by_ref.append(r)
    k0 = by_ref[0]["context"]["subject"]["$hrs"]
    cases = [_case(store.populate(synth.c2_store()), FULL_URNS, reqs2, reqs2[:500], refreshTwice=True),
             _case(store.populate(synth.c3_store()), FULL_URNS, by_ref, by_ref[:100],
                   scopes={k: json.loads(v) for k, v in scopes.items()}, evict=[k0], hostEvaluator=True)]
    out = _run(tmp_path, cases, "decide", timeout=900)
    # c2: every request decided on the GPU, equal to the Python product (and to the packed batch)
    t = native.Tables(compiler.store_blob(cs2), 0)
    packed = t.is_allowed(sb2.batch)
    t.close()
    want_ia, want_wa = _py_results(native, cs2, reqs2, reqs2[:500])
    assert [_strip(x) for x in out[0]["isAllowed"]] == want_ia
    assert [_strip(x) for x in out[0]["whatIsAllowed"]] == want_wa
    assert out[0]["afterRefresh"] == out[0]["isAllowed"] and out[0]["stats"]["compiles"] == 2
    assert [gpu_outcome(cs2, d)[1] for d in packed[:2000]] == [r["decision"] for r in out[0]["isAllowed"][:2000]]
    assert out[0]["stats"]["host"] == 0
    # c3 by reference == Python product on the inline forests
    want3, want3w = _py_results(native, cs3, inline, inline[:100])
    assert [_strip(x) for x in out[1]["isAllowed"]] == want3
    assert [_strip(x) for x in out[1]["whatIsAllowed"]] == want3w
    assert out[1]["evicted"] == [True]
    gone = {i for i, r in enumerate(by_ref) if r["context"]["subject"]["$hrs"] == k0}
    for i, r in enumerate(out[1]["afterEvict"]):
        if i in gone:
            assert r == {"host": "isAllowed", "keys": ["context", "target"]}, i
        else:
            assert r == out[1]["isAllowed"][i], i
    assert np.isfinite(out[1]["stats"]["requests"])
