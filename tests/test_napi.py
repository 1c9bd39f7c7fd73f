"""N-API addon (lib/acs_mi355x.node): loads in Node with the full surface (CPU), and
a Node-driven batch is bit-identical to the Python-driven C ABI (GPU)."""
import json
import os
import shutil
import subprocess

import numpy as np
import pytest

from acs_mi355x import build, compiler, store, synth
from oracle.acs_oracle import FULL_URNS, DEFAULT_CAS

NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None or not os.path.exists("/usr/include/node/node_api.h")
                                and not os.path.exists(build.NAPI_OUT), reason="no node / N-API headers")
RUNNER = os.path.join(os.path.dirname(os.path.abspath(__file__)), "js", "acs_napi_run.js")


def _addon():
    p = build.build_napi() if os.path.exists("/usr/include/node/node_api.h") else build.NAPI_OUT
    assert p and os.path.exists(p)
    return p


def test_addon_loads_with_surface():
    p = _addon()
    js = ("const a=require(process.argv[1]);"
          "console.log(JSON.stringify({keys:Object.keys(a).sort(),sizes:a.layoutSizes()}));"
          "let msg='';try{a.compile(new Uint8Array(64),0)}catch(e){msg=e.message};console.log(msg)")
    r = subprocess.run([NODE, "-e", js, p], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    info = json.loads(r.stdout.splitlines()[0])
    assert info["keys"] == sorted(["compileStore", "compile", "free", "codecCreate", "codecFree", "batchFree",
                                   "codecSetSubjectScopes",
                                   "codecEvictSubject", "codecEcValues", "encode", "batchInfo", "batchString",
                                   "decideAsync", "pipelineCreate", "pipelineFree", "pipelineDecideAsync",
                                   "storeBuilderCreate", "storeBuilderStage", "storeBuilderCompile", "storeBuilderFree",
                                   "devices", "isAllowed", "isAllowedAsync", "whatIsAllowed", "whatIsAllowedObl",
                                   "wordsPerRequest", "layoutSizes", "deviceCount", "lastError", "compileUpdate",
                                   "uploadBytes"])
    assert info["sizes"] == [64, 16, 16, 16, 8]
    assert "magic" in r.stdout.splitlines()[1]  # a bad image is rejected with acs_last_error's message


def _dump(tmp, cs, b):
    tmp.joinpath("blob.bin").write_bytes(compiler.store_blob(cs))
    for k in ("hdr", "res", "subj", "act", "roles", "arena", "rx", "cand"):
        tmp.joinpath(k + ".bin").write_bytes(np.ascontiguousarray(getattr(b, k)).tobytes())
    tmp.joinpath("meta.json").write_text(json.dumps({
        "n": b.n, "rxCols": int(b.rx.shape[0]), "rxRows": int(b.rx_rows), "candWords": int(b.cand.shape[1]),
        "candWp": int(b.cand_wp), "candWr": int(b.cand_wr), "candWsu": int(b.cand_wsu), "candWpu": int(b.cand_wpu),
        "candWv": int(b.cand_wv),
        "candRows": int(b.cand.shape[0])}))


@pytest.mark.gpu
def test_node_batch_matches_c_abi(tmp_path):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from acs_mi355x import native
    _addon()
    cs = compiler.compile_store(store.populate(synth.c2_store()), FULL_URNS, DEFAULT_CAS)
    sb = synth.requests(cs, 20_000, "c2", seed=99)
    _dump(tmp_path, cs, sb.batch)
    r = subprocess.run([NODE, RUNNER, str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    t = native.Tables(compiler.store_blob(cs), 0)
    want = t.is_allowed(sb.batch).view(np.uint8).reshape(-1)
    bits, obl, obl_n, out = t.what_is_allowed(sb.batch)
    pobl, pobl_n = t.what_is_allowed_obl(sb.batch, np.arange(16, dtype=np.uint32), 128, 3)
    t.close()
    assert np.array_equal(np.frombuffer(tmp_path.joinpath("obl_n.bin").read_bytes(), np.uint32), pobl_n.reshape(-1))
    # log entries past a range's count are unspecified (device scratch): compare the logs
    nobl = np.frombuffer(tmp_path.joinpath("obl.bin").read_bytes(), np.uint32).reshape(pobl.shape)
    for c in range(pobl.shape[0]):
        for j in range(pobl.shape[1]):
            k = min(int(pobl_n[c, j]), pobl.shape[2])
            assert np.array_equal(nobl[c, j, :k], pobl[c, j, :k]), (c, j)
    for f in ("out_sync.bin", "out_async.bin"):
        assert np.array_equal(np.frombuffer(tmp_path.joinpath(f).read_bytes(), np.uint8), want), f
    assert np.array_equal(np.frombuffer(tmp_path.joinpath("wia_bits.bin").read_bytes(), np.uint32),
                          bits.reshape(-1))
    assert np.array_equal(np.frombuffer(tmp_path.joinpath("wia_obl_n.bin").read_bytes(), np.uint32), obl_n)


def test_addon_checks_batch_sizes():
    """A plain-object batch whose arrays are shorter than n and its counts imply is refused
    (RangeError naming the field) before anything reads it; handles are type-checked."""
    p = _addon()
    js = r"""
const a = require(process.argv[1]);
const n = 4, ok = () => ({n, hdr: new Uint8Array(16*n), res: new Uint8Array(16*16*n), subj: new Uint8Array(8*8*n),
  act: new Uint8Array(8*4*n), roles: new Uint32Array(8*n), arena: new Uint32Array(8), rx: new Uint8Array(0)});
const out = [];
const tryit = (f) => { try { f(); out.push('ok'); } catch (e) { out.push(e.constructor.name + ':' + e.message); } };
for (const k of ['hdr', 'res', 'subj', 'act', 'roles']) { const b = ok(); b[k] = b[k].subarray(0, b[k].length - 1); tryit(() => a.isAllowed(null, b)); }
{ const b = ok(); b.rxCols = 3; b.rxRows = 2; tryit(() => a.isAllowed(null, b)); }
{ const b = ok(); b.cand = new Uint32Array(10); b.candRows = 3; b.candWords = 4; tryit(() => a.whatIsAllowed(null, b)); }
{ const b = ok(); const h = new Uint32Array(b.hdr.buffer); h[2] = 1000; tryit(() => a.isAllowed(null, b)); }
{ const b = ok(); b.hdr[4] = 17; tryit(() => a.isAllowed(null, b)); }
tryit(() => a.isAllowed(null, ok()));
tryit(() => a.encode({}, '[]'));
console.log(JSON.stringify(out));
"""
    r = subprocess.run([NODE, "-e", js, p], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    out = json.loads(r.stdout)
    for k, msg in zip(["hdr", "res", "subj", "act", "roles", "rx", "cand", "hdr.arena_off", "hdr counts"], out):
        assert msg.startswith("RangeError") and f"batch.{k} " in msg, (k, msg)
    assert out[9].startswith("TypeError") and "tables handle" in out[9]
    assert out[10].startswith("TypeError") and "codec handle" in out[10]


def test_addon_handle_lifecycle(tmp_path):
    """Handles are registry slots, not napi externals (napi/acs_napi.c "handles"): a freed
    handle throws on use and frees twice as a no-op, a batch keeps its freed codec working, a
    stale id does not reach a reused slot, and handles left live in the main thread and in
    worker_threads are released by each environment's cleanup hook — every run exits 0
    (Node 12's teardown use-after-free on externals, which this layout avoids, crashed ~1 in
    6 loaded runs)."""
    from acs_mi355x import compiler, store
    from kat_utils import load_fixture
    p = _addon()
    cs = compiler.compile_store(store.populate(load_fixture("simple_policies.yml")), FULL_URNS, DEFAULT_CAS)
    tmp_path.joinpath("blob.bin").write_bytes(compiler.store_blob(cs))
    js = r"""
const { Worker, isMainThread, parentPort, workerData } = require('worker_threads');
const fs = require('fs');
const a = require(workerData ? workerData.addon : process.argv[2]);
const blob = new Uint8Array(fs.readFileSync(workerData ? workerData.blob : process.argv[3]));
const req = JSON.stringify([{ target: { subjects: [], resources: [], actions: [] }, context: {} }]);
function round(live) {
  const out = [];
  const tryit = (f) => { try { const v = f(); out.push(v === undefined ? 'ok' : v); } catch (e) { out.push(e.constructor.name + ':' + e.message); } };
  const c = a.codecCreate(blob);
  const b = a.encode(c, req, 1);
  a.codecFree(c);
  tryit(() => a.batchInfo(b).n);            // the batch keeps its codec alive
  tryit(() => a.codecEcValues(c));          // the freed handle throws
  tryit(() => a.codecFree(c));              // freeing twice: no-op
  a.batchFree(b);
  tryit(() => a.batchInfo(b));
  const c2 = a.codecCreate(blob);           // may reuse the slot: the stale id must not name it
  tryit(() => a.codecEcValues(c));
  tryit(() => typeof a.codecEcValues(c2));
  for (let k = 0; k < live; ++k) a.encode(a.codecCreate(blob), req, 1);  // left for the cleanup hook
  return out;
}
if (isMainThread) {
  const res = { main: round(50) };
  let left = 2;
  for (let w = 0; w < 2; ++w) {
    const wk = new Worker(__filename, { workerData: { addon: process.argv[2], blob: process.argv[3] } });
    wk.on('message', (m) => { res['w' + w] = m; if (--left === 0) console.log(JSON.stringify(res)); });
  }
} else {
  parentPort.postMessage(round(20));
}
"""
    f = tmp_path.joinpath("life.js")
    f.write_text(js)
    for _ in range(3):
        r = subprocess.run([NODE, str(f), p, str(tmp_path.joinpath("blob.bin"))], capture_output=True, text=True,
                           timeout=120)
        assert r.returncode == 0, (r.returncode, r.stderr[-3000:])
        res = json.loads(r.stdout)
        for k in ("main", "w0", "w1"):
            o = res[k]
            assert o[0] == 1, (k, o)
            assert o[1] == "Error:codec handle already freed", (k, o)
            assert o[2] == "ok" and o[3].startswith("TypeError:batchInfo"), (k, o)
            assert o[4].startswith(("Error:codec handle already freed", "TypeError:expected a codec handle")), (k, o)
            assert o[5] == "string", (k, o)
