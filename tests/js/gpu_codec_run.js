// TEST INFRASTRUCTURE: drive napi/gpuCodec.js (GpuAccessController) the way a TS host would:
// policySets Maps + JSON requests in, the reference's Response / ReverseQuery objects out.
// usage: node gpu_codec_run.js <dir> compile|decide
//   <dir>/cases.json: [{snapshot, urns, cas, isAllowed: [req], whatIsAllowed: [req], scopes: {key: forest}}]
//   compile: per case, blob_<k>.bin (compileStore of the re-built Maps) + encode() host info
//   decide:  per case, isAllowedBatch / whatIsAllowedBatch results (errors as {$error, reason})
// written to <dir>/out.json.  Called by tests/test_gpucodec_js.py.
'use strict';
const fs = require('fs');
const path = require('path');
const g = require(path.join(__dirname, '..', '..', 'access-control-srv_amd', 'napi', 'gpuCodec.js'));

const [dir, mode] = process.argv.slice(2);
const cases = JSON.parse(fs.readFileSync(path.join(dir, 'cases.json'), 'utf8'));

// the snapshot arrays -> the reference's in-memory shape (Maps keyed by position, so
// duplicate or missing ids keep every entry)
function toMaps(snapshot) {
  const m = new Map();
  snapshot.forEach((ps, i) => {
    if (!ps) { m.set('s' + i, ps); return; }
    const pols = new Map();
    (ps.combinables || []).forEach((p, j) => {
      if (!p) { pols.set('p' + j, p); return; }
      const rules = new Map();
      (p.combinables || []).forEach((r, k) => rules.set('r' + k, r));
      pols.set('p' + j, Object.assign({}, p, { combinables: rules }));
    });
    m.set('s' + i, Object.assign({}, ps, { combinables: pols }));
  });
  return m;
}

const enc = (x) => (x instanceof Error ? { $error: x.name, reason: x.reason } : x);

(async () => {
  const out = [];
  for (let k = 0; k < cases.length; ++k) {
    const c = cases[k];
    const maps = toMaps(c.snapshot);
    if (mode === 'compile') {
      let blob;
      try {
        blob = g.addon.compileStore(g.snapshotStore(maps), JSON.stringify(c.urns), JSON.stringify(c.cas));
      } catch (e) {
        out.push({ compileError: e.message });
        continue;
      }
      fs.writeFileSync(path.join(dir, 'blob_' + k + '.bin'), blob);
      const codec = g.addon.codecCreate(blob);
      const b = g.addon.encode(codec, JSON.stringify(c.isAllowed), 2);
      out.push({ info: g.addon.batchInfo(b), ec: JSON.parse(g.addon.codecEcValues(codec)) });
      // half the handles are freed here, the rest by the environment's cleanup hook at exit
      if (k % 2) {
        g.addon.codecFree(codec); // the batch keeps the codec alive until it is freed
        g.addon.batchFree(b);
      }
      continue;
    }
    let ctl;
    const opts = { threads: 2 };
    try {
      if (c.hostEvaluator) opts.hostEvaluator = (op, req) => ({ host: op, keys: Object.keys(req).sort() });
      ctl = new g.GpuAccessController(maps, c.urns, c.cas, opts);
    } catch (e) {
      out.push({ compileError: e.message });
      continue;
    }
    for (const key of Object.keys(c.scopes || {})) ctl.setSubjectScopes(key, c.scopes[key]);
    const ia = await ctl.isAllowedBatch(c.isAllowed);
    const wa = await ctl.whatIsAllowedBatch(c.whatIsAllowed);
    const res = { isAllowed: ia.map(enc), whatIsAllowed: wa.map(enc), stats: ctl.stats };
    {  // single calls, micro-batched (one event-loop turn), and the same requests as gRPC
       // messages (context members as protobuf Any with JSON values): the same answers
      const settle = (p) => p.then((x) => x, (e) => e);
      const ia1 = await Promise.all(c.isAllowed.map((r) => settle(ctl.isAllowed(r))));
      const wa1 = await Promise.all(c.whatIsAllowed.map((r) => settle(ctl.whatIsAllowed(r))));
      // a request as the gRPC message it came from: context members as protobuf Any (resources a
      // repeated Any); requests without an object context (the service would pass {}, not what
      // the controller got) go as they are
      const grpcable = (r) => r && typeof r === 'object' && r.context && typeof r.context === 'object' &&
        !Array.isArray(r.context);
      const grpc = (r) => {
        const ctx = r.context;
        const out = { target: r.target };
        if (ctx) {
          out.context = {};
          const anyOf = (x) => ({ type_url: 't', value: Buffer.from(JSON.stringify(x)) });
          for (const k of Object.keys(ctx)) {
            const v = ctx[k];
            if (v === undefined) continue;
            out.context[k] = k === 'resources' && Array.isArray(v) ? v.map((x) => (x === undefined ? null : anyOf(x)))
              : anyOf(v);
          }
        }
        return out;
      };
      const ia2 = await Promise.all(c.isAllowed.map((r) => settle(grpcable(r) ? ctl.isAllowedGrpc(grpc(r))
        : ctl.isAllowed(r))));
      res.microSame = JSON.stringify(ia1.map(enc)) === JSON.stringify(res.isAllowed) &&
        JSON.stringify(wa1.map(enc)) === JSON.stringify(res.whatIsAllowed);
      res.grpcSame = JSON.stringify(ia2.map(enc)) === JSON.stringify(res.isAllowed);
      // a concurrent call whose Any value would splice a request of its own into the batch
      // (ADVICE r4): it rejects alone, and its neighbours get their own answers
      if (c.isAllowed.length >= 2 && grpcable(c.isAllowed[0]) && grpcable(c.isAllowed[1])) {
        const inj = '1}},{"target":' + JSON.stringify(c.isAllowed[1].target || {}) + ',"context":{"a":1';
        const bad = { target: c.isAllowed[0].target, context: { subject: { type_url: 't', value: Buffer.from(inj) } } };
        const r3 = await Promise.all([settle(ctl.isAllowedGrpc(grpc(c.isAllowed[0]))), settle(ctl.isAllowedGrpc(bad)),
          settle(ctl.isAllowedGrpc(grpc(c.isAllowed[1])))]);
        res.injectSafe = JSON.stringify(enc(r3[0])) === JSON.stringify(res.isAllowed[0]) &&
          r3[1] instanceof SyntaxError && JSON.stringify(enc(r3[2])) === JSON.stringify(res.isAllowed[1]);
      }
    }
    {  // the same requests through the decision pipeline (3-request chunks) on a handle
       // replicated twice on device 0: the same answers
      const opts2 = Object.assign({}, opts, { pipelineBytes: 0, chunk: 3, device: [0, 0] });
      const ctl2 = new g.GpuAccessController(maps, c.urns, c.cas, opts2);
      for (const key of Object.keys(c.scopes || {})) ctl2.setSubjectScopes(key, c.scopes[key]);
      const ia2 = await ctl2.isAllowedBatch(c.isAllowed);
      res.pipelineSame = JSON.stringify(ia2.map(enc)) === JSON.stringify(res.isAllowed);
      res.devices = ctl2.devices();
      ctl2.close();
    }
    if (c.evict) {
      res.evicted = c.evict.map((key) => ctl.evictSubject(key));
      res.afterEvict = (await ctl.isAllowedBatch(c.isAllowed)).map(enc);
    }
    if (c.refreshTwice) {  // a policy CRUD event: recompile, same answers
      ctl.refresh(maps);
      res.afterRefresh = (await ctl.isAllowedBatch(c.isAllowed)).map(enc);
    }
    ctl.close();
    out.push(res);
  }
  fs.writeFileSync(path.join(dir, 'out.json'), JSON.stringify(out));
  console.log(JSON.stringify({ ok: true, cases: cases.length }));
})().catch((e) => { console.error(e && e.stack ? e.stack : e); process.exit(1); });
