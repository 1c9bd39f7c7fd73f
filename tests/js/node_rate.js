// MEASUREMENT HARNESS (tools/node_rate.py): requests/s of the drop-in from JS request objects in
// Node — the gRPC messages AccessControlService.isAllowed receives (context members as protobuf
// Any with JSON values, accessControlService.ts:62-65, 103-127) through
// GpuAccessController.isAllowedGrpc, micro-batched over one event-loop turn; the same requests
// as plain objects through isAllowed (micro-batched) and isAllowedBatch — each checked against
// the product's decisions for the same requests (expect.bin, written by the Python side).
// usage: node node_rate.js <dir> [repeats]
'use strict';
const fs = require('fs');
const path = require('path');
const g = require(path.join(__dirname, '..', '..', 'access-control-srv_amd', 'napi', 'gpuCodec.js'));

const dir = process.argv[2];
const repeats = +(process.argv[3] || 3);
const meta = JSON.parse(fs.readFileSync(path.join(dir, 'meta.json'), 'utf8'));
const snapshot = JSON.parse(fs.readFileSync(path.join(dir, 'store.json'), 'utf8'));

function toMaps(snap) {  // the reference's in-memory policySets Map (accessController.ts:32)
  const m = new Map();
  snap.forEach((ps) => {
    const pols = new Map();
    for (const p of ps.combinables) {
      const rules = new Map();
      for (const r of p.combinables) rules.set(r.id, r);
      pols.set(p.id, Object.assign({}, p, { combinables: rules }));
    }
    m.set(ps.id, Object.assign({}, ps, { combinables: pols }));
  });
  return m;
}

const DEC = { PERMIT: 2, DENY: 3, NOT_APPLICABLE: 4, INDETERMINATE: 5, UNRECOGNIZED: 6 };
const now = () => Number(process.hrtime.bigint()) / 1e9;

(async () => {
  const ctl = new g.GpuAccessController(toMaps(snapshot), meta.urns, meta.cas,
    { threads: meta.threads, batchMax: meta.batchMax, pipelineBytes: null });
  // the per-subject HR forests (createHRScope's cache): one per (scope org, role)
  for (const line of fs.readFileSync(path.join(dir, 'forests.tsv'), 'utf8').split('\n')) {
    if (!line) continue;
    const tab = line.indexOf('\t');
    ctl.setSubjectScopes(line.slice(0, tab), line.slice(tab + 1));
  }
  const objs = JSON.parse(fs.readFileSync(path.join(dir, 'requests.json'), 'utf8'));
  const expect = fs.readFileSync(path.join(dir, 'expect.bin'));
  // the gRPC messages (decoded protobuf): context members as Any, resources a repeated Any
  const anyOf = (x) => ({ type_url: 'type.googleapis.com/google.protobuf.Struct', value: Buffer.from(JSON.stringify(x)) });
  const grpc = objs.map((r) => ({ target: r.target, context: { subject: anyOf(r.context.subject),
                                                               resources: r.context.resources.map(anyOf) } }));
  const check = (out) => {
    let bad = 0;
    for (let i = 0; i < out.length; ++i) if (out[i] instanceof Error || DEC[out[i].decision] !== expect[i]) ++bad;
    return bad;
  };
  const settle = (p) => p.then((x) => x, (e) => e);
  const runs = {
    grpc_micro: () => Promise.all(grpc.map((r) => settle(ctl.isAllowedGrpc(r)))),
    objects_micro: () => Promise.all(objs.map((r) => settle(ctl.isAllowed(r)))),
    objects_batch: () => ctl.isAllowedBatch(objs),
  };
  const res = { requests: objs.length, threads: meta.threads, batchMax: meta.batchMax, node: process.version };
  for (const [name, fn] of Object.entries(runs)) {
    const mismatches = check(await fn());  // warm: codec caches, page-locked blocks
    let best = Infinity;
    for (let k = 0; k < repeats; ++k) {
      const t0 = now();
      await fn();
      best = Math.min(best, now() - t0);
    }
    res[name] = { requests_per_s: objs.length / best, seconds: best, mismatches };
    console.error(`[node_rate] ${name}: ${(objs.length / best / 1e6).toFixed(3)} M req/s, ${mismatches} mismatches`);
  }
  ctl.close();
  console.log(JSON.stringify(res));
})().catch((e) => { console.error(e && e.stack ? e.stack : e); process.exit(1); });
