// TEST INFRASTRUCTURE: GpuAccessController's micro-batcher rejects a call whose request cannot be
// made into one JSON value at the call itself (no device needed: compileOnly), so it never joins a
// batch: a gRPC context Any value that is not one JSON value alone (the reference's JSON.parse in
// unmarshallProtobufAny throws; spliced, `1}},{"target":…` would add a request of its own), a
// BigInt, a cycle, a request JSON.stringify maps to undefined.
// usage: node microbatch_guard_run.js <snapshot.json>   -> prints {"rejected": [...names]}
'use strict';
const fs = require('fs');
const path = require('path');
const g = require(path.join(__dirname, '..', '..', 'access-control-srv_amd', 'napi', 'gpuCodec.js'));

const snap = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
const maps = new Map(snap.map((ps, i) => [
  's' + i, Object.assign({}, ps, { combinables: new Map((ps.combinables || []).map((p, j) => [
    'p' + j, Object.assign({}, p, { combinables: new Map((p.combinables || []).map((r, k) => ['r' + k, r])) })])) })]));
const ctl = new g.GpuAccessController(maps, JSON.parse(process.argv[3]), JSON.parse(process.argv[4]),
  { compileOnly: true });
const any = (t) => ({ type_url: 't', value: Buffer.from(t) });
const cyc = { target: {} };
cyc.self = cyc;
const calls = [
  () => ctl.isAllowedGrpc({ target: {}, context: { subject: any('1}},{"target":{},"context":{"a":1') } }),
  () => ctl.isAllowedGrpc({ target: {}, context: { subject: any('{"id":"x"},"extra":2') } }),
  () => ctl.whatIsAllowedGrpc({ target: {}, context: { resources: [any('[1')] } }),
  () => ctl.isAllowed({ target: {}, context: { n: BigInt(1) } }),
  () => ctl.isAllowed(cyc),
  () => ctl.whatIsAllowed(undefined),
];
(async () => {
  const names = [];
  for (const c of calls) {
    try {
      await c();
      names.push('resolved');
    } catch (e) {
      names.push(e.name);
    }
  }
  console.log(JSON.stringify({ rejected: names, queued: ctl._queues.isAllowed.length + ctl._queues.whatIsAllowed.length }));
})().catch((e) => { console.error(e && e.stack ? e.stack : e); process.exit(1); });
