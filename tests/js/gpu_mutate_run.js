// TEST INFRASTRUCTURE: the reference's in-memory store handlers (accessController.ts:897-937)
// through GpuAccessController on a policySets Map, one step at a time.
// usage: node gpu_mutate_run.js <dir> compile|decide|latency
//   <dir>/script.json: {doc: {policy_sets}, urns, cas, requests, steps: [{op, args}]}
//   compile: compileOnly controller; per step the image (blob_<k>.bin) and the refresh stats
//   decide:  per step isAllowedBatch(requests) (errors as {$error, reason}) + refresh stats
//   latency: the store, then one updateRule: the refresh after it vs a full refresh (ms)
// written to <dir>/out.json.  Called by tests/test_gpucodec_js.py.
'use strict';
const fs = require('fs');
const path = require('path');
const g = require(path.join(__dirname, '..', '..', 'access-control-srv_amd', 'napi', 'gpuCodec.js'));

const [dir, mode] = process.argv.slice(2);
const sc = JSON.parse(fs.readFileSync(path.join(dir, 'script.json'), 'utf8'));

// test/utils.ts:345-383: YAML-shaped documents -> Maps keyed by id (later duplicates overwrite)
const rulesMap = (p) => new Map((p.rules || []).map((r) => [r.id, r]));
const policy = (p) => Object.assign({}, p, { combinables: rulesMap(p) });
const policySet = (ps) => Object.assign({}, ps, { combinables: new Map((ps.policies || []).map((p) => [p.id, policy(p)])) });
const load = (doc) => new Map(doc.policy_sets.map((ps) => [ps.id, policySet(ps)]));
const enc = (x) => (x instanceof Error ? { $error: x.name, reason: x.reason } : x);

function apply(ctl, st) {
  const a = st.args;
  switch (st.op) {
    case 'updatePolicySet': return ctl.updatePolicySet(policySet(a[0]));
    case 'removePolicySet': return ctl.removePolicySet(a[0]);
    case 'updatePolicy': return ctl.updatePolicy(a[0], policy(a[1]));
    case 'removePolicy': return ctl.removePolicy(a[0], a[1]);
    case 'updateRule': return ctl.updateRule(a[0], a[1], a[2]);
    case 'removeRule': return ctl.removeRule(a[0], a[1], a[2]);
    case 'clearPolicies': return ctl.clearPolicies();
    default: throw new Error('unknown op ' + st.op);
  }
}

(async () => {
  const out = [];
  const maps = load(sc.doc);
  sc.doc = null; // the Maps hold the store (c5: 1M rules in the default V8 heap)
  if (mode === 'latency') {
    const t0 = Date.now();
    const ctl = new g.GpuAccessController(maps, sc.urns, sc.cas, { threads: 8 });
    const first = Date.now() - t0;
    // one batch's wall time (ms); the codec's class rows are cached across batches of one store
    const batch = async () => {
      const tb = process.hrtime.bigint();
      const r = await ctl.isAllowedBatch(sc.requests);
      return { ms: Number(process.hrtime.bigint() - tb) / 1e6, n: r.length };
    };
    const cold = await batch();
    const warm = await batch();
    const [sid, pid, rule] = sc.steps[0].args;
    ctl.updateRule(sid, pid, rule);
    const t1 = Date.now();
    ctl._sync();
    const incr = { ms: Date.now() - t1, stats: ctl.lastRefresh };
    // the first batch after the update recomputes the class rows (DESIGN §8.4), the next is warm
    const afterUpdate = await batch();
    const afterWarm = await batch();
    const t2 = Date.now();
    ctl.refresh(ctl.policySets);
    const full = { ms: Date.now() - t2, stats: ctl.lastRefresh };
    const r = await ctl.isAllowedBatch(sc.requests);
    out.push({ first_ms: first, incremental: incr, full_refresh: full, decided: r.length,
               batch_ms: { cold: cold.ms, warm: warm.ms, first_after_update: afterUpdate.ms,
                           second_after_update: afterWarm.ms, requests: warm.n } });
    ctl.close();
  } else {
    const ctl = new g.GpuAccessController(maps, sc.urns, sc.cas, { threads: 2, compileOnly: mode === 'compile' });
    for (let k = 0; k <= sc.steps.length; ++k) {
      if (k > 0) apply(ctl, sc.steps[k - 1]);
      const res = {};
      if (mode === 'compile') {
        ctl._sync();
        fs.writeFileSync(path.join(dir, 'blob_' + k + '.bin'), ctl.blob);
      } else {
        res.isAllowed = (await ctl.isAllowedBatch(sc.requests)).map(enc);
      }
      res.refresh = ctl.lastRefresh;
      out.push(res);
    }
    ctl.close();
  }
  fs.writeFileSync(path.join(dir, 'out.json'), JSON.stringify(out));
  console.log('gpu_mutate_run: done');
})().catch((e) => {
  console.error(e && e.stack ? e.stack : e);
  process.exit(1);
});
