// TEST INFRASTRUCTURE: gpuCodec.grpcRequestJson vs the reference's own unmarshalling
// (src/accessControlService.ts:62-65, 103-127, restated with the same lodash functions) on
// random gRPC-shaped requests: Any members with JSON / empty / missing values, null members,
// array members before and after `resources` (the :106 quirk), objects as `resources`.
// usage: node grpc_json_run.js <cases>   -> prints {"checked": n}
'use strict';
const path = require('path');
const _ = { isArray: require('lodash.isarray'), map: require('lodash.map'), isEmpty: require('lodash.isempty') };
const { grpcRequestJson } = require(path.join(__dirname, '..', '..', 'access-control-srv_amd', 'napi', 'gpuCodec.js'));

// the reference (accessControlService.ts:62-65, 103-127)
function unmarshallProtobufAny(object) {
  if (!object || _.isEmpty(object.value)) return null;
  return JSON.parse(object.value.toString());
}
function unmarshallContext(context) {
  for (const prop in context) {
    if (_.isArray(context[prop])) context[prop] = _.map(context.resources, unmarshallProtobufAny);
    else context[prop] = unmarshallProtobufAny(context[prop]);
  }
  return context;
}
function reference(request) {
  return { target: request.target, context: request.context ? unmarshallContext(request.context) : {} };
}

let seed = 12345;
const rnd = () => ((seed = (seed * 1103515245 + 12345) >>> 0) / 4294967296);
const pick = (a) => a[Math.floor(rnd() * a.length)];
const jsonValue = () => pick([
  { id: 'u1', role_associations: [{ role: 'r1', attributes: [] }], hierarchical_scopes: [] },
  { id: 'res7', meta: { owners: [{ id: 'urn:o', value: 'urn:org', attributes: [{ id: 'urn:oi', value: 'org3' }] }] } },
  { a: [1, 2, { b: 'x"y\\\\z' }], u: 'ü€\\u2028' }, 'text', 42, true, null, [], {},
]);
const any = () => {
  const r = rnd();
  if (r < 0.1) return null;
  if (r < 0.2) return { type_url: 't', value: Buffer.alloc(0) };
  if (r < 0.25) return { type_url: 't' };
  if (r < 0.3) return { type_url: 't', value: '' };
  if (r < 0.35) return { type_url: 't', value: JSON.stringify(jsonValue()) };  // a string value
  // texts that are not one JSON value alone but splice into valid JSON: the reference throws
  if (r < 0.4) return { type_url: 't', value: Buffer.from(pick(['1}},{"target":{},"context":{"a":1', '1,"x":2', '"a"]', '[1', '1 2', '{}{}'])) };
  return { type_url: 't', value: Buffer.from(JSON.stringify(jsonValue())) };
};
function grpcRequest() {
  const req = {};
  if (rnd() < 0.9) req.target = { subjects: [{ id: 'urn:role', value: 'r' + Math.floor(rnd() * 3) }], resources: [], actions: [] };
  if (rnd() < 0.1) return req;  // no context
  const ctx = {};
  const props = [];
  for (const p of ['subject', 'resources', 'security', 'extra']) if (rnd() < 0.75) props.push(p);
  if (rnd() < 0.5) props.reverse();
  for (const p of props) {
    const r = rnd();
    if (p === 'resources' && r < 0.1) ctx[p] = { k1: any(), k2: any() };  // _.map over an object
    else if (r < 0.5 || p === 'resources') ctx[p] = Array.from({ length: Math.floor(rnd() * 3) }, any);
    else ctx[p] = any();
  }
  req.context = ctx;
  return req;
}

const n = +(process.argv[2] || 2000);
let checked = 0;
for (let k = 0; k < n; ++k) {
  const req = grpcRequest();
  // the reference mutates its context in place: evaluate it on a structural copy (Buffers kept)
  const clone = (v) => (Buffer.isBuffer(v) ? Buffer.from(v) : Array.isArray(v) ? v.map(clone)
    : v && typeof v === 'object' ? Object.fromEntries(Object.entries(v).map(([a, b]) => [a, clone(b)])) : v);
  let want, got;
  try {
    want = JSON.stringify(reference(clone(req)));
  } catch (e) {
    want = 'throws';
  }
  try {
    got = JSON.stringify(JSON.parse(grpcRequestJson(req)));
  } catch (e) {
    got = 'throws';
  }
  if (got !== want) {
    console.error(JSON.stringify({ case: k, want, got }));
    process.exit(1);
  }
  ++checked;
}
console.log(JSON.stringify({ checked }));
