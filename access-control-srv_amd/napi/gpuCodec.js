// gpuCodec.js — the JS side of the drop-in for a TypeScript access-control-srv host.
//
// GpuAccessController evaluates batches of the reference's isAllowed / whatIsAllowed requests
// (src/core/accessController.ts:88-324, :326-427) on the MI355X through lib/acs_mi355x.node
// (napi/acs_napi.c) and returns the reference's Response / ReverseQuery objects:
//
//   const { GpuAccessController } = require('.../napi/gpuCodec.js');
//   const gpu = new GpuAccessController(accessController.policySets, urnsConfig, casConfig,
//                                       { hostEvaluator: (op, req) => accessController[op](req) });
//   const responses = await gpu.isAllowedBatch(requests);        // Response | Error per request
//   const queries = await gpu.whatIsAllowedBatch(requests);      // ReverseQuery | Error
//   gpu.refresh(accessController.policySets);                    // after a policy CRUD event
//
// The policySets Map is snapshotted (snapshotStore) and compiled natively (acs_store_compile,
// byte-identical to acs_mi355x/compiler.py); requests go to the native codec as one JSON
// text (acs_codec_encode on the libuv pool) and straight on to the kernels (decideAsync);
// a batch of at least `pipelineBytes` of JSON goes through the decision pipeline instead
// (pipelineDecideAsync: encode of chunk k+1 overlapped with the device work of chunk k).
// `device` may be an array of device ids: one image per device, large batches split
// across them (acs_compile_multi).
// Requests the packed form cannot carry (a JS rule condition, a subject token to resolve, a
// RegExp outside the precomputed subset) go to
// `hostEvaluator` — normally the reference's own AccessController — or, without one, come
// back as HostPathRequired errors.  Node >= 12: no optional chaining, no structuredClone.
'use strict';

const path = require('path');

const addon = require(process.env.ACS_MI355X_ADDON ||
  path.join(__dirname, '..', 'lib', 'acs_mi355x.node'));

// csrc/acs_layout.h
const DECISIONS = [undefined, undefined, 'PERMIT', 'DENY', 'NOT_APPLICABLE', 'INDETERMINATE', 'UNRECOGNIZED'];
const OF_ERR = 0x01, OF_HOST_COND = 0x02, OF_HOST_REQ = 0x04, OF_NO_TARGET = 0x08, OF_OBL_OVERFLOW = 0x20;
const ERR_KINDS = { 1: 'TypeError', 2: 'InvalidCombiningAlgorithm', 3: 'SyntaxError', 4: 'RegexHost' };
const ERR_REGEX_HOST = 4;
const REC_BYTES = 8;
const OBL_MAX = 128; // ACS_OBL_MAX: (entity, mask) pairs per request in the whatIsAllowed log
const OVERFLOW_CAP = 1024, OVERFLOW_CHUNKS = 8;

class HostPathRequired extends Error {
  constructor(reason, ruleIndex) {
    super(reason);
    this.name = 'HostPathRequired';
    this.reason = reason;
    this.ruleIndex = ruleIndex;
  }
}

// The reference's promise would reject with this kind of error (TypeError from a null
// policy / malformed target, errors.InvalidCombiningAlgorithm, RegExp SyntaxError).
class GpuEvaluationError extends Error {
  constructor(kind) {
    super(kind);
    this.name = kind;
    this.kind = kind;
  }
}

function mapValues(m) {
  if (m instanceof Map) return Array.from(m.values());
  return Array.isArray(m) ? m : [];
}

function without(o, drop) {
  const out = {};
  for (const k of Object.keys(o)) if (drop.indexOf(k) < 0 && o[k] !== undefined) out[k] = o[k];
  return out;
}

// One policy set as an element of the snapshot acs_store_compile reads: the set with its
// `combinables` the array of its Map's values, each policy's likewise (null entries kept).
function snapshotSet(ps) {
  if (!ps || typeof ps !== 'object') return null;
  const s = without(ps, ['combinables', 'policies']);
  s.combinables = mapValues(ps.combinables).map((p) => {
    if (!p || typeof p !== 'object') return null;
    const po = without(p, ['combinables']);
    po.combinables = mapValues(p.combinables).map((r) => (r && typeof r === 'object' ? r : null));
    return po;
  });
  return s;
}

// The policySets Map as the JSON text acs_store_compile reads: the Map's values in order.
function snapshotStore(policySets) {
  return JSON.stringify(mapValues(policySets).map(snapshotSet));
}

const isNil = (v) => v === undefined || v === null; // lodash _.isNil

// The node order of the compiled image (acs_mi355x/compiler.py _compile_set/_assemble):
// sets in Map order, their policies flattened (null entries keep a slot), then rules.
function nodeIndex(policySets) {
  const sets = [], pols = [], rules = [], setPols = [], polRules = [];
  for (const ps of mapValues(policySets)) {
    const p0 = pols.length;
    for (const p of mapValues(ps && ps.combinables)) {
      const r0 = rules.length;
      pols.push(p || null);
      if (p) for (const r of mapValues(p.combinables)) rules.push(r || null);
      polRules.push([r0, rules.length]);
    }
    sets.push(ps);
    setPols.push([p0, pols.length]);
  }
  return { sets, pols, rules, setPols, polRules };
}

function parseRequests(requests) {
  if (Array.isArray(requests)) return requests;
  return JSON.parse(typeof requests === 'string' ? requests : Buffer.from(requests).toString('utf8'));
}

// lodash _.isEmpty for the values a protobuf Any's `value` can hold (Buffer / typed array /
// string: length; plain object: own keys; anything else: empty)
function isEmptyValue(v) {
  if (v === undefined || v === null) return true;
  if (typeof v === 'string' || Array.isArray(v) || ArrayBuffer.isView(v)) return v.length === 0;
  if (typeof v === 'object') return Object.keys(v).length === 0;
  return true;
}

// unmarshallProtobufAny (src/accessControlService.ts:116-127) as JSON text: null for a nil
// message or an empty value, else the value's text.  The reference JSON.parses that text alone
// and throws when it is not exactly one JSON value; it is parsed here alone too, so a value
// that only parses as part of the batch text (`1}},{"target":…` injecting a request of its
// own, or `1,"x":2` a context member) throws the same SyntaxError instead of being spliced.
function unmarshalText(x) {
  if (!x || isEmptyValue(x.value)) return 'null';
  const text = x.value.toString();
  JSON.parse(text);
  return text;
}

// The JSON text of the request AccessControlService.isAllowed / whatIsAllowed builds from a
// gRPC request (accessControlService.ts:62-65, 83-86: {target, context: unmarshallContext(
// context) or {}}), without parsing the context: its members are protobuf Any messages whose
// `value` already holds JSON text, which is spliced in as is.  The :106 quirk is kept: every
// array member becomes _.map(context.resources, unmarshallProtobufAny), of the resources as
// they are at that point (an array member after `resources` maps the already-unmarshalled
// resources: those are parsed back for it).  The spliced text must be JSON the reference's
// JSON.parse accepts: GpuAccessController.isAllowedGrpc re-runs a batch whose text does not
// parse request by request.
function grpcRequestJson(request) {
  const ctx = request.context;
  let body = '{}';
  if (ctx) {
    const done = new Map(); // member -> JSON text of its unmarshalled value
    for (const prop in ctx) {
      const x = ctx[prop];
      if (Array.isArray(x)) {
        const R = done.has('resources') ? JSON.parse(done.get('resources')) : ctx.resources;
        const list = Array.isArray(R) ? R : (R && typeof R === 'object' ? Object.values(R) : []);
        done.set(prop, '[' + list.map(unmarshalText).join(',') + ']');
      } else {
        done.set(prop, unmarshalText(x));
      }
    }
    const parts = [];
    for (const [k, v] of done) parts.push(JSON.stringify(k) + ':' + v);
    body = '{' + parts.join(',') + '}';
  }
  const target = request.target === undefined ? '' : '"target":' + JSON.stringify(request.target) + ',';
  return '{' + target + '"context":' + body + '}';
}

const clone = (v) => (v === undefined || v === null || typeof v !== 'object' ? v : JSON.parse(JSON.stringify(v)));

function pick(obj, keys, into) {
  for (const k of keys) if (k in obj) into[k] = clone(obj[k]);
  return into;
}

function ecDecoder(codec) {
  const extra = JSON.parse(addon.codecEcValues(codec));
  const table = [undefined, null, false, true].concat(extra);
  return (code) => (code < table.length ? table[code] : undefined);
}

class GpuAccessController {
  // urns: policies.options.urns (cfg/config.json:270-307) as an object or Map;
  // combiningAlgorithms: policies.options.combiningAlgorithms (array of {urn, method}).
  constructor(policySets, urns, combiningAlgorithms, options) {
    const o = options || {};
    this.device = o.device || 0; // a device id, or an array of them
    this.threads = o.threads || 4;
    this.chunk = o.chunk || 0; // pipeline chunk (requests); 0: the library's default
    this.pipelineBytes = o.pipelineBytes === undefined ? (1 << 20) : o.pipelineBytes; // null: never
    this.compileOnly = !!o.compileOnly; // compile the image only (no device): this.blob
    // the host edits rule / policy objects in place on the shared Map without the store
    // handlers or markChanged: every refresh re-serialises every set (the builder still
    // recompiles only the sets whose JSON text changed)
    this.mapEditsInPlace = !!o.mapEditsInPlace;
    this.pipeline = null;
    this.hostEvaluator = o.hostEvaluator || null;
    // micro-batching (SURVEY §8(f) rank 1): single isAllowed / whatIsAllowed calls — one per gRPC
    // request (accessControlService.ts:62-101) — are gathered over one event-loop turn
    // (batchWindowMs 0: setImmediate) or a window of batchWindowMs, at most batchMax at a time,
    // and decided as one batch; each promise resolves to its own Response / ReverseQuery
    this.batchMax = o.batchMax || 65536;
    this.batchWindowMs = o.batchWindowMs || 0;
    this._queues = { isAllowed: [], whatIsAllowed: [] };
    this._armed = { isAllowed: false, whatIsAllowed: false };
    this.urns = urns instanceof Map ? Object.fromEntries(urns) : urns;
    this.cas = combiningAlgorithms;
    this.stats = { requests: 0, host: 0, compiles: 0 };
    this.tables = null;
    this.codec = null;
    // incremental compile (acs_store_builder): one compiled fragment per policy set; a refresh
    // passes the sets it knows unchanged by their previous index, the others as JSON text
    this.builder = addon.storeBuilderCreate(JSON.stringify(this.urns), JSON.stringify(this.cas));
    this.setIndex = new Map(); // set key -> {obj, index} of the last compile
    this.dirty = new Set();    // set keys the mutators touched since (null: unknown, re-serialise all)
    this.stale = false;
    this.lastRefresh = null;   // {ms, recompiled, sets}
    this.refresh(policySets);
  }

  // Recompile from the (mutated) policySets Map; the reference re-reads its Map on every
  // request, so call this after each policy CRUD event (before the next batch).  `changed`
  // (optional): the ids of the policy sets the event touched; every other set still holding
  // the object it held at the last refresh is passed to the builder as unchanged (neither
  // re-serialised nor recompiled).  Without it every set is re-serialised, and the builder
  // still recompiles only the sets whose JSON text changed.
  //
  // A refresh that throws (a set that does not compile, a device failure) leaves the
  // controller stale: the next batch retries it, and succeeds once the store is fixed.  The
  // builder keeps the fragments of its last successful compile when a compile fails, and
  // setIndex always describes the builder's fragments, so the unchanged-set indices passed
  // to it stay valid either way.
  refresh(policySets, changed) {
    const t0 = Date.now();
    const dirty = changed && !this.mapEditsInPlace ? new Set(changed) : null;
    const entries = policySets instanceof Map ? Array.from(policySets.entries())
      : mapValues(policySets).map((ps, k) => [k, ps]);
    const items = new Array(entries.length);
    this.stale = true;
    for (let k = 0; k < entries.length; ++k) {
      const [key, ps] = entries[k];
      const prev = this.setIndex.get(key);
      // a changed set's text is staged at once (compiled, or matched to its unchanged fragment),
      // so no more than one set's JSON text is held at a time (c5: 1M rules in V8's default heap)
      items[k] = dirty && prev && prev.obj === ps && !dirty.has(key) ? prev.index
        : addon.storeBuilderStage(this.builder, JSON.stringify(snapshotSet(ps)));
    }
    const tStaged = Date.now();
    const r = addon.storeBuilderCompile(this.builder, items); // throws: the builder is unchanged
    const blob = r.blob;
    const tCompiled = Date.now();
    // the builder now holds this compile's fragments, in this Map order
    const setIndex = new Map();
    for (let k = 0; k < entries.length; ++k) setIndex.set(entries[k][0], { obj: entries[k][1], index: k });
    this.setIndex = setIndex;
    if (this.compileOnly) { // tooling: the image without a device (no tables / codec / pipeline)
      this.blob = blob;
      this._index = null; // built on the first whatIsAllowed (a refresh stays O(changed sets))
      this.stats.compiles += 1;
      this.policySets = policySets;
      this.dirty = new Set();
      this.stale = false;
      this.lastRefresh = { ms: Date.now() - t0, recompiled: r.recompiled, sets: entries.length };
      return;
    }
    // the previous image with only its changed blocks uploaded (acs_compile_update; replicas on
    // further devices take the primary's changed blocks device to device)
    const tables = this.tables ? addon.compileUpdate(this.tables, blob) : addon.compile(blob, this.device);
    const tDevice = Date.now();
    const codec = addon.codecCreate(blob);
    const tCodec = Date.now();
    const pipeline = this.pipelineBytes === null ? null : addon.pipelineCreate(tables, codec, this.threads, this.chunk);
    // the old handles: released once the batches still in flight are done with them
    if (this.pipeline) addon.pipelineFree(this.pipeline);
    if (this.tables) addon.free(this.tables);
    if (this.codec) addon.codecFree(this.codec);
    this.tables = tables;
    this.codec = codec;
    this.pipeline = pipeline;
    this.ec = ecDecoder(codec);
    this._index = null; // built on the first whatIsAllowed (a refresh stays O(changed sets))
    this.scopes = this.scopes || new Map();
    for (const [k, v] of this.scopes) addon.codecSetSubjectScopes(codec, k, v);
    this.stats.compiles += 1;
    this.policySets = policySets;
    this.dirty = new Set();
    this.stale = false;
    // phases (ms): the changed sets serialised and staged, the image compiled, the device image
    // updated, the request codec built for the new image
    this.lastRefresh = { ms: Date.now() - t0, recompiled: r.recompiled, sets: entries.length,
                         uploadBytes: addon.uploadBytes(tables),
                         phases: { stage: tStaged - t0, compile: tCompiled - tStaged, device: tDevice - tCompiled,
                                   codec: tCodec - tDevice } };
  }

  // node index of the compiled Map (whatIsAllowed's ReverseQuery assembly), built lazily: it
  // walks every rule, and isAllowed-only hosts never need it
  get index() {
    if (!this._index) this._index = nodeIndex(this.policySets);
    return this._index;
  }

  // The reference's in-memory store handlers (accessController.ts:897-937) on the Map this
  // controller compiled (the host's AccessController.policySets, shared): each mutates the
  // Map as the reference does and marks the touched set, and the next batch recompiles only
  // that set.  A host that mutates the Map itself calls markChanged(setId) instead.
  updatePolicySet(policySet) {
    this.policySets.set(policySet.id, policySet);
    this.markChanged(policySet.id);
  }

  removePolicySet(policySetID) {
    this.policySets.delete(policySetID);
    this.markChanged(null);
  }

  updatePolicy(policySetID, policy) {
    const ps = this.policySets.get(policySetID);
    if (!isNil(ps)) {
      ps.combinables.set(policy.id, policy);
      this.markChanged(policySetID);
    }
  }

  removePolicy(policySetID, policyID) {
    const ps = this.policySets.get(policySetID);
    if (!isNil(ps)) {
      ps.combinables.delete(policyID);
      this.markChanged(policySetID);
    }
  }

  updateRule(policySetID, policyID, rule) {
    const ps = this.policySets.get(policySetID);
    if (!isNil(ps)) {
      const p = ps.combinables.get(policyID);
      if (!isNil(p)) {
        p.combinables.set(rule.id, rule);
        this.markChanged(policySetID);
      }
    }
  }

  removeRule(policySetID, policyID, ruleID) {
    const ps = this.policySets.get(policySetID);
    if (!isNil(ps)) {
      const p = ps.combinables.get(policyID);
      if (!isNil(p)) {
        p.combinables.delete(ruleID);
        this.markChanged(policySetID);
      }
    }
  }

  clearPolicies() {
    this.policySets.clear();
    this.markChanged(null);
  }

  // setId: a policy set whose contents changed in place (null: only the Map's key set changed)
  markChanged(setId) {
    if (setId !== null && setId !== undefined) this.dirty.add(setId);
    this.stale = true;
  }

  _sync() {
    if (this.stale) this.refresh(this.policySets, Array.from(this.dirty));
  }

  // The per-subject HR-scope cache (createHRScope / evictHRScopes, accessController.ts:717-783):
  // a request whose context.subject has "$hrs": key uses this forest.
  setSubjectScopes(key, hierarchicalScopes) {
    const text = typeof hierarchicalScopes === 'string' ? hierarchicalScopes : JSON.stringify(hierarchicalScopes);
    addon.codecSetSubjectScopes(this.codec, key, text);
    this.scopes.set(key, text);
  }

  evictSubject(key) {
    this.scopes.delete(key);
    return addon.codecEvictSubject(this.codec, key);
  }

  // Releases the GPU tables and the codec (handles are freed explicitly, napi/acs_napi.c).
  close() {
    if (this.builder) addon.storeBuilderFree(this.builder);
    this.builder = null;
    if (this.pipeline) addon.pipelineFree(this.pipeline);
    if (this.tables) addon.free(this.tables);
    if (this.codec) addon.codecFree(this.codec);
    this.pipeline = null;
    this.tables = null;
    this.codec = null;
  }

  // The devices the tables live on (primary first).
  devices() {
    return addon.devices(this.tables);
  }

  _host(op, request, err) {
    this.stats.host += 1;
    if (!this.hostEvaluator) return Promise.resolve(err);
    return Promise.resolve().then(() => this.hostEvaluator(op, request)).catch((e) => e);
  }

  // record i of `rec` -> Response, or the error the reference would reject with
  _response(rec, i, hostReason, ec) {
    const flags = rec[i * REC_BYTES + 2];
    if (flags & OF_HOST_REQ) return new HostPathRequired(hostReason || 'request flagged for the host path');
    const aux = rec[i * REC_BYTES + 4] | (rec[i * REC_BYTES + 5] << 8) | (rec[i * REC_BYTES + 6] << 16) |
      (rec[i * REC_BYTES + 7] << 24);
    if (flags & OF_HOST_COND) return new HostPathRequired('rule condition (JS eval)', aux >>> 0);
    if (flags & OF_ERR) {
      const err = rec[i * REC_BYTES + 3];
      if (err === ERR_REGEX_HOST) return new HostPathRequired('entity RegExp outside the precomputed subset');
      return new GpuEvaluationError(ERR_KINDS[err] || 'Error');
    }
    if (flags & OF_NO_TARGET) {
      return { decision: 'DENY', evaluation_cacheable: false, obligations: [],
               operation_status: { code: 400, message: 'Access request had no target. Skipping request' } };
    }
    return { decision: DECISIONS[rec[i * REC_BYTES]], obligations: [],
             evaluation_cacheable: ec(rec[i * REC_BYTES + 1]),
             operation_status: { code: 200, message: 'success' } };
  }

  // requests: an array of Request objects, or their JSON text.  Resolves to one entry per
  // request: a Response, or an Error (per request, as the reference's promises would reject).
  async isAllowedBatch(requests) {
    const text = typeof requests === 'string' || requests instanceof Uint8Array ? requests : JSON.stringify(requests);
    let parsed = null;
    return this._isAllowedText(text, (i) => {
      if (parsed === null) parsed = parseRequests(requests);
      return parsed[i];
    });
  }

  // The JSON array `text` of requests; request(i): request i as an object (host-path requests).
  async _isAllowedText(text, request) {
    this._sync();
    const ec = this.ec; // the codec's table: refresh() may swap this.ec while the batch is in flight
    const bytes = typeof text === 'string' ? text.length : text.byteLength;
    const r = this.pipeline && bytes >= this.pipelineBytes
      ? await addon.pipelineDecideAsync(this.pipeline, text)
      : await addon.decideAsync(this.tables, this.codec, text, this.threads);
    const n = r.records.length / REC_BYTES;
    this.stats.requests += n;
    const out = new Array(n);
    const pending = [];
    for (let i = 0; i < n; ++i) {
      const v = this._response(r.records, i, r.host[i], ec);
      if (v instanceof HostPathRequired) {
        pending.push(this._host('isAllowed', request(i), v).then((x) => { out[i] = x; }));
      } else {
        out[i] = v;
      }
    }
    await Promise.all(pending);
    return out;
  }

  // AccessController.isAllowed (accessController.ts:88-324) for one request, micro-batched with
  // the concurrent calls (batchWindowMs / batchMax): resolves to its Response or rejects with
  // the error the reference's promise would.
  isAllowed(request) {
    return this._enqueue('isAllowed', request, null);
  }

  // AccessControlService.isAllowed (accessControlService.ts:62-81) for a gRPC request whose
  // context members are protobuf Any messages: their JSON text goes to the codec as is
  // (grpcRequestJson), micro-batched like isAllowed().
  isAllowedGrpc(grpcRequest) {
    return this._enqueue('isAllowed', null, () => grpcRequestJson(grpcRequest));
  }

  whatIsAllowedGrpc(grpcRequest) {
    return this._enqueue('whatIsAllowed', null, () => grpcRequestJson(grpcRequest));
  }

  // The call's JSON text is made here, inside the promise executor: a request that cannot be
  // serialised (BigInt, a cycle, a context Any value that is not one JSON value) rejects this
  // call alone, as the reference's promise would, and never reaches a batch.
  _enqueue(op, request, makeText) {
    return new Promise((resolve, reject) => {
      const text = makeText ? makeText() : JSON.stringify(request);
      if (typeof text !== 'string') throw new TypeError('request is not serialisable as JSON');
      const q = this._queues[op];
      q.push({ request, text, resolve, reject });
      if (q.length >= this.batchMax) {
        this._flush(op);
      } else if (!this._armed[op]) {
        this._armed[op] = true;
        const go = () => {
          this._armed[op] = false;
          this._flush(op);
        };
        if (this.batchWindowMs > 0) setTimeout(go, this.batchWindowMs);
        else setImmediate(go);
      }
    });
  }

  // Decide the queued calls of `op` as one batch.
  _flush(op) {
    const items = this._queues[op];
    if (!items.length) return;
    this._queues[op] = [];
    this._decide(op, items);
  }

  // Decide `items` (queued calls of `op`) as one batch and settle each call with its own
  // record.  A batch the codec rejects as a whole is re-run without the requests whose text does
  // not parse (those reject with the SyntaxError of the reference's JSON.parse).  Records are
  // matched to callers by position, so a batch must come back with exactly one record per call:
  // if it does not, nothing is delivered, every call is re-run as a batch of its own, and a call
  // that still does not decode as exactly one request rejects.
  _decide(op, items) {
    const request = (i) => (items[i].request !== null ? items[i].request : JSON.parse(items[i].text));
    let run;
    try {
      const text = '[' + items.map((x) => x.text).join(',') + ']';
      run = op === 'isAllowed' ? this._isAllowedText(text, request) : this.whatIsAllowedBatch(text, request);
    } catch (e) {
      for (const it of items) it.reject(e);
      return;
    }
    run.then((out) => {
      if (!out || out.length !== items.length) {
        if (items.length === 1) {
          items[0].reject(new Error('request text decoded as ' + (out ? out.length : 0) + ' requests'));
          return;
        }
        for (const it of items) this._decide(op, [it]);
        return;
      }
      for (let i = 0; i < items.length; ++i) {
        if (out[i] instanceof Error) items[i].reject(out[i]);
        else items[i].resolve(out[i]);
      }
    }, (err) => {
      const ok = [];
      for (const it of items) {
        try {
          JSON.parse(it.text);
          ok.push(it);
        } catch (e) {
          it.reject(e);
        }
      }
      if (ok.length === items.length) { // not a text problem: the batch failed as a whole
        for (const it of items) it.reject(err);
        return;
      }
      if (ok.length) this._decide(op, ok);
    });
  }

  // maskedProperty push log -> obligations (find by entity value, else append;
  // accessController.ts:599-613, 624-638)
  _obligations(batch, log, k) {
    const out = [];
    const ent = this.urns.entity, masked = this.urns.maskedProperty;
    for (let j = 0; j < k; ++j) {
      const ev = addon.batchString(batch, log[2 * j]);
      const mv = addon.batchString(batch, log[2 * j + 1]);
      const entry = { id: masked, value: mv, attributes: [] };
      let hit = null;
      for (const m of out) if (m.value === ev) { hit = m; break; }
      if (hit === null) out.push({ id: ent, value: ev, attributes: [entry] });
      else hit.attributes.push(entry);
    }
    return out;
  }

  // Full maskedProperty logs of the requests whose 128-entry log overflowed: the
  // obligation-only pass over 8 policy-set ranges with 1024-entry logs, then once more at the
  // exact count for any range still truncated (INTEGRATION.md §4; native.resolve_overflow).
  _resolveOverflow(batch, flagged) {
    const logs = new Map();
    const chunks = OVERFLOW_CHUNKS;
    let idx = Uint32Array.from(flagged), cap = OVERFLOW_CAP;
    while (idx.length) {
      const r = addon.whatIsAllowedObl(this.tables, batch, idx, chunks, cap);
      const m = idx.length, left = [];
      let need = cap;
      for (let j = 0; j < m; ++j) {
        const parts = [];
        let total = 0, truncated = false;
        for (let c = 0; c < chunks; ++c) {
          const n = r.oblN[c * m + j];
          if (n > cap) {
            truncated = true;
            need = Math.max(need, n);
            continue;
          }
          const base = (c * m + j) * cap * 2;
          parts.push(r.obl.subarray(base, base + 2 * n));
          total += n;
        }
        if (truncated) {
          left.push(idx[j]);
          continue;
        }
        const log = new Uint32Array(2 * total);
        let at = 0;
        for (const p of parts) {
          log.set(p, at);
          at += p.length;
        }
        logs.set(idx[j], log);
      }
      idx = Uint32Array.from(left);
      cap = need;
    }
    return logs;
  }

  // inclusion bitset row -> the reference's PolicySetRQ list (accessController.ts:342-420)
  _reverseQuery(bits, row, words, wp, wr) {
    const ix = this.index;
    const has = (sec, i) => (bits[row * words + sec + (i >>> 5)] >>> (i & 31)) & 1;
    const policySets = [];
    for (let s = 0; s < ix.sets.length; ++s) {
      if (!has(0, s)) continue;
      const ps = ix.sets[s];
      const rq = pick(ps, ['id', 'target', 'effect'], { combining_algorithm: ps.combining_algorithm });
      rq.policies = [];
      for (let p = ix.setPols[s][0]; p < ix.setPols[s][1]; ++p) {
        if (!has(wp, p)) continue;
        const po = ix.pols[p];
        const prq = pick(po, ['id', 'target', 'effect', 'evaluation_cacheable'],
                         { combining_algorithm: po.combining_algorithm });
        prq.rules = [];
        prq.has_rules = !!po.combinables && mapValues(po.combinables).length > 0;
        for (let r = ix.polRules[p][0]; r < ix.polRules[p][1]; ++r) {
          if (!has(wr, r)) continue;
          const ro = ix.rules[r];
          prq.rules.push(pick(ro, ['id', 'target', 'effect', 'condition', 'evaluation_cacheable'],
                              { context_query: clone(ro.context_query) }));
        }
        rq.policies.push(prq);
      }
      policySets.push(rq);
    }
    return policySets;
  }

  // Batch whatIsAllowed (encode + kernels on the calling thread; host-path requests then go
  // to the host evaluator).  Resolves to one entry per request: a ReverseQuery or an Error.
  // request(i) (optional): request i as an object, for the host path (default: parsed from
  // `requests`).
  async whatIsAllowedBatch(requests, request) {
    this._sync();
    const text = typeof requests === 'string' || requests instanceof Uint8Array ? requests : JSON.stringify(requests);
    let parsed = null;
    const req = request || ((i) => {
      if (parsed === null) parsed = parseRequests(requests);
      return parsed[i];
    });
    const batch = addon.encode(this.codec, text, this.threads);
    try {
      return await this._whatIsAllowedEncoded(batch, req);
    } finally {
      addon.batchFree(batch);
    }
  }

  async _whatIsAllowedEncoded(batch, request) {
    const info = addon.batchInfo(batch);
    const w = addon.whatIsAllowed(this.tables, batch);
    const words = addon.wordsPerRequest(this.tables);
    const ns = this.index.sets.length, np = this.index.pols.length;
    const up4 = (x) => (x + 3) & ~3;
    const wp = up4((ns + 31) >>> 5), wr = wp + up4((np + 31) >>> 5);
    const flagged = [];
    for (let i = 0; i < info.n; ++i) {
      const f = w.out[i * REC_BYTES + 2];
      if ((f & OF_OBL_OVERFLOW) && !(f & (OF_HOST_REQ | OF_ERR))) flagged.push(i);
    }
    const long = flagged.length ? this._resolveOverflow(batch, flagged) : new Map();
    const out = new Array(info.n);
    const pending = [];
    for (let i = 0; i < info.n; ++i) {
      const flags = w.out[i * REC_BYTES + 2] & (long.has(i) ? ~OF_OBL_OVERFLOW : 0xff);
      let err = null;
      if (flags & OF_HOST_REQ) err = new HostPathRequired(info.host[i] || 'request flagged for the host path');
      else if (flags & OF_ERR) {
        const e = w.out[i * REC_BYTES + 3];
        err = e === ERR_REGEX_HOST ? new HostPathRequired('entity RegExp outside the precomputed subset')
          : new GpuEvaluationError(ERR_KINDS[e] || 'Error');
      } else if (flags & OF_OBL_OVERFLOW) err = new HostPathRequired('maskedProperty log overflow');
      if (err instanceof HostPathRequired) {
        const at = i;
        pending.push(this._host('whatIsAllowed', request(i), err).then((x) => { out[at] = x; }));
        continue;
      }
      if (err) {
        out[i] = err;
        continue;
      }
      const log = long.has(i) ? long.get(i)
        : w.obl.subarray(i * 2 * OBL_MAX, i * 2 * OBL_MAX + 2 * Math.min(w.oblN[i], OBL_MAX));
      out[i] = {
        policy_sets: this._reverseQuery(w.bits, i, words, wp, wr),
        obligations: this._obligations(batch, log, log.length / 2),
        operation_status: { code: 200, message: 'success' },
      };
    }
    this.stats.requests += info.n;
    await Promise.all(pending);
    return out;
  }

  // AccessController.whatIsAllowed (accessController.ts:326-427) for one request,
  // micro-batched like isAllowed().
  whatIsAllowed(request) {
    return this._enqueue('whatIsAllowed', request, null);
  }
}

module.exports = { GpuAccessController, HostPathRequired, GpuEvaluationError, snapshotStore, nodeIndex,
                   grpcRequestJson, addon };
