/* acs_mi355x.h — C ABI of the MI355X access-control evaluator (libacs_mi355x.so).
 *
 * Drop-in boundary for the decision path of restorecommerce/access-control-srv:
 * the reference's AccessController.isAllowed / whatIsAllowed
 * (src/core/accessController.ts:88-324, 326-427), reached from the gRPC handlers
 * AccessControlService.isAllowed / whatIsAllowed (src/accessControlService.ts:62-101).
 * A host shim (Python: acs_mi355x.controller; Node: INTEGRATION.md) keeps the
 * reference's AccessController surface, compiles its `policySets` Map into a
 * table image, encodes request batches, and calls these entry points.
 *
 * Plain pointers and sizes only.  Return 0 on success, a negative code on
 * failure with a thread-local message from acs_last_error().  Per-request
 * reference errors (a rejected isAllowed promise) are NOT ABI errors: they are
 * reported in the request's acs_decision (flags & ACS_OF_ERR, err kind).
 */
#ifndef ACS_MI355X_H
#define ACS_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ACS_BLOB_MAGIC 0x31534341u /* "ACS1" */
#define ACS_ABI_VERSION 5u

/* Compiled policy-store image (host compiler output, see csrc/acs_layout.h).
 * Header followed by 16-byte aligned sections in this order: set / policy / rule
 * node records (64 B each, target inline), rule resource attrs, (id,value) pairs,
 * u32 pool. */
typedef struct {
  uint32_t magic, version;
  uint32_t n_sets, n_pols, n_rules, n_rres, n_pairs, n_u32pool;
  uint32_t id_user;
  uint32_t reserved[7];
} acs_blob_header;

typedef struct acs_tables acs_tables; /* device-resident tables, immutable once built */

/* One request batch in the packed layout of csrc/acs_layout.h: SoA rows (+ optional request
 * lines), or compact (request lines + extension records, the native codec's form: about
 * 220 B per request instead of 620).  The same struct describes host buffers
 * (acs_is_allowed) or device buffers (acs_is_allowed_device). */
typedef struct {
  uint32_t n;
  const void* hdr;     /* [n] ReqHdr                         */
  const void* res;     /* [QMAX][n] ReqRes                   */
  const void* subj;    /* [SMAX][n] (id,value) u32 pairs     */
  const void* act;     /* [AMAX][n] (id,value) u32 pairs     */
  const uint32_t* roles;  /* [RMAX][n]                        */
  const uint32_t* arena;  /* context arena words               */
  size_t arena_words;
  const uint8_t* rx;      /* [rx_cols][rx_rows] regex matrix   */
  uint32_t rx_cols, rx_rows;
  /* [cand_rows][cand_words] candidate bitsets, one row per request class (entity column x
   * required roles x action, acs_mi355x/candidates.py); the class id is in ReqHdr.flags >> 16.
   * Sections (word offsets): candidate sets at 0, candidate policies at cand_wp, candidate
   * rules at cand_wr, and — isAllowed only, 0 when absent — the sets / policies that can
   * change an isAllowed result at cand_wsu / cand_wpu, and the class's target verdicts at
   * cand_wv: policies whose exact / RegExp target match is known true / false (4 sections
   * of ceil(P/32) words), then rules whose retried match is known true (ceil(R/32) words).
   * NULL = evaluate every node. */
  const uint32_t* cand;
  uint32_t cand_words, cand_wp, cand_wr;
  uint32_t cand_rows;
  uint32_t cand_wsu, cand_wpu, cand_wv;
  /* Optional role factor (large stores, where class rows keyed by roles would not fit):
   * [role_rows][cand_words] bitsets of the nodes a request holding a required role (or a
   * whole role set past two) can reach (checkSubjectMatches, accessController.ts:793-823),
   * with role-relaxed useful sections so that rows OR; AND-ed with the class row.
   * role_key[n] = row | (1 + second row) << 16 (high half 0: one row; a row index >=
   * role_rows: unfiltered); the kernel ORs the two rows.  role_rows < 0xFFFF.  NULL = none. */
  const uint32_t* role_key;
  const uint32_t* role_rows_bits;
  uint32_t role_rows;
  /* [n] 128-B ReqLine (csrc/acs_layout.h): each request's header, first 4 resource
   * attributes, 2 subjects, action, 2 roles and arena counts in one line, so the evaluation
   * kernel reads a request with one gather instead of ~8.  With the SoA rows above: optional,
   * equal to them (checked by the host entry points).  Compact batch (hdr, res, subj, act,
   * roles all NULL): required, and the rows past the line live in `ext`. */
  const void* lines;
  /* Compact batches: the requests' extension records (ReqLine.ext; acs_layout.h ext_geom),
   * u32 words.  May be NULL when no request needs one. */
  const uint32_t* ext;
  size_t ext_words;
  /* Optional coherence order, written by the encoder that assigned the classes (it knows every
   * request's class, so the device does not sort): perm_lanes entries (>= n), each a request
   * index or 0xFFFFFFFF for a hole that pads a class's run to a 64-lane wave boundary; every
   * request appears exactly once.  Lane k of the evaluation kernels takes request perm[k];
   * records are still written in request order.  NULL = the device entry points sort the batch
   * themselves (ACS_OPT_SORT).  A request line's `cls2` (1 + a second class, csrc/acs_layout.h)
   * composes its filter from two class rows. */
  const uint32_t* perm;
  size_t perm_lanes;
  /* Hints (optional, 0: none): ACS_HINT_ACL_NONE — some request carries the ACL_NONE verifyACL
   * state (csrc/acs_layout.h), so K1 is launched with the code that skips the rules its ACLs
   * veto.  Without the hint such requests are still decided exactly (verifyACL returns false
   * for them), only without the skip; both encoders set it. */
  uint32_t hints;
} acs_req_batch;

/* 8-byte decision record (csrc/acs_layout.h: Decision). */
typedef struct {
  uint8_t decision; /* 2 PERMIT 3 DENY 4 NOT_APPLICABLE 5 INDETERMINATE 6 UNRECOGNIZED */
  uint8_t ec;       /* evaluation_cacheable code */
  uint8_t flags;    /* ACS_OF_* */
  uint8_t err;      /* error kind when flags & ACS_OF_ERR */
  uint32_t aux;     /* 1 + index of the last applicable policy set (0: none) / rule index */
} acs_decision;

#define ACS_OF_ERR 0x01u
#define ACS_OF_HOST_COND 0x02u
#define ACS_OF_HOST_REQ 0x04u
#define ACS_OF_NO_TARGET 0x08u
#define ACS_OF_HAS_EFFECT 0x10u
#define ACS_OF_OBL_OVERFLOW 0x20u

#define ACS_HINT_ACL_NONE 0x1u /* acs_req_batch.hints */

/* Replaces: the in-memory `AccessController.policySets` Map the reference scans
 * per request (accessController.ts:32,125; loaded by accessControlService.ts:36-54).
 * Uploads a compiled image to `device`.  NULL on error. */
acs_tables* acs_compile(const void* blob, size_t n_bytes, int device);
void acs_free(acs_tables* t);

/* Multi-GPU (requests are independent, accessController.ts:125-297 keeps no
 * cross-request state): one image replicated to every device in `devices` (C0: uploaded to
 * devices[0], copied to the others over xGMI).  The host-buffer entry points (acs_is_allowed,
 * acs_what_is_allowed, acs_pipeline_*) then split a compact batch of >= 8192 requests into
 * contiguous shards, one per device, each on its own stream with only its shard's request
 * lines / extension records / arena words uploaded, and gather the records (whatIsAllowed: the
 * bitset rows and logs too) in request order; the *_device entry points and
 * acs_what_is_allowed_obl use devices[0].  acs_last_kernel_ms is not set by a split call.
 * acs_device_list: the handle's devices (returns their count). */
acs_tables* acs_compile_multi(const void* blob, size_t n_bytes, const int* devices, int n_devices);
int acs_device_list(const acs_tables* t, int* devices, int n);

/* Rule-sharded handle (SURVEY §8(e) configs[4] variant ii, in one process): the store's policy
 * sets cut into n_devices contiguous runs balanced by node count (acs_mi355x/shard.partition),
 * run k compiled alone onto devices[k].  acs_is_allowed then evaluates every request on every
 * device — the batch uploaded to each, its class rows cut to the device's nodes on the device —
 * turns each device's records into acs_shard_keys_device keys, MAX-reduces them on devices[0]
 * (peer copies over xGMI) and decodes them: the records of an unsharded evaluation.
 * acs_what_is_allowed / acs_what_is_allowed_obl (host buffers) evaluate every request on every
 * device and join the devices' set / policy / rule sections into the caller's rows, obligation
 * logs merged in set order.  The decision pipeline (acs_pipeline_*) runs each chunk that way on a
 * worker thread while the host encodes the next; acs_compile_update serves the handle (below);
 * the device-buffer entry points refuse it. */
acs_tables* acs_compile_sharded(const void* blob, size_t n_bytes, const int* devices, int n_devices);

/* Replaces: the device side of a store change (AccessController.updateRule / updatePolicy / ...,
 * accessController.ts:897-937, after the host recompiles the changed sets).  A new handle for the
 * changed store's blob on prev's device: when the image keeps prev's shape (same node and pool
 * counts), the device image is a device-side copy of prev's with only the 64-KB blocks that differ
 * uploaded (acs_image_upload_bytes: the bytes a compile uploaded); otherwise a full upload.  prev
 * stays valid (batches in flight keep it) and is freed by the caller.  A replicated handle
 * (acs_compile_multi): each replica is its previous image copied on its device with the primary's
 * changed blocks copied over the interconnect.  A rule-sharded handle (acs_compile_sharded): the new
 * store cut again, each shard compiled against the previous shard on its device (a delta when the
 * shard's slice keeps its shape); acs_image_upload_bytes sums the shards. */
acs_tables* acs_compile_update(const acs_tables* prev, const void* blob, size_t n_bytes);
size_t acs_image_upload_bytes(const acs_tables* t);

/* Replaces: AccessController.isAllowed (accessController.ts:88-324), for a batch.
 * Host buffers in and out; synchronous (H2D, kernel, D2H on an internal stream).  Safe to
 * call from several host threads on one handle (calls are serialised per handle). */
int acs_is_allowed(acs_tables* t, const acs_req_batch* host_batch, acs_decision* out);

/* Same, on device-resident buffers, enqueued on `stream` (a hipStream_t; NULL = default).
 * The handle's sort workspace is shared: issue the *_device calls of one handle on one
 * stream (or serialise them). */
int acs_is_allowed_device(acs_tables* t, const acs_req_batch* dev_batch, acs_decision* dev_out, void* stream);

/* Replaces: AccessController.whatIsAllowed (accessController.ts:326-427).
 * bits: [n][words_per_req] inclusion bitsets, one row per request: the set section at word
 * 0, the policy section at word wp = up4(ceil(S/32)), the rule section at word
 * wr = wp + up4(ceil(P/32)); words_per_req = wr + up4(ceil(R/32)) (up4: round up to a
 * multiple of 4, so every section starts on a 16-byte boundary); bit i of a section is
 * bit (i & 31) of its word i >> 5.  The device form needs a 16-byte aligned `bits`.
 * obl: [n][ACS_OBL_MAX][2] maskedProperty push log (entity id, mask id), obl_n: [n]; log entries
 * past a request's count are unspecified. */
#define ACS_OBL_MAX 128
uint32_t acs_wia_words_per_request(const acs_tables* t);
int acs_what_is_allowed(acs_tables* t, const acs_req_batch* host_batch, uint32_t* bits, uint32_t* obl,
                        uint32_t* obl_n, acs_decision* out);
int acs_what_is_allowed_device(acs_tables* t, const acs_req_batch* dev_batch, uint32_t* dev_bits,
                               uint32_t* dev_obl, uint32_t* dev_obl_n, acs_decision* dev_out, void* stream);

/* Obligation-only pass (no reference counterpart: the reference's obligations list is
 * unbounded, accessController.ts:592-640).  Re-evaluates the m requests idx[0..m) of the
 * batch — those whose acs_what_is_allowed record carries OF_OBL_OVERFLOW — with a
 * cap-entry maskedProperty log per lane (1 <= cap <= 2^20) and no bitset.  The policy sets
 * are cut into `chunks` (1..64) contiguous ranges evaluated by separate lanes:
 * obl: [chunks][m][cap][2], obl_n: [chunks][m] = that range's total push count (> cap:
 * still truncated, re-run with cap = obl_n); request j's log is the concatenation of its
 * ranges' logs in range order.  0xFFFFFFFF (device form) = idx[j] outside the batch, which
 * the host form rejects with an error. */
int acs_what_is_allowed_obl(acs_tables* t, const acs_req_batch* host_batch, const uint32_t* idx, size_t m,
                            uint32_t chunks, uint32_t cap, uint32_t* obl, uint32_t* obl_n);
int acs_what_is_allowed_obl_device(acs_tables* t, const acs_req_batch* dev_batch, const uint32_t* dev_idx, size_t m,
                                   uint32_t chunks, uint32_t cap, uint32_t* dev_obl, uint32_t* dev_obl_n,
                                   void* stream);

/* The device path's bookkeeping around the obligation-only pass, on the GPU (stable
 * selection: per-tile counts, one-block scan, ballot-ranked writes; no atomics).
 * acs_overflow_index_device: dev_idx[0..*m) <- the requests of dev_batch whose record in
 * dev_out (an acs_what_is_allowed_device output) carries ACS_OF_OBL_OVERFLOW, in K2's
 * coherence order (class / role key, then request index); dev_idx holds dev_batch->n entries.
 * acs_overflow_repass_device: after a pass over dev_idx[0..m) with `chunks` ranges of cap
 * `cap` (dev_obl_n [chunks][m]), dev_idx_out[0..*m_out) <- the requests some range still
 * truncated (order kept) and *cap_out <- their largest range count, the next pass's cap.
 * Both synchronise `stream` (the count sizes the next pass) and share one scratch per handle:
 * one stream at a time. */
int acs_overflow_index_device(acs_tables* t, const acs_req_batch* dev_batch, const acs_decision* dev_out,
                              uint32_t* dev_idx, size_t* m, void* stream);
int acs_overflow_repass_device(acs_tables* t, const uint32_t* dev_obl_n, const uint32_t* dev_idx, size_t m,
                               uint32_t chunks, uint32_t cap, uint32_t* dev_idx_out, size_t* m_out,
                               uint32_t* cap_out, void* stream);

/* Rule-sharded isAllowed (configs[4] variant ii).  A rank compiles only the
 * policy sets [set_base, set_base + n_sets) of the store (whole sets, Map order) and
 * evaluates every request against them with acs_is_allowed_device.  acs_shard_keys_device
 * turns its decision records into 64-bit keys whose integer MAX over ranks (an RCCL
 * all-reduce, ncclMax on int64) reproduces the reference's two cross-set rules: the last
 * set with a policy effect decides (accessController.ts:293-295) and the first set whose
 * evaluation throws or reaches a rule condition ends the request (:125-295).
 * acs_shard_decode_device turns the reduced keys back into the records an unsharded
 * evaluation writes (aux = global set / rule index).  csrc/acs_eval.h: shard_key. */
typedef struct {
  uint32_t set_base, pol_base, rule_base; /* global index of the rank's first set / policy / rule */
} acs_shard;
int acs_shard_keys_device(acs_tables* t, const acs_decision* dev_dec, size_t n, const acs_shard* shard,
                          uint64_t* dev_keys, void* stream);
int acs_shard_decode_device(const uint64_t* dev_keys, size_t n, acs_decision* dev_out, void* stream);

/* Options.  ACS_OPT_SORT (default 1): evaluate in coherence order — the batch's own `perm`
 * (the encoder's class order) when it carries one, else the device entry points order the
 * batch by request class (entity, roles, action; + role key with a role factor) with a
 * counting / LSD radix sort — so that every wave shares its table-driven branches; results
 * are written in input order.  0: input order. */
#define ACS_OPT_SORT 1
/* ACS_OPT_TIMING: record HIP events on the launch stream around every eval kernel (K1 of
 * acs_is_allowed_device, K2 of acs_what_is_allowed_device); acs_kernel_times returns the durations (ms) of the last n
 * launches (a ring of 256), returning how many were written. */
#define ACS_OPT_TIMING 2
/* ACS_OPT_CHUNK (default 262144): acs_is_allowed on one device cuts a compact batch of at least
 * eight times this many requests into 8 to 16 contiguous chunks and overlaps chunk k + 1's upload
 * with chunk k's evaluation and chunk k - 1's download (two streams); 0: one upload, one
 * launch, one download.  The records are the same either way. */
#define ACS_OPT_CHUNK 3
int acs_set_option(acs_tables* t, int option, int value);
int acs_kernel_times(acs_tables* t, float* ms, int n);

/* Average kernel time (ms) of the last `*_device` launch measured with HIP events on
 * its stream; -1 if none. */
float acs_last_kernel_ms(const acs_tables* t);

/* ------------------------------------------------------------------ native request codec
 * Replaces: the per-request JS work the reference does before and around its matchers —
 * unmarshallContext's JSON (accessControlService.ts:103-125), the request-only parts of
 * resourceAttributesMatch / checkHierarchicalScope / verifyACLList (attribute kinds, lodash
 * _.find context lookups, the verifyACL request loop, the HR-scope flattening of
 * hierarchicalScope.ts:199-245) — for a whole batch, on host threads, producing the packed
 * acs_req_batch the kernels read.  csrc/acs_codec.cpp restates acs_mi355x/encoder.py.
 *
 * acs_codec_create: from the same image acs_compile takes (its codec section, written by
 *   acs_mi355x/compiler.store_blob: dictionary, URN ids, regex rows, candidate specs).
 * acs_codec_encode: `json` = a JSON array of requests ({target, context}, the shape
 *   AccessController.isAllowed receives); `threads` host threads.  NULL on a malformed
 *   array (acs_last_error); a request the packed form cannot carry is encoded with
 *   ACS_RQ_HOST and acs_codec_batch_reason(b, i) says why.  A subject's
 *   `hierarchical_scopes` tree is cached per distinct JSON text; a subject may instead name
 *   a forest registered with acs_codec_set_subject_scopes by a "$hrs": "<key>" member (the
 *   per-subject cache createHRScope fills from Redis, accessController.ts:735-783;
 *   acs_codec_evict_subject = evictHRScopes, :717-725).
 * acs_codec_batch_view: the batch's host buffers as an acs_req_batch (valid until
 *   acs_codec_batch_free), for acs_is_allowed / acs_what_is_allowed or a device upload: the
 *   compact form (request lines + extension records + arena + regex matrix + class rows, in
 *   page-locked memory when a device is present), plus the SoA rows once
 *   acs_codec_batch_expand materialised them.  A batch refers to its codec's dictionary and
 *   buffer pool: free batches before their codec.
 * Candidate-class rows are cached per codec across batches (a steady request stream computes
 *   each class row once).
 * acs_codec_string: interned id -> string (0 undefined, 1 null, 2 string; -1 unknown), e.g.
 *   for maskedProperty obligation ids. */
/* Replaces: the Map -> table snapshot step (acs_mi355x/compiler.py, in C++: csrc/acs_compiler.cpp)
 * for a host without Python.  store_json: the policySets Map as JSON — an array of the Map's
 * values in order, each set's / policy's `combinables` the array of its Map's values
 * (null entries kept); urns_json: policies.options.urns (cfg/config.json:270-307);
 * cas_json: policies.options.combiningAlgorithms.  *blob_out (free with acs_blob_free) is
 * the image for acs_compile / acs_codec_create, byte-identical to compiler.store_blob. */
int acs_store_compile(const char* store_json, size_t store_len, const char* urns_json, size_t urns_len,
                      const char* cas_json, size_t cas_len, void** blob_out, size_t* blob_len);
void acs_blob_free(void* blob);

/* Incremental store compile for a host that mutates its policySets Map
 * in place (accessController.ts:897-937 updatePolicySet .. removeRule, resourceManager.ts:274,
 * 305): the builder keeps each policy set's compiled fragment keyed by the set's JSON text (the
 * snapshot element acs_store_compile reads: JSON.stringify of the set with its combinables as
 * arrays), so a compile recompiles only the sets whose text changed and re-concatenates the
 * rest with shifted offsets.  Interned strings only accumulate (ids stay valid); the first
 * compile of a builder is byte-identical to acs_store_compile of the same store.
 * sets[k] / lens[k]: set k's JSON text in Map order — or sets[k] = NULL and lens[k] = j: set k
 * is set j of the previous compile, unchanged (no text passed, nothing hashed) — or sets[k] =
 * NULL and lens[k] = ACS_BUILDER_STAGED | h: the set staged as handle h; *recompiled: sets
 * compiled afresh.
 * acs_store_builder_stage: one set's JSON text taken ahead of the next compile (compiled now,
 * or matched to an unchanged fragment of the previous compile by its text), so a host can
 * serialise a large store one set at a time instead of holding every set's text at once.
 * Returns the handle (>= 0) or -1 (the set does not compile; the error names it).  A compile
 * consumes every staged set, used or not. */
typedef struct acs_store_builder acs_store_builder;
#define ACS_BUILDER_STAGED ((size_t)1 << (8 * sizeof(size_t) - 1))
acs_store_builder* acs_store_builder_create(const char* urns_json, size_t urns_len, const char* cas_json,
                                            size_t cas_len);
long long acs_store_builder_stage(acs_store_builder* b, const char* set_json, size_t len);
int acs_store_builder_compile(acs_store_builder* b, const char* const* sets, const size_t* lens, size_t n,
                              void** blob_out, size_t* blob_len, size_t* recompiled);
void acs_store_builder_free(acs_store_builder* b);

typedef struct acs_codec acs_codec;
typedef struct acs_codec_batch acs_codec_batch;
#define ACS_RQ_HOST 0x2u
acs_codec* acs_codec_create(const void* blob, size_t n_bytes);
void acs_codec_free(acs_codec* c);
int acs_codec_set_subject_scopes(acs_codec* c, const char* key, size_t key_len, const char* json, size_t len);
int acs_codec_evict_subject(acs_codec* c, const char* key, size_t key_len);
acs_codec_batch* acs_codec_encode(acs_codec* c, const char* json, size_t len, int threads);
int acs_codec_batch_view(const acs_codec_batch* b, acs_req_batch* out);
/* Materialise the SoA rows (hdr / res / subj / act / roles) of an encoded batch, for consumers
 * of that layout (the CPU build of the evaluator core, tests); acs_codec_batch_view then
 * returns them beside the compact arrays. */
int acs_codec_batch_expand(acs_codec_batch* b);
const char* acs_codec_batch_reason(const acs_codec_batch* b, uint32_t i);
int acs_codec_string(const acs_codec_batch* b, uint32_t id, const char** s, size_t* len);
/* The evaluation_cacheable values of the store beyond codes 0..3 (undefined, null, false,
 * true), as a JSON array: code k >= 4 is element k - 4 (acs_decision.ec). */
int acs_codec_ec_values(const acs_codec* c, const char** json, size_t* len);
/* out[0..7]: seconds parse+encode, regex matrix + assembly, candidate classes, total; HR cache
 * hits, misses; class rows computed by this batch (not served by the codec's cache), classes */
int acs_codec_batch_stats(const acs_codec_batch* b, double* out, int n);
void acs_codec_batch_free(acs_codec_batch* b);

/* ------------------------------------------------------------------ decision pipeline
 * Replaces: the reference's per-request evaluation behind AccessControlService.isAllowed
 * (accessControlService.ts:62-81 -> accessController.ts:88-324) for a micro-batch of requests
 * arriving as JSON text, end to end: the request array is delimited once and cut into chunks
 * of `chunk` requests; chunk k+1 is encoded (acs_codec) on `threads` host threads while chunk
 * k is uploaded from the codec's page-locked blocks, sorted and decided (K1) and its records
 * downloaded, on one of the pipeline's two streams per device (each with its own device
 * workspace; a multi-device handle's chunks go round the devices).
 * out[0..n) receives the records in request order (out_cap >= n, else an error with *n_out set,
 * before any encoding).  Requests flagged for the host path carry ACS_OF_HOST_REQ;
 * acs_pipeline_host_reason gives the codec's reason for request i of the last run (NULL for a
 * request that is not one), valid until the next run.  One run at a time per pipeline; the
 * tables and codec must outlive it. */
typedef struct acs_pipeline acs_pipeline;
typedef struct {
  double encode_s;      /* host time encoding (all chunks) */
  double wait_s;        /* host time blocked on the device */
  double total_s;       /* wall time of the call */
  double gpu_ms;        /* device time (upload + sort + K1 + download), summed over chunks */
  double upload_bytes;  /* bytes copied to the device */
  uint64_t requests, chunks, host_requests;
  double split_s;       /* host time delimiting the request array */
  double check_s;       /* host time validating the encoded chunks (acs_is_allowed's batch checks) */
} acs_pipeline_stats;
acs_pipeline* acs_pipeline_create(acs_tables* t, acs_codec* c, int threads, uint32_t chunk);
void acs_pipeline_free(acs_pipeline* p);
int acs_pipeline_is_allowed(acs_pipeline* p, const char* json, size_t len, acs_decision* out, size_t out_cap,
                            size_t* n_out, acs_pipeline_stats* st);
const char* acs_pipeline_host_reason(acs_pipeline* p, size_t i);

const char* acs_last_error(void);
int acs_layout_sizes(uint32_t* out, int n); /* sizeof of the 5 packed structs, for host checks */
int acs_device_count(void);

#ifdef __cplusplus
}
#endif
#endif /* ACS_MI355X_H */
