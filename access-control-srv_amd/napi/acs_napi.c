/* acs_napi.c — N-API addon over the C ABI of libacs_mi355x.so (include/acs_mi355x.h).
 *
 * The binding a TypeScript host (src/core/accessController.ts) loads to compile its
 * policySets Map, encode JSON requests and evaluate them on the MI355X; gpuCodec.js (next
 * to this file) is the JS layer over it and INTEGRATION.md the TS side.  Plain C over
 * node_api.h (N-API 8, Node >= 12.22): no V8 headers, no node-gyp —
 * access-control-srv_amd/acs_mi355x/build.py compiles it with gcc.
 *
 * JS surface:
 *   compileStore(storeJson, urnsJson, casJson) -> Uint8Array   acs_store_compile
 *   storeBuilderCreate(urnsJson, casJson) -> builder            acs_store_builder_create
 *   storeBuilderStage(builder, setJson) -> -(1 + h)             acs_store_builder_stage
 *   storeBuilderCompile(builder, sets[]) -> {blob, recompiled}  acs_store_builder_compile
 *     (sets[k]: set k's JSON text, j >= 0 = the previous compile's set j, unchanged, or a
 *     storeBuilderStage result)
 *   storeBuilderFree(builder)                                   acs_store_builder_free
 *   compile(blob: Uint8Array, device?) -> tables                acs_compile
 *     (device = [d0, d1, ...]: one image per device, acs_compile_multi)
 *   devices(tables) -> number[]                                 acs_device_list
 *   free(tables)                                                acs_free (deferred past in-flight work)
 *   codecCreate(blob) -> codec                                  acs_codec_create
 *   codecFree(codec), batchFree(batch)                          acs_codec_free / acs_codec_batch_free
 *   codecSetSubjectScopes(codec, key, scopesJson)               acs_codec_set_subject_scopes
 *   codecEvictSubject(codec, key) -> bool                       acs_codec_evict_subject
 *   codecEcValues(codec) -> string (JSON array)                 acs_codec_ec_values
 *   encode(codec, json, threads?) -> batch                      acs_codec_encode
 *   batchInfo(batch) -> {n, host: {index: reason}}
 *   batchString(batch, id) -> string | null | undefined         acs_codec_string
 *   decideAsync(tables, codec, json, threads?) -> Promise<{records, host}>
 *                                    encode + acs_is_allowed on the libuv pool, one step
 *   pipelineCreate(tables, codec, threads?, chunk?) -> pipeline acs_pipeline_create
 *   pipelineFree(pipeline)                                      acs_pipeline_free (after in-flight work)
 *   pipelineDecideAsync(pipeline, json) -> Promise<{records, host, stats}>
 *                                    acs_pipeline_is_allowed on the libuv pool: encode of
 *                                    chunk k+1 overlapped with the device work of chunk k
 *   isAllowed(tables, batch) -> Uint8Array(8 n)                 acs_is_allowed (sync)
 *   isAllowedAsync(tables, batch) -> Promise<Uint8Array>        same, on the libuv pool
 *   whatIsAllowed(tables, batch) -> {bits, obl, oblN, out}      acs_what_is_allowed
 *   whatIsAllowedObl(tables, batch, idx, chunks, cap) -> {obl, oblN}
 *   wordsPerRequest(tables), layoutSizes(), deviceCount(), lastError()
 * `batch` = an encode() handle, or a plain object {n, hdr, res, subj, act, roles, arena,
 * rx, rxCols, rxRows, cand, candWords, candWp, candWr, candRows[, candWsu, candWpu, candWv, roleKey, roleRowsBits,
 * roleRows, lines]} of typed arrays in the layout of csrc/acs_layout.h — or, compact, {n, lines,
 * ext, arena, rx, ...} without the SoA rows; every array is checked against the sizes `n` and
 * the counts imply before the library reads it.
 *
 * Handles are plain objects naming a per-environment registry slot (see "handles" below:
 * no napi externals, whose weak references Node 12 can touch after freeing them at exit).
 * They are released explicitly (free / codecFree / batchFree) or at environment teardown.
 * free() on tables with async work in flight defers the release until that work completes;
 * any call on a freed handle throws.  A batch keeps its codec alive (a counted reference), the
 * codec's dictionary being part of the batch's meaning.
 */
#define NAPI_VERSION 8
#include <node_api.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/acs_mi355x.h"

#define CHECK(env, call)                                              \
  do {                                                                \
    if ((call) != napi_ok) {                                          \
      napi_throw_error((env), NULL, "N-API call failed: " #call);     \
      return NULL;                                                    \
    }                                                                 \
  } while (0)

/* csrc/acs_layout.h sizes (checked against acs_layout_sizes by tests/test_napi.py) */
enum { HDR_B = 16, RES_B = 16, PAIR_B = 8, LINE_B = 128, QMAX = 16, SMAX = 8, AMAX = 4, RMAX = 8 };

static napi_value throw_acs(napi_env env, const char* what) {
  char msg[512];
  const char* e = acs_last_error();
  snprintf(msg, sizeof msg, "%s", e && *e ? e : what);
  napi_throw_error(env, NULL, msg);
  return NULL;
}

/* ------------------------------------------------------------------ handles
 * A handle is a plain JS object ({acsTables: id}, {acsCodec: id} or {acsBatch: id}) naming a
 * slot of this environment's registry, not a napi external.  Node 12's environment teardown
 * (napi_env__'s destructor, RefTracker::FinalizeAll) deletes every napi reference while V8 may
 * still hold a queued second-pass phantom callback for an external collected just before
 * exit; Environment::CleanupHandles then runs that callback on the deleted reference
 * (SIGSEGV in v8::internal::GlobalHandles::PendingPhantomCallback::Invoke, reproduced with a
 * backtrace: 22 of 128 runs of tests/js/gpu_codec_run.js under load).  A handle that holds no
 * weak reference cannot be hit.  Lifetimes are therefore explicit — free(tables),
 * codecFree(codec), batchFree(batch) — and whatever is still registered when the environment
 * is torn down is released by its cleanup hook (objects with work in flight are left to the
 * process exit).  Each environment (main thread, worker_threads) has its own registry. */
enum { H_TABLES = 1, H_CODEC = 2, H_BATCH = 3, H_PIPELINE = 4, H_BUILDER = 5 };
static const char* const KIND_KEY[6] = {"", "acsTables", "acsCodec", "acsBatch", "acsPipeline", "acsStoreBuilder"};

typedef struct env_state env_state;

typedef struct {
  int kind;
  env_state* st;
  uint32_t slot; /* registry slot while the JS handle is live, UINT32_MAX after free */
  int refs;      /* the JS handle + in-flight work (+ live batches, for a codec) */
} obj_base;

typedef struct {
  obj_base base;
  acs_tables* t;
  int inflight; /* async work items using t */
} tables_h;

typedef struct {
  obj_base base;
  acs_codec* c;
} codec_h;

typedef struct {
  obj_base base;
  acs_codec_batch* b;
  codec_h* codec; /* counted reference: the codec outlives its batches */
} batch_h;

typedef struct {
  obj_base base;
  acs_pipeline* p;
  tables_h* tables; /* counted references: both outlive the pipeline */
  codec_h* codec;
  int inflight;      /* queued / running pipelineDecideAsync work */
  pthread_mutex_t mu; /* a run and the reading of its host reasons, together */
} pipeline_h;

typedef struct {
  obj_base base;
  acs_store_builder* b;
} builder_h;

typedef struct {
  int kind; /* 0: never used */
  uint32_t gen;
  obj_base* obj; /* NULL: freed (slot reusable) */
} slot_t;

struct env_state {
  slot_t* slots;
  uint32_t n, cap;
  int dead; /* the environment is being torn down */
};

static void obj_unref(obj_base* o);

static void obj_release(obj_base* o) {
  if (o->kind == H_TABLES) {
    tables_h* h = (tables_h*)o;
    if (h->t) acs_free(h->t);
    h->t = NULL;
  } else if (o->kind == H_CODEC) {
    codec_h* h = (codec_h*)o;
    if (h->c) acs_codec_free(h->c);
    h->c = NULL;
  } else if (o->kind == H_PIPELINE) {
    pipeline_h* h = (pipeline_h*)o;
    if (h->p) acs_pipeline_free(h->p); /* before its tables and codec */
    h->p = NULL;
    pthread_mutex_destroy(&h->mu);
    if (h->tables) obj_unref(&h->tables->base);
    if (h->codec) obj_unref(&h->codec->base);
    h->tables = NULL;
    h->codec = NULL;
  } else if (o->kind == H_BUILDER) {
    builder_h* h = (builder_h*)o;
    if (h->b) acs_store_builder_free(h->b);
    h->b = NULL;
  } else if (o->kind == H_BATCH) {
    batch_h* h = (batch_h*)o;
    if (h->b) acs_codec_batch_free(h->b); /* before its codec */
    h->b = NULL;
    if (h->codec) obj_unref(&h->codec->base);
    h->codec = NULL;
  }
  o->kind = 0;
  free(o);
}

static void obj_unref(obj_base* o) {
  if (--o->refs == 0) obj_release(o);
}

static void on_env_exit(void* arg) {
  env_state* st = (env_state*)arg;
  st->dead = 1;
  /* pipelines and batches first (they hold their codec / tables), then codecs and tables */
  static const int order[5] = {H_PIPELINE, H_BATCH, H_CODEC, H_TABLES, H_BUILDER};
  for (int k = 0; k < 5; ++k)
    for (uint32_t i = 0; i < st->n; ++i) {
      slot_t* s = &st->slots[i];
      if (!s->obj || s->obj->kind != order[k]) continue;
      obj_base* o = s->obj;
      s->obj = NULL;
      o->slot = UINT32_MAX;
      if (o->kind == H_TABLES && ((tables_h*)o)->inflight) continue; /* the pool still uses it */
      if (o->kind == H_PIPELINE && ((pipeline_h*)o)->inflight) continue;
      obj_unref(o);
    }
}

static env_state* get_state(napi_env env) {
  void* d = NULL;
  if (napi_get_instance_data(env, &d) == napi_ok && d) return (env_state*)d;
  env_state* st = (env_state*)calloc(1, sizeof *st);
  if (!st) return NULL;
  /* no finalizer: the struct is tiny and may be read by work completing during teardown */
  if (napi_set_instance_data(env, st, NULL, NULL) != napi_ok) {
    free(st);
    return NULL;
  }
  napi_add_env_cleanup_hook(env, on_env_exit, st);
  return st;
}

/* Register `o` (refs = 1, the JS handle) and return its handle object. */
static napi_value make_handle(napi_env env, obj_base* o, int kind) {
  env_state* st = get_state(env);
  napi_value h, id;
  o->kind = kind;
  o->st = st;
  o->refs = 1;
  o->slot = UINT32_MAX;
  if (!st) goto fail;
  uint32_t i = 0;
  while (i < st->n && st->slots[i].obj) ++i;
  if (i == st->n) {
    if (st->n == st->cap) {
      const uint32_t cap = st->cap ? 2 * st->cap : 64;
      slot_t* s = (slot_t*)realloc(st->slots, cap * sizeof *s);
      if (!s) goto fail;
      memset(s + st->cap, 0, (cap - st->cap) * sizeof *s);
      st->slots = s;
      st->cap = cap;
    }
    ++st->n;
  }
  slot_t* s = &st->slots[i];
  s->kind = kind;
  s->gen = (s->gen + 1) & 0x0FFFFFFFu;
  s->obj = o;
  o->slot = i;
  const double v = (double)s->gen * 16777216.0 + (double)i; /* < 2^53 */
  napi_property_descriptor d = {KIND_KEY[kind], NULL, NULL, NULL, NULL, NULL, napi_enumerable, NULL};
  if (napi_create_double(env, v, &id) != napi_ok || napi_create_object(env, &h) != napi_ok) goto fail;
  d.value = id;
  if (napi_define_properties(env, h, 1, &d) != napi_ok) goto fail;
  return h;
fail:
  if (o->slot != UINT32_MAX) st->slots[o->slot].obj = NULL;
  o->slot = UINT32_MAX;
  obj_unref(o);
  napi_throw_error(env, NULL, "could not register a handle");
  return NULL;
}

/* The live object a handle names, or NULL: *freed = 1 when it names a handle of this kind
 * that was already freed. */
static obj_base* lookup(napi_env env, napi_value v, int kind, int* freed) {
  napi_valuetype t;
  napi_value idv;
  bool has = false;
  double d = -1;
  *freed = 0;
  env_state* st = get_state(env);
  if (!st || napi_typeof(env, v, &t) != napi_ok || t != napi_object) return NULL;
  if (napi_has_named_property(env, v, KIND_KEY[kind], &has) != napi_ok || !has) return NULL;
  if (napi_get_named_property(env, v, KIND_KEY[kind], &idv) != napi_ok ||
      napi_get_value_double(env, idv, &d) != napi_ok || !(d >= 0) || d >= 9007199254740992.0)
    return NULL;
  const uint64_t id = (uint64_t)d;
  const uint32_t i = (uint32_t)(id & 0xFFFFFFu), gen = (uint32_t)(id >> 24);
  if (i >= st->n || st->slots[i].kind != kind || st->slots[i].gen != gen) return NULL;
  if (!st->slots[i].obj) {
    *freed = 1;
    return NULL;
  }
  return st->slots[i].obj;
}

/* JS free of a handle: the slot is released now, the object when its last ref goes. */
static void handle_free(obj_base* o) {
  if (o->slot != UINT32_MAX && o->st) o->st->slots[o->slot].obj = NULL;
  o->slot = UINT32_MAX;
  obj_unref(o);
}

static tables_h* get_tables(napi_env env, napi_value v) {
  int freed;
  tables_h* h = (tables_h*)lookup(env, v, H_TABLES, &freed);
  if (!h) {
    if (freed) napi_throw_error(env, NULL, "tables handle already freed");
    else napi_throw_type_error(env, NULL, "expected a tables handle (compile())");
    return NULL;
  }
  return h;
}

static codec_h* get_codec(napi_env env, napi_value v) {
  int freed;
  codec_h* h = (codec_h*)lookup(env, v, H_CODEC, &freed);
  if (!h) {
    if (freed) napi_throw_error(env, NULL, "codec handle already freed");
    else napi_throw_type_error(env, NULL, "expected a codec handle (codecCreate())");
    return NULL;
  }
  return h;
}

static batch_h* find_batch(napi_env env, napi_value v) {
  int freed;
  return (batch_h*)lookup(env, v, H_BATCH, &freed);
}

/* ------------------------------------------------------------------ buffers */
/* Bytes of a typed array / Buffer / ArrayBuffer (NULL for null / undefined). */
static int get_bytes(napi_env env, napi_value v, void** data, size_t* len) {
  napi_valuetype t;
  bool is;
  *data = NULL;
  *len = 0;
  if (napi_typeof(env, v, &t) != napi_ok) return -1;
  if (t == napi_null || t == napi_undefined) return 0;
  if (napi_is_typedarray(env, v, &is) == napi_ok && is) {
    napi_typedarray_type tt;
    size_t n, off;
    napi_value ab;
    if (napi_get_typedarray_info(env, v, &tt, &n, data, &ab, &off) != napi_ok) return -1;
    size_t es = 1;
    switch (tt) {
      case napi_int16_array: case napi_uint16_array: es = 2; break;
      case napi_int32_array: case napi_uint32_array: case napi_float32_array: es = 4; break;
      case napi_float64_array: case napi_bigint64_array: case napi_biguint64_array: es = 8; break;
      default: es = 1;
    }
    *len = n * es;
    return 0;
  }
  if (napi_is_arraybuffer(env, v, &is) == napi_ok && is)
    return napi_get_arraybuffer_info(env, v, data, len) == napi_ok ? 0 : -1;
  return -1;
}

/* A JS string (UTF-8, malloc'd copy in *out) or bytes (borrowed).  *owned: free it. */
static int get_text(napi_env env, napi_value v, char** out, size_t* len, int* owned) {
  napi_valuetype t;
  *out = NULL;
  *len = 0;
  *owned = 0;
  if (napi_typeof(env, v, &t) != napi_ok) return -1;
  if (t == napi_string) {
    size_t n = 0;
    if (napi_get_value_string_utf8(env, v, NULL, 0, &n) != napi_ok) return -1;
    char* s = (char*)malloc(n + 1);
    if (!s) return -1;
    if (napi_get_value_string_utf8(env, v, s, n + 1, &n) != napi_ok) {
      free(s);
      return -1;
    }
    *out = s;
    *len = n;
    *owned = 1;
    return 0;
  }
  void* p;
  if (get_bytes(env, v, &p, len) || !p) return -1;
  *out = (char*)p;
  return 0;
}

static int prop_bytes(napi_env env, napi_value obj, const char* key, void** data, size_t* len) {
  napi_value v;
  if (napi_get_named_property(env, obj, key, &v) != napi_ok) return -1;
  return get_bytes(env, v, data, len);
}

static int prop_u32(napi_env env, napi_value obj, const char* key, uint32_t* out) {
  napi_value v;
  napi_valuetype t;
  *out = 0;
  if (napi_get_named_property(env, obj, key, &v) != napi_ok) return -1;
  if (napi_typeof(env, v, &t) != napi_ok) return -1;
  if (t == napi_undefined || t == napi_null) return 0;
  return napi_get_value_uint32(env, v, out) == napi_ok ? 0 : -1;
}

/* one typed-array field of a plain batch object, required to hold at least `need` bytes */
static int field(napi_env env, napi_value obj, const char* key, size_t need, int required, const void** out,
                 size_t* len_out, const char** bad) {
  void* p;
  size_t len;
  if (prop_bytes(env, obj, key, &p, &len)) {
    *bad = key;
    return -1;
  }
  if ((required && need && !p) || (p && len < need)) {  /* an absent optional field is fine */
    *bad = key;
    return -1;
  }
  *out = p;
  if (len_out) *len_out = len;
  return 0;
}

/* JS batch (encode() handle or plain object) -> acs_req_batch with every buffer checked
 * against the sizes its counts imply (pointers into JS buffers; the caller keeps them alive). */
static int read_batch(napi_env env, napi_value v, acs_req_batch* b) {
  memset(b, 0, sizeof *b);
  batch_h* bh = find_batch(env, v);
  if (bh) return acs_codec_batch_view(bh->b, b) == 0 ? 0 : -1;
  napi_valuetype t;
  if (napi_typeof(env, v, &t) != napi_ok || t != napi_object) return -1;
  const char* bad = NULL;
  size_t len = 0;
  if (prop_u32(env, v, "n", &b->n)) return -1;
  const size_t n = b->n;
  const void* p;
  if (prop_u32(env, v, "rxCols", &b->rx_cols) || prop_u32(env, v, "rxRows", &b->rx_rows) ||
      prop_u32(env, v, "candWords", &b->cand_words) || prop_u32(env, v, "candWp", &b->cand_wp) ||
      prop_u32(env, v, "candWr", &b->cand_wr) || prop_u32(env, v, "candRows", &b->cand_rows) ||
      prop_u32(env, v, "roleRows", &b->role_rows) || prop_u32(env, v, "candWsu", &b->cand_wsu) ||
      prop_u32(env, v, "candWpu", &b->cand_wpu) || prop_u32(env, v, "candWv", &b->cand_wv) ||
      prop_u32(env, v, "hints", &b->hints))
    return -1;
  /* compact batch (csrc/acs_layout.h): lines + ext, no SoA rows */
  if (field(env, v, "lines", n * LINE_B, 0, &b->lines, NULL, &bad)) goto fail;
  {
    napi_value hv;
    napi_valuetype ht;
    const int compact = napi_get_named_property(env, v, "hdr", &hv) == napi_ok && napi_typeof(env, hv, &ht) == napi_ok &&
                        (ht == napi_undefined || ht == napi_null) && b->lines;
    if (compact) {
      if (field(env, v, "ext", 0, 0, &p, &len, &bad)) goto fail;
      b->ext = (const uint32_t*)p;
      b->ext_words = len / 4;
    } else {
      if (field(env, v, "hdr", n * HDR_B, n > 0, &b->hdr, NULL, &bad) ||
          field(env, v, "res", n * QMAX * RES_B, n > 0, &b->res, NULL, &bad) ||
          field(env, v, "subj", n * SMAX * PAIR_B, n > 0, &b->subj, NULL, &bad) ||
          field(env, v, "act", n * AMAX * PAIR_B, n > 0, &b->act, NULL, &bad) ||
          field(env, v, "roles", n * RMAX * 4, n > 0, &p, NULL, &bad))
        goto fail;
      b->roles = (const uint32_t*)p;
    }
  }
  if (field(env, v, "arena", 0, 0, &p, &len, &bad)) goto fail;
  b->arena = (const uint32_t*)p;
  b->arena_words = len / 4;
  if (n > 0 && (!p || len < 8)) {
    bad = "arena";
    goto fail;
  }
  if (field(env, v, "rx", (size_t)b->rx_cols * b->rx_rows, n > 0, &p, NULL, &bad)) goto fail;
  b->rx = (const uint8_t*)p;
  if (field(env, v, "cand", (size_t)b->cand_rows * b->cand_words * 4, 0, &p, &len, &bad)) goto fail;
  b->cand = (const uint32_t*)p;
  if (b->cand && (b->cand_wp > b->cand_words || b->cand_wr > b->cand_words || b->cand_wsu > b->cand_words ||
                  b->cand_wpu > b->cand_words || b->cand_wv > b->cand_words)) {
    bad = "candWp / candWr / candWsu / candWpu / candWv";
    goto fail;
  }
  if (field(env, v, "roleKey", 0, 0, &p, &len, &bad)) goto fail;
  b->role_key = (const uint32_t*)p;
  if (b->role_key) {
    if (len < n * 4) {
      bad = "roleKey";
      goto fail;
    }
    if (field(env, v, "roleRowsBits", (size_t)b->role_rows * b->cand_words * 4, 1, &p, NULL, &bad)) goto fail;
    b->role_rows_bits = (const uint32_t*)p;
  } else {
    b->role_rows = 0;
  }
  /* per-request offsets the kernels follow (the library checks everything again) */
  {
    const uint8_t* hdr = b->hdr ? (const uint8_t*)b->hdr : (const uint8_t*)b->lines;
    const size_t stride = b->hdr ? HDR_B : LINE_B;
    for (size_t i = 0; i < n; ++i) {
      uint32_t arena_off;
      memcpy(&arena_off, hdr + i * stride + 8, 4);
      if ((size_t)arena_off + 2 > b->arena_words) {
        bad = "hdr.arena_off";
        goto fail;
      }
      if (hdr[i * stride + 4] > QMAX || hdr[i * stride + 5] > SMAX || hdr[i * stride + 6] > AMAX ||
          hdr[i * stride + 7] > RMAX) {
        bad = "hdr counts";
        goto fail;
      }
    }
  }
  return 0;
fail : {
  char msg[160];
  snprintf(msg, sizeof msg, "batch.%s is missing or shorter than its counts require", bad ? bad : "?");
  napi_throw_range_error(env, NULL, msg);
  return -2;
}
}

static napi_value new_u8(napi_env env, size_t n, void** data) {
  napi_value ab, arr;
  if (napi_create_arraybuffer(env, n, data, &ab) != napi_ok) return NULL;
  if (napi_create_typedarray(env, napi_uint8_array, n, ab, 0, &arr) != napi_ok) return NULL;
  return arr;
}

static napi_value new_u32(napi_env env, size_t n, void** data) {
  napi_value ab, arr;
  if (napi_create_arraybuffer(env, n * 4, data, &ab) != napi_ok) return NULL;
  if (napi_create_typedarray(env, napi_uint32_array, n, ab, 0, &arr) != napi_ok) return NULL;
  return arr;
}

static int batch_arg(napi_env env, napi_value v, acs_req_batch* b, const char* usage) {
  const int rc = read_batch(env, v, b);
  if (rc == -1) napi_throw_type_error(env, NULL, usage);
  return rc;
}

/* ------------------------------------------------------------------ store compile */
static napi_value js_compile_store(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3], out;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  char* s[3] = {NULL, NULL, NULL};
  size_t n[3] = {0, 0, 0};
  int own[3] = {0, 0, 0};
  int ok = argc == 3;
  for (int k = 0; k < 3 && ok; ++k) ok = get_text(env, argv[k], &s[k], &n[k], &own[k]) == 0;
  napi_value ret = NULL;
  if (!ok) {
    napi_throw_type_error(env, NULL, "compileStore(storeJson, urnsJson, casJson)");
  } else {
    void* blob = NULL;
    size_t len = 0;
    if (acs_store_compile(s[0], n[0], s[1], n[1], s[2], n[2], &blob, &len) != 0) {
      throw_acs(env, "acs_store_compile");
    } else {
      void* d;
      out = new_u8(env, len, &d);
      if (out) {
        memcpy(d, blob, len);
        ret = out;
      }
      acs_blob_free(blob);
    }
  }
  for (int k = 0; k < 3; ++k)
    if (own[k]) free(s[k]);
  return ret;
}

/* storeBuilderCreate(urnsJson, casJson) -> builder: acs_store_builder_create (incremental
 * compile, one fragment per policy set). */
static napi_value js_builder_create(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  char* s[2] = {NULL, NULL};
  size_t n[2] = {0, 0};
  int own[2] = {0, 0};
  int ok = argc == 2;
  for (int k = 0; k < 2 && ok; ++k) ok = get_text(env, argv[k], &s[k], &n[k], &own[k]) == 0;
  napi_value ret = NULL;
  if (!ok) {
    napi_throw_type_error(env, NULL, "storeBuilderCreate(urnsJson, casJson)");
  } else {
    acs_store_builder* b = acs_store_builder_create(s[0], n[0], s[1], n[1]);
    if (!b) {
      throw_acs(env, "acs_store_builder_create");
    } else {
      builder_h* h = (builder_h*)calloc(1, sizeof *h);
      if (!h) {
        acs_store_builder_free(b);
        napi_throw_error(env, NULL, "out of memory");
      } else {
        h->b = b;
        ret = make_handle(env, &h->base, H_BUILDER);
      }
    }
  }
  for (int k = 0; k < 2; ++k)
    if (own[k]) free(s[k]);
  return ret;
}

/* storeBuilderCompile(builder, sets) -> {blob: Uint8Array, recompiled}: sets[k] is policy set
 * k's JSON text (Map order), or a number j: the previous compile's set j, unchanged. */
static napi_value js_builder_compile(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int freed = 0;
  builder_h* h = argc == 2 ? (builder_h*)lookup(env, argv[0], H_BUILDER, &freed) : NULL;
  bool is_arr = false;
  if (!h || napi_is_array(env, argv[1], &is_arr) != napi_ok || !is_arr) {
    napi_throw_type_error(env, NULL, freed ? "store builder already freed" : "storeBuilderCompile(builder, sets[])");
    return NULL;
  }
  uint32_t n = 0;
  CHECK(env, napi_get_array_length(env, argv[1], &n));
  const char** texts = (const char**)calloc(n ? n : 1, sizeof *texts);
  size_t* lens = (size_t*)calloc(n ? n : 1, sizeof *lens);
  int* own = (int*)calloc(n ? n : 1, sizeof *own);
  napi_value ret = NULL;
  int ok = texts && lens && own;
  for (uint32_t k = 0; k < n && ok; ++k) {
    napi_value e;
    napi_valuetype t;
    ok = napi_get_element(env, argv[1], k, &e) == napi_ok && napi_typeof(env, e, &t) == napi_ok;
    if (!ok) break;
    if (t == napi_number) {  /* j >= 0: previous set j; j < 0: staged handle -(j + 1) */
      int64_t j = 0;
      ok = napi_get_value_int64(env, e, &j) == napi_ok;
      texts[k] = NULL;
      lens[k] = j >= 0 ? (size_t)j : (ACS_BUILDER_STAGED | (size_t)(-(j + 1)));
    } else {
      char* p = NULL;
      ok = get_text(env, e, &p, &lens[k], &own[k]) == 0;
      texts[k] = p;
    }
  }
  if (!ok) {
    napi_throw_type_error(env, NULL, "storeBuilderCompile: sets[] holds JSON texts or previous indices");
  } else {
    void* blob = NULL;
    size_t len = 0, rec = 0;
    if (acs_store_builder_compile(h->b, texts, lens, n, &blob, &len, &rec) != 0) {
      throw_acs(env, "acs_store_builder_compile");
    } else {
      void* d;
      napi_value arr = new_u8(env, len, &d), obj, rv;
      if (arr && napi_create_object(env, &obj) == napi_ok && napi_create_double(env, (double)rec, &rv) == napi_ok &&
          napi_set_named_property(env, obj, "blob", arr) == napi_ok &&
          napi_set_named_property(env, obj, "recompiled", rv) == napi_ok) {
        memcpy(d, blob, len);
        ret = obj;
      }
      acs_blob_free(blob);
    }
  }
  for (uint32_t k = 0; k < n && own; ++k)
    if (own[k]) free((void*)texts[k]);
  free(texts);
  free(lens);
  free(own);
  return ret;
}

/* storeBuilderStage(builder, setJson) -> -(1 + handle): one set's text staged for the next
 * storeBuilderCompile (acs_store_builder_stage); pass the returned number in its sets[]. */
static napi_value js_builder_stage(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int freed = 0;
  builder_h* h = argc == 2 ? (builder_h*)lookup(env, argv[0], H_BUILDER, &freed) : NULL;
  if (!h) {
    napi_throw_type_error(env, NULL, freed ? "store builder already freed" : "storeBuilderStage(builder, setJson)");
    return NULL;
  }
  char* p = NULL;
  size_t len = 0;
  int own = 0;
  if (get_text(env, argv[1], &p, &len, &own) != 0) {
    napi_throw_type_error(env, NULL, "storeBuilderStage: setJson must be a string or bytes");
    return NULL;
  }
  const long long id = acs_store_builder_stage(h->b, p, len);
  if (own) free(p);
  if (id < 0) {
    throw_acs(env, "acs_store_builder_stage");
    return NULL;
  }
  napi_value ret;
  CHECK(env, napi_create_double(env, -(double)(id + 1), &ret));
  return ret;
}

/* storeBuilderFree(builder). */
static napi_value js_builder_free(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  int freed = 0;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  builder_h* h = argc > 0 ? (builder_h*)lookup(env, argv[0], H_BUILDER, &freed) : NULL;
  if (!h) {
    if (!freed) napi_throw_type_error(env, NULL, "storeBuilderFree(builder)");
    return NULL;
  }
  handle_free(&h->base);
  return NULL;
}

/* ------------------------------------------------------------------ tables */
static napi_value js_compile(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2], out;
  void* blob;
  size_t len;
  int32_t device = 0, devs[64];
  uint32_t n_devs = 0;
  bool is_array = false;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 1 || get_bytes(env, argv[0], &blob, &len) || !blob) {
    napi_throw_type_error(env, NULL, "compile(blob: Uint8Array, device?: number | number[])");
    return NULL;
  }
  if (argc > 1) {
    CHECK(env, napi_is_array(env, argv[1], &is_array));
    if (is_array) {
      CHECK(env, napi_get_array_length(env, argv[1], &n_devs));
      if (n_devs < 1 || n_devs > 64) {
        napi_throw_range_error(env, NULL, "compile: 1..64 devices");
        return NULL;
      }
      for (uint32_t k = 0; k < n_devs; ++k) {
        napi_value e;
        CHECK(env, napi_get_element(env, argv[1], k, &e));
        if (napi_get_value_int32(env, e, &devs[k]) != napi_ok) {
          napi_throw_type_error(env, NULL, "compile: device ids must be numbers");
          return NULL;
        }
      }
    } else {
      CHECK(env, napi_get_value_int32(env, argv[1], &device));
    }
  }
  acs_tables* t = is_array ? acs_compile_multi(blob, len, devs, (int)n_devs) : acs_compile(blob, len, device);
  if (!t) return throw_acs(env, "acs_compile");
  tables_h* h = (tables_h*)calloc(1, sizeof *h);
  if (!h) {
    acs_free(t);
    napi_throw_error(env, NULL, "out of memory");
    return NULL;
  }
  h->t = t;
  out = make_handle(env, &h->base, H_TABLES);
  return out;
}

/* compileUpdate(prev, blob): acs_compile_update — the changed store's image from prev's with
 * only the differing blocks uploaded (same shape), else a full upload; prev stays valid */
static napi_value js_compile_update(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  void* blob;
  size_t len;
  int freed = 0;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  tables_h* prev = argc > 0 ? (tables_h*)lookup(env, argv[0], H_TABLES, &freed) : NULL;
  if (!prev || argc < 2 || get_bytes(env, argv[1], &blob, &len) || !blob) {
    if (!freed) napi_throw_type_error(env, NULL, "compileUpdate(tables, blob: Uint8Array)");
    return NULL;
  }
  acs_tables* t = acs_compile_update(prev->t, blob, len);
  if (!t) return throw_acs(env, "acs_compile_update");
  tables_h* h = (tables_h*)calloc(1, sizeof *h);
  if (!h) {
    acs_free(t);
    napi_throw_error(env, NULL, "out of memory");
    return NULL;
  }
  h->t = t;
  return make_handle(env, &h->base, H_TABLES);
}

/* uploadBytes(tables): the bytes its compile uploaded (acs_image_upload_bytes) */
static napi_value js_upload_bytes(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], out;
  int freed = 0;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  tables_h* h = argc > 0 ? (tables_h*)lookup(env, argv[0], H_TABLES, &freed) : NULL;
  if (!h) {
    if (!freed) napi_throw_type_error(env, NULL, "uploadBytes(tables)");
    return NULL;
  }
  CHECK(env, napi_create_double(env, (double)acs_image_upload_bytes(h->t), &out));
  return out;
}

static napi_value js_devices(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], out;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int freed = 0;
  tables_h* h = argc > 0 ? (tables_h*)lookup(env, argv[0], H_TABLES, &freed) : NULL;
  if (!h) {
    if (!freed) napi_throw_type_error(env, NULL, "devices(tables)");
    return NULL;
  }
  int devs[64];
  const int m = acs_device_list(h->t, devs, 64);
  if (m < 0) return throw_acs(env, "acs_device_list");
  CHECK(env, napi_create_array_with_length(env, (size_t)m, &out));
  for (int k = 0; k < m && k < 64; ++k) {
    napi_value e;
    CHECK(env, napi_create_int32(env, devs[k], &e));
    CHECK(env, napi_set_element(env, out, (uint32_t)k, e));
  }
  return out;
}

static napi_value js_free(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int freed = 0;
  tables_h* h = argc > 0 ? (tables_h*)lookup(env, argv[0], H_TABLES, &freed) : NULL;
  if (!h) {
    if (!freed) napi_throw_type_error(env, NULL, "free(tables)");
    return NULL; /* freeing twice is a no-op */
  }
  handle_free(&h->base); /* work in flight holds its own reference: the last one releases */
  return NULL;
}

static napi_value js_is_allowed(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  acs_req_batch b;
  void* out;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc != 2) {
    napi_throw_type_error(env, NULL, "isAllowed(tables, batch)");
    return NULL;
  }
  /* the batch first: its checks need no device */
  if (batch_arg(env, argv[1], &b, "isAllowed(tables, batch)")) return NULL;
  tables_h* h = get_tables(env, argv[0]);
  if (!h) return NULL;
  napi_value arr = new_u8(env, (size_t)b.n * sizeof(acs_decision), &out);
  if (!arr) return NULL;
  if (acs_is_allowed(h->t, &b, (acs_decision*)out) != 0) return throw_acs(env, "acs_is_allowed");
  return arr;
}

/* ------------------------------------------------------------------ async work */
typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  napi_ref keep_batch, keep_out; /* strong references (no weak callbacks) */
  tables_h* th;
  codec_h* ch;
  acs_req_batch b;
  acs_decision* out;
  /* decideAsync: encode on the pool too */
  char* text;
  size_t text_len;
  int text_owned;
  int threads;
  acs_codec_batch* enc;
  int rc;
  char err[512];
} async_req;

static void work_done_tables(async_req* r) {
  r->th->inflight--;
  obj_unref(&r->th->base);
}

static void exec_is_allowed(napi_env env, void* data) {
  (void)env;
  async_req* r = (async_req*)data;
  r->rc = acs_is_allowed(r->th->t, &r->b, r->out);
  if (r->rc) snprintf(r->err, sizeof r->err, "acs_is_allowed: %s", acs_last_error());
}

static void done_is_allowed(napi_env env, napi_status status, void* data) {
  async_req* r = (async_req*)data;
  napi_value out;
  napi_get_reference_value(env, r->keep_out, &out);
  work_done_tables(r);
  if (status == napi_ok && r->rc == 0) {
    napi_resolve_deferred(env, r->deferred, out);
  } else {
    napi_value msg, err;
    napi_create_string_utf8(env, r->rc ? r->err : "async work cancelled", NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_reject_deferred(env, r->deferred, err);
  }
  napi_delete_reference(env, r->keep_batch);
  napi_delete_reference(env, r->keep_out);
  napi_delete_async_work(env, r->work);
  free(r);
}

static napi_value js_is_allowed_async(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2], promise, name;
  void* out;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc != 2) {
    napi_throw_type_error(env, NULL, "isAllowedAsync(tables, batch)");
    return NULL;
  }
  tables_h* th = get_tables(env, argv[0]);
  if (!th) return NULL;
  async_req* r = (async_req*)calloc(1, sizeof *r);
  if (!r) {
    napi_throw_error(env, NULL, "out of memory");
    return NULL;
  }
  r->th = th;
  if (batch_arg(env, argv[1], &r->b, "isAllowedAsync(tables, batch)")) {
    free(r);
    return NULL;
  }
  napi_value arr = new_u8(env, (size_t)r->b.n * sizeof(acs_decision), &out);
  if (!arr) {
    free(r);
    return NULL;
  }
  r->out = (acs_decision*)out;
  CHECK(env, napi_create_reference(env, argv[1], 1, &r->keep_batch));
  CHECK(env, napi_create_reference(env, arr, 1, &r->keep_out));
  CHECK(env, napi_create_promise(env, &r->deferred, &promise));
  CHECK(env, napi_create_string_utf8(env, "acs_is_allowed", NAPI_AUTO_LENGTH, &name));
  CHECK(env, napi_create_async_work(env, NULL, name, exec_is_allowed, done_is_allowed, r, &r->work));
  th->inflight++;
  th->base.refs++;
  CHECK(env, napi_queue_async_work(env, r->work));
  return promise;
}

/* decideAsync: JSON text -> acs_codec_encode -> acs_is_allowed, all on the libuv pool */
static void exec_decide(napi_env env, void* data) {
  (void)env;
  async_req* r = (async_req*)data;
  r->enc = acs_codec_encode(r->ch->c, r->text, r->text_len, r->threads);
  if (!r->enc) {
    r->rc = -1;
    snprintf(r->err, sizeof r->err, "%s", acs_last_error());
    return;
  }
  if (acs_codec_batch_view(r->enc, &r->b) != 0) {
    r->rc = -1;
    snprintf(r->err, sizeof r->err, "%s", acs_last_error());
    return;
  }
  r->out = (acs_decision*)malloc((size_t)r->b.n * sizeof(acs_decision) + 1);
  if (!r->out) {
    r->rc = -1;
    snprintf(r->err, sizeof r->err, "out of memory");
    return;
  }
  r->rc = acs_is_allowed(r->th->t, &r->b, r->out);
  if (r->rc) snprintf(r->err, sizeof r->err, "acs_is_allowed: %s", acs_last_error());
}

static napi_value host_map(napi_env env, acs_codec_batch* b, uint32_t n) {
  napi_value host, v;
  if (napi_create_object(env, &host) != napi_ok) return NULL;
  acs_req_batch view;
  if (acs_codec_batch_view(b, &view) != 0) return host;
  /* the header is the first 16 B of each 128-B request line (csrc/acs_layout.h ReqLine) */
  const uint8_t* hdr = view.hdr ? (const uint8_t*)view.hdr : (const uint8_t*)view.lines;
  const size_t stride = view.hdr ? HDR_B : LINE_B;
  for (uint32_t i = 0; i < n; ++i) {
    uint32_t flags;
    memcpy(&flags, hdr + (size_t)i * stride, 4);
    if (!(flags & ACS_RQ_HOST)) continue;
    const char* why = acs_codec_batch_reason(b, i);
    char key[16];
    snprintf(key, sizeof key, "%u", i);
    napi_create_string_utf8(env, why ? why : "host path", NAPI_AUTO_LENGTH, &v);
    napi_set_named_property(env, host, key, v);
  }
  return host;
}

static void done_decide(napi_env env, napi_status status, void* data) {
  async_req* r = (async_req*)data;
  work_done_tables(r);
  if (status == napi_ok && r->rc == 0) {
    napi_value res, rec;
    void* d;
    napi_create_object(env, &res);
    rec = new_u8(env, (size_t)r->b.n * sizeof(acs_decision), &d);
    if (rec) memcpy(d, r->out, (size_t)r->b.n * sizeof(acs_decision));
    napi_set_named_property(env, res, "records", rec);
    napi_set_named_property(env, res, "host", host_map(env, r->enc, r->b.n));
    napi_resolve_deferred(env, r->deferred, res);
  } else {
    napi_value msg, err;
    napi_create_string_utf8(env, r->rc ? r->err : "async work cancelled", NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_reject_deferred(env, r->deferred, err);
  }
  if (r->enc) acs_codec_batch_free(r->enc);
  obj_unref(&r->ch->base);
  free(r->out);
  if (r->text_owned) free(r->text);
  if (r->keep_batch) napi_delete_reference(env, r->keep_batch);
  napi_delete_async_work(env, r->work);
  free(r);
}

static napi_value js_decide_async(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4], promise, name;
  int32_t threads = 4;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 3) {
    napi_throw_type_error(env, NULL, "decideAsync(tables, codec, json, threads?)");
    return NULL;
  }
  tables_h* th = get_tables(env, argv[0]);
  codec_h* ch = th ? get_codec(env, argv[1]) : NULL;
  if (!th || !ch) return NULL;
  if (argc > 3) CHECK(env, napi_get_value_int32(env, argv[3], &threads));
  async_req* r = (async_req*)calloc(1, sizeof *r);
  if (!r) {
    napi_throw_error(env, NULL, "out of memory");
    return NULL;
  }
  r->th = th;
  r->ch = ch;
  r->threads = threads;
  if (get_text(env, argv[2], &r->text, &r->text_len, &r->text_owned)) {
    free(r);
    napi_throw_type_error(env, NULL, "decideAsync: json must be a string or bytes");
    return NULL;
  }
  if (!r->text_owned) CHECK(env, napi_create_reference(env, argv[2], 1, &r->keep_batch));  /* borrowed bytes */
  CHECK(env, napi_create_promise(env, &r->deferred, &promise));
  CHECK(env, napi_create_string_utf8(env, "acs_decide", NAPI_AUTO_LENGTH, &name));
  CHECK(env, napi_create_async_work(env, NULL, name, exec_decide, done_decide, r, &r->work));
  th->inflight++;
  th->base.refs++;
  ch->base.refs++;
  CHECK(env, napi_queue_async_work(env, r->work));
  return promise;
}

/* ------------------------------------------------------------------ pipeline */
static napi_value js_pipeline_create(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  int32_t threads = 4;
  uint32_t chunk = 0;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 2) {
    napi_throw_type_error(env, NULL, "pipelineCreate(tables, codec, threads?, chunk?)");
    return NULL;
  }
  tables_h* th = get_tables(env, argv[0]);
  codec_h* ch = th ? get_codec(env, argv[1]) : NULL;
  if (!th || !ch) return NULL;
  if (argc > 2) CHECK(env, napi_get_value_int32(env, argv[2], &threads));
  if (argc > 3) CHECK(env, napi_get_value_uint32(env, argv[3], &chunk));
  acs_pipeline* p = acs_pipeline_create(th->t, ch->c, threads, chunk);
  if (!p) return throw_acs(env, "acs_pipeline_create");
  pipeline_h* h = (pipeline_h*)calloc(1, sizeof *h);
  if (!h || pthread_mutex_init(&h->mu, NULL) != 0) {
    free(h);
    acs_pipeline_free(p);
    napi_throw_error(env, NULL, "out of memory");
    return NULL;
  }
  h->p = p;
  h->tables = th;
  h->codec = ch;
  th->base.refs++;
  ch->base.refs++;
  return make_handle(env, &h->base, H_PIPELINE);
}

static napi_value js_pipeline_free(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int freed = 0;
  obj_base* h = argc > 0 ? lookup(env, argv[0], H_PIPELINE, &freed) : NULL;
  if (!h) {
    if (!freed) napi_throw_type_error(env, NULL, "pipelineFree(pipeline)");
    return NULL;
  }
  handle_free(h);
  return NULL;
}

typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  napi_ref keep_text;
  pipeline_h* ph;
  char* text;
  size_t text_len;
  int text_owned;
  acs_decision* out;
  size_t n;
  size_t n_host;
  uint32_t* host_idx;
  char** host_why;
  acs_pipeline_stats st;
  int rc;
  char err[512];
} pipe_req;

static void exec_pipeline(napi_env env, void* data) {
  (void)env;
  pipe_req* r = (pipe_req*)data;
  pthread_mutex_lock(&r->ph->mu);
  /* the request count is known only once the array is delimited: a first guess, then (an
   * error before any encoding, with the count) the exact size */
  size_t cap = r->text_len / 32 + 16;
  for (int attempt = 0; attempt < 2; ++attempt) {
    r->out = (acs_decision*)malloc(cap * sizeof(acs_decision) + 1);
    if (!r->out) {
      r->rc = -1;
      snprintf(r->err, sizeof r->err, "out of memory");
      break;
    }
    size_t n = 0;
    r->rc = acs_pipeline_is_allowed(r->ph->p, r->text, r->text_len, r->out, cap, &n, &r->st);
    if (r->rc == 0) {
      r->n = n;
      break;
    }
    snprintf(r->err, sizeof r->err, "acs_pipeline_is_allowed: %s", acs_last_error());
    free(r->out);
    r->out = NULL;
    if (n <= cap) break;
    cap = n;
  }
  if (r->rc == 0) {
    for (size_t i = 0; i < r->n; ++i) r->n_host += (r->out[i].flags & ACS_OF_HOST_REQ) ? 1 : 0;
    if (r->n_host) {
      r->host_idx = (uint32_t*)calloc(r->n_host, sizeof *r->host_idx);
      r->host_why = (char**)calloc(r->n_host, sizeof *r->host_why);
      size_t k = 0;
      for (size_t i = 0; i < r->n && r->host_idx && r->host_why; ++i) {
        if (!(r->out[i].flags & ACS_OF_HOST_REQ)) continue;
        const char* why = acs_pipeline_host_reason(r->ph->p, i);
        r->host_idx[k] = (uint32_t)i;
        const char* w = why ? why : "host path";
        const size_t wl = strlen(w);
        r->host_why[k] = (char*)malloc(wl + 1);
        if (r->host_why[k]) memcpy(r->host_why[k], w, wl + 1);
        ++k;
      }
      if (!r->host_idx || !r->host_why) r->n_host = 0;
    }
  }
  pthread_mutex_unlock(&r->ph->mu);
}

static void done_pipeline(napi_env env, napi_status status, void* data) {
  pipe_req* r = (pipe_req*)data;
  if (status == napi_ok && r->rc == 0) {
    napi_value res, rec, host, stats, v;
    void* d;
    napi_create_object(env, &res);
    rec = new_u8(env, r->n * sizeof(acs_decision), &d);
    if (rec && r->n) memcpy(d, r->out, r->n * sizeof(acs_decision));
    napi_set_named_property(env, res, "records", rec);
    napi_create_object(env, &host);
    for (size_t k = 0; k < r->n_host; ++k) {
      char key[16];
      snprintf(key, sizeof key, "%u", r->host_idx[k]);
      napi_create_string_utf8(env, r->host_why[k] ? r->host_why[k] : "host path", NAPI_AUTO_LENGTH, &v);
      napi_set_named_property(env, host, key, v);
    }
    napi_set_named_property(env, res, "host", host);
    napi_create_object(env, &stats);
    const double sv[8] = {r->st.encode_s, r->st.wait_s, r->st.total_s, r->st.gpu_ms, r->st.upload_bytes,
                          (double)r->st.requests, (double)r->st.chunks, (double)r->st.host_requests};
    static const char* const sk[8] = {"encodeS", "waitS", "totalS", "gpuMs", "uploadBytes", "requests", "chunks",
                                      "hostRequests"};
    for (int k = 0; k < 8; ++k) {
      napi_create_double(env, sv[k], &v);
      napi_set_named_property(env, stats, sk[k], v);
    }
    napi_set_named_property(env, res, "stats", stats);
    napi_resolve_deferred(env, r->deferred, res);
  } else {
    napi_value msg, err;
    napi_create_string_utf8(env, r->rc ? r->err : "async work cancelled", NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, NULL, msg, &err);
    napi_reject_deferred(env, r->deferred, err);
  }
  r->ph->inflight--;
  obj_unref(&r->ph->base);
  for (size_t k = 0; k < r->n_host; ++k) free(r->host_why[k]);
  free(r->host_why);
  free(r->host_idx);
  free(r->out);
  if (r->text_owned) free(r->text);
  if (r->keep_text) napi_delete_reference(env, r->keep_text);
  napi_delete_async_work(env, r->work);
  free(r);
}

static napi_value js_pipeline_decide_async(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2], promise, name;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  int freed = 0;
  pipeline_h* ph = argc == 2 ? (pipeline_h*)lookup(env, argv[0], H_PIPELINE, &freed) : NULL;
  if (!ph) {
    if (freed) napi_throw_error(env, NULL, "pipeline handle already freed");
    else napi_throw_type_error(env, NULL, "pipelineDecideAsync(pipeline, json)");
    return NULL;
  }
  pipe_req* r = (pipe_req*)calloc(1, sizeof *r);
  if (!r) {
    napi_throw_error(env, NULL, "out of memory");
    return NULL;
  }
  r->ph = ph;
  if (get_text(env, argv[1], &r->text, &r->text_len, &r->text_owned)) {
    free(r);
    napi_throw_type_error(env, NULL, "pipelineDecideAsync: json must be a string or bytes");
    return NULL;
  }
  if (!r->text_owned) CHECK(env, napi_create_reference(env, argv[1], 1, &r->keep_text)); /* borrowed bytes */
  CHECK(env, napi_create_promise(env, &r->deferred, &promise));
  CHECK(env, napi_create_string_utf8(env, "acs_pipeline", NAPI_AUTO_LENGTH, &name));
  CHECK(env, napi_create_async_work(env, NULL, name, exec_pipeline, done_pipeline, r, &r->work));
  ph->inflight++;
  ph->base.refs++;
  CHECK(env, napi_queue_async_work(env, r->work));
  return promise;
}

/* ------------------------------------------------------------------ codec */
static napi_value js_codec_create(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], out;
  void* blob;
  size_t len;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 1 || get_bytes(env, argv[0], &blob, &len) || !blob) {
    napi_throw_type_error(env, NULL, "codecCreate(blob: Uint8Array)");
    return NULL;
  }
  acs_codec* c = acs_codec_create(blob, len);
  if (!c) return throw_acs(env, "acs_codec_create");
  codec_h* h = (codec_h*)calloc(1, sizeof *h);
  if (!h) {
    acs_codec_free(c);
    napi_throw_error(env, NULL, "out of memory");
    return NULL;
  }
  h->c = c;
  out = make_handle(env, &h->base, H_CODEC);
  return out;
}

/* codecFree(codec): release the JS handle; the codec itself goes once its batches and any
 * work in flight are done with it.  Freeing twice is a no-op. */
static napi_value js_codec_free(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  int freed = 0;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  codec_h* h = argc > 0 ? (codec_h*)lookup(env, argv[0], H_CODEC, &freed) : NULL;
  if (!h) {
    if (!freed) napi_throw_type_error(env, NULL, "codecFree(codec)");
    return NULL;
  }
  handle_free(&h->base);
  return NULL;
}

/* batchFree(batch): release an encode() batch (and its reference on the codec). */
static napi_value js_batch_free(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  int freed = 0;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  batch_h* h = argc > 0 ? (batch_h*)lookup(env, argv[0], H_BATCH, &freed) : NULL;
  if (!h) {
    if (!freed) napi_throw_type_error(env, NULL, "batchFree(batch)");
    return NULL;
  }
  handle_free(&h->base);
  return NULL;
}

static napi_value js_codec_set_scopes(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  codec_h* h = argc == 3 ? get_codec(env, argv[0]) : NULL;
  if (!h) return NULL;
  char *k, *j;
  size_t kn, jn;
  int ko, jo;
  if (get_text(env, argv[1], &k, &kn, &ko)) {
    napi_throw_type_error(env, NULL, "codecSetSubjectScopes(codec, key: string, scopesJson)");
    return NULL;
  }
  if (get_text(env, argv[2], &j, &jn, &jo)) {
    if (ko) free(k);
    napi_throw_type_error(env, NULL, "codecSetSubjectScopes(codec, key: string, scopesJson)");
    return NULL;
  }
  const int rc = acs_codec_set_subject_scopes(h->c, k, kn, j, jn);
  if (ko) free(k);
  if (jo) free(j);
  if (rc != 0) return throw_acs(env, "acs_codec_set_subject_scopes");
  return NULL;
}

static napi_value js_codec_evict(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2], v;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  codec_h* h = argc == 2 ? get_codec(env, argv[0]) : NULL;
  if (!h) return NULL;
  char* k;
  size_t kn;
  int ko;
  if (get_text(env, argv[1], &k, &kn, &ko)) {
    napi_throw_type_error(env, NULL, "codecEvictSubject(codec, key: string)");
    return NULL;
  }
  const int rc = acs_codec_evict_subject(h->c, k, kn);
  if (ko) free(k);
  CHECK(env, napi_get_boolean(env, rc == 1, &v));
  return v;
}

static napi_value js_codec_ec_values(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], v;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  codec_h* h = argc == 1 ? get_codec(env, argv[0]) : NULL;
  if (!h) return NULL;
  const char* j;
  size_t n;
  if (acs_codec_ec_values(h->c, &j, &n) != 0) return throw_acs(env, "acs_codec_ec_values");
  CHECK(env, napi_create_string_utf8(env, j, n, &v));
  return v;
}

static napi_value js_encode(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3], out;
  int32_t threads = 1;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  codec_h* h = argc >= 2 ? get_codec(env, argv[0]) : NULL;
  if (!h) return NULL;
  if (argc > 2) CHECK(env, napi_get_value_int32(env, argv[2], &threads));
  char* s;
  size_t n;
  int own;
  if (get_text(env, argv[1], &s, &n, &own)) {
    napi_throw_type_error(env, NULL, "encode(codec, json: string | Uint8Array, threads?)");
    return NULL;
  }
  acs_codec_batch* b = acs_codec_encode(h->c, s, n, threads);
  if (own) free(s);
  if (!b) return throw_acs(env, "acs_codec_encode");
  batch_h* bh = (batch_h*)calloc(1, sizeof *bh);
  if (!bh) {
    acs_codec_batch_free(b);
    napi_throw_error(env, NULL, "out of memory");
    return NULL;
  }
  bh->b = b;
  bh->codec = h;
  h->base.refs++;
  out = make_handle(env, &bh->base, H_BATCH);
  return out;
}

static napi_value js_batch_info(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], res, v;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  batch_h* bh = argc == 1 ? find_batch(env, argv[0]) : NULL;
  if (!bh) {
    napi_throw_type_error(env, NULL, "batchInfo(batch)");
    return NULL;
  }
  acs_req_batch view;
  acs_codec_batch_view(bh->b, &view);
  CHECK(env, napi_create_object(env, &res));
  CHECK(env, napi_create_uint32(env, view.n, &v));
  CHECK(env, napi_set_named_property(env, res, "n", v));
  CHECK(env, napi_set_named_property(env, res, "host", host_map(env, bh->b, view.n)));
  return res;
}

static napi_value js_batch_string(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2], v;
  uint32_t id;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  batch_h* bh = argc == 2 ? find_batch(env, argv[0]) : NULL;
  if (!bh || napi_get_value_uint32(env, argv[1], &id) != napi_ok) {
    napi_throw_type_error(env, NULL, "batchString(batch, id)");
    return NULL;
  }
  const char* s;
  size_t n;
  const int k = acs_codec_string(bh->b, id, &s, &n);
  if (k == 0) {
    CHECK(env, napi_get_undefined(env, &v));
  } else if (k == 1) {
    CHECK(env, napi_get_null(env, &v));
  } else if (k == 2) {
    CHECK(env, napi_create_string_utf8(env, s, n, &v));
  } else {
    napi_throw_range_error(env, NULL, "batchString: unknown id");
    return NULL;
  }
  return v;
}

/* ------------------------------------------------------------------ whatIsAllowed */
static napi_value js_what_is_allowed(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2], res;
  acs_req_batch b;
  void *bits, *obl, *obl_n, *out;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc != 2) {
    napi_throw_type_error(env, NULL, "whatIsAllowed(tables, batch)");
    return NULL;
  }
  if (batch_arg(env, argv[1], &b, "whatIsAllowed(tables, batch)")) return NULL;
  tables_h* h = get_tables(env, argv[0]);
  if (!h) return NULL;
  const size_t w = acs_wia_words_per_request(h->t);
  napi_value a_bits = new_u32(env, (size_t)b.n * w, &bits);
  napi_value a_obl = new_u32(env, (size_t)b.n * ACS_OBL_MAX * 2, &obl);
  napi_value a_obl_n = new_u32(env, b.n, &obl_n);
  napi_value a_out = new_u8(env, (size_t)b.n * sizeof(acs_decision), &out);
  if (!a_bits || !a_obl || !a_obl_n || !a_out) return NULL;
  if (acs_what_is_allowed(h->t, &b, (uint32_t*)bits, (uint32_t*)obl, (uint32_t*)obl_n, (acs_decision*)out) != 0)
    return throw_acs(env, "acs_what_is_allowed");
  CHECK(env, napi_create_object(env, &res));
  CHECK(env, napi_set_named_property(env, res, "bits", a_bits));
  CHECK(env, napi_set_named_property(env, res, "obl", a_obl));
  CHECK(env, napi_set_named_property(env, res, "oblN", a_obl_n));
  CHECK(env, napi_set_named_property(env, res, "out", a_out));
  return res;
}

/* whatIsAllowedObl(tables, batch, idx: Uint32Array, chunks, cap) -> {obl, oblN}: the
 * obligation-only pass (acs_what_is_allowed_obl) for requests whose whatIsAllowed record
 * carries ACS_OF_OBL_OVERFLOW; obl [chunks][m][cap][2], oblN [chunks][m]. */
static napi_value js_what_is_allowed_obl(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5], res;
  acs_req_batch b;
  void *idx, *obl, *obl_n;
  size_t idx_len;
  uint32_t chunks = 0, cap = 0;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  const char* usage = "whatIsAllowedObl(tables, batch, idx: Uint32Array, chunks 1..64, cap 1..2^20)";
  if (argc != 5) {
    napi_throw_type_error(env, NULL, usage);
    return NULL;
  }
  tables_h* h = get_tables(env, argv[0]);
  if (!h || batch_arg(env, argv[1], &b, usage)) return NULL;
  if (get_bytes(env, argv[2], &idx, &idx_len) || idx_len % 4 ||
      napi_get_value_uint32(env, argv[3], &chunks) != napi_ok || napi_get_value_uint32(env, argv[4], &cap) != napi_ok ||
      chunks == 0 || chunks > 64 || cap == 0 || cap > (1u << 20)) {
    napi_throw_type_error(env, NULL, usage);
    return NULL;
  }
  const size_t m = idx_len / 4;
  napi_value a_obl = new_u32(env, m * chunks * (size_t)cap * 2, &obl);
  napi_value a_obl_n = new_u32(env, m * chunks, &obl_n);
  if (!a_obl || !a_obl_n) return NULL;
  if (acs_what_is_allowed_obl(h->t, &b, (const uint32_t*)idx, m, chunks, cap, (uint32_t*)obl, (uint32_t*)obl_n) != 0)
    return throw_acs(env, "acs_what_is_allowed_obl");
  CHECK(env, napi_create_object(env, &res));
  CHECK(env, napi_set_named_property(env, res, "obl", a_obl));
  CHECK(env, napi_set_named_property(env, res, "oblN", a_obl_n));
  return res;
}

/* ------------------------------------------------------------------ misc */
static napi_value js_words(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1], v;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  tables_h* h = argc ? get_tables(env, argv[0]) : NULL;
  if (!h) return NULL;
  CHECK(env, napi_create_uint32(env, acs_wia_words_per_request(h->t), &v));
  return v;
}

static napi_value js_layout_sizes(napi_env env, napi_callback_info info) {
  (void)info;
  uint32_t s[5];
  napi_value arr, v;
  int n = acs_layout_sizes(s, 5);
  CHECK(env, napi_create_array_with_length(env, 5, &arr));
  for (int i = 0; i < n && i < 5; ++i) {
    CHECK(env, napi_create_uint32(env, s[i], &v));
    CHECK(env, napi_set_element(env, arr, (uint32_t)i, v));
  }
  return arr;
}

static napi_value js_device_count(napi_env env, napi_callback_info info) {
  (void)info;
  napi_value v;
  CHECK(env, napi_create_int32(env, acs_device_count(), &v));
  return v;
}

static napi_value js_last_error(napi_env env, napi_callback_info info) {
  (void)info;
  napi_value v;
  const char* e = acs_last_error();
  CHECK(env, napi_create_string_utf8(env, e ? e : "", NAPI_AUTO_LENGTH, &v));
  return v;
}

static napi_value init(napi_env env, napi_value exports) {
  if (!get_state(env)) return NULL; /* this environment's handle registry + its cleanup hook */
  const napi_property_descriptor d[] = {
      {"compileStore", NULL, js_compile_store, NULL, NULL, NULL, napi_enumerable, NULL},
      {"storeBuilderCreate", NULL, js_builder_create, NULL, NULL, NULL, napi_enumerable, NULL},
      {"storeBuilderStage", NULL, js_builder_stage, NULL, NULL, NULL, napi_enumerable, NULL},
      {"storeBuilderCompile", NULL, js_builder_compile, NULL, NULL, NULL, napi_enumerable, NULL},
      {"storeBuilderFree", NULL, js_builder_free, NULL, NULL, NULL, napi_enumerable, NULL},
      {"compile", NULL, js_compile, NULL, NULL, NULL, napi_enumerable, NULL},
      {"compileUpdate", NULL, js_compile_update, NULL, NULL, NULL, napi_enumerable, NULL},
      {"uploadBytes", NULL, js_upload_bytes, NULL, NULL, NULL, napi_enumerable, NULL},
      {"free", NULL, js_free, NULL, NULL, NULL, napi_enumerable, NULL},
      {"codecCreate", NULL, js_codec_create, NULL, NULL, NULL, napi_enumerable, NULL},
      {"codecFree", NULL, js_codec_free, NULL, NULL, NULL, napi_enumerable, NULL},
      {"batchFree", NULL, js_batch_free, NULL, NULL, NULL, napi_enumerable, NULL},
      {"codecSetSubjectScopes", NULL, js_codec_set_scopes, NULL, NULL, NULL, napi_enumerable, NULL},
      {"codecEvictSubject", NULL, js_codec_evict, NULL, NULL, NULL, napi_enumerable, NULL},
      {"codecEcValues", NULL, js_codec_ec_values, NULL, NULL, NULL, napi_enumerable, NULL},
      {"encode", NULL, js_encode, NULL, NULL, NULL, napi_enumerable, NULL},
      {"batchInfo", NULL, js_batch_info, NULL, NULL, NULL, napi_enumerable, NULL},
      {"batchString", NULL, js_batch_string, NULL, NULL, NULL, napi_enumerable, NULL},
      {"decideAsync", NULL, js_decide_async, NULL, NULL, NULL, napi_enumerable, NULL},
      {"pipelineCreate", NULL, js_pipeline_create, NULL, NULL, NULL, napi_enumerable, NULL},
      {"pipelineFree", NULL, js_pipeline_free, NULL, NULL, NULL, napi_enumerable, NULL},
      {"pipelineDecideAsync", NULL, js_pipeline_decide_async, NULL, NULL, NULL, napi_enumerable, NULL},
      {"devices", NULL, js_devices, NULL, NULL, NULL, napi_enumerable, NULL},
      {"isAllowed", NULL, js_is_allowed, NULL, NULL, NULL, napi_enumerable, NULL},
      {"isAllowedAsync", NULL, js_is_allowed_async, NULL, NULL, NULL, napi_enumerable, NULL},
      {"whatIsAllowed", NULL, js_what_is_allowed, NULL, NULL, NULL, napi_enumerable, NULL},
      {"whatIsAllowedObl", NULL, js_what_is_allowed_obl, NULL, NULL, NULL, napi_enumerable, NULL},
      {"wordsPerRequest", NULL, js_words, NULL, NULL, NULL, napi_enumerable, NULL},
      {"layoutSizes", NULL, js_layout_sizes, NULL, NULL, NULL, napi_enumerable, NULL},
      {"deviceCount", NULL, js_device_count, NULL, NULL, NULL, napi_enumerable, NULL},
      {"lastError", NULL, js_last_error, NULL, NULL, NULL, napi_enumerable, NULL},
  };
  if (napi_define_properties(env, exports, sizeof d / sizeof d[0], d) != napi_ok) return NULL;
  return exports;
}

NAPI_MODULE(NODE_GYP_MODULE_NAME, init)
