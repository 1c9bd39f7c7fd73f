/* acs_napi.c — N-API addon over the C ABI of libacs_mi355x.so (include/acs_mi355x.h).
 *
 * The binding a TypeScript host (src/core/accessController.ts) loads to hand
 * packed request batches to the MI355X evaluator; see INTEGRATION.md for the
 * TS side.  Plain C over node_api.h (N-API 8, Node >= 12.22): no V8 headers, no
 * node-gyp needed — access-control-srv_amd/acs_mi355x/build.py compiles it with gcc.
 *
 * JS surface:
 *   compile(blob: Uint8Array, device: number) -> handle      acs_compile
 *   free(handle)                                             acs_free
 *   isAllowed(handle, batch) -> Uint8Array(8 n)              acs_is_allowed (sync)
 *   isAllowedAsync(handle, batch) -> Promise<Uint8Array>     same, on the libuv pool
 *   whatIsAllowed(handle, batch) -> {bits, obl, oblN, out}   acs_what_is_allowed
 *   wordsPerRequest(handle), layoutSizes(), deviceCount(), lastError()
 * `batch` = {n, hdr, res, subj, act, roles, arena, rx, rxCols, rxRows,
 *            cand, candWords, candWp, candWr, candRows[, roleKey, roleRowsBits, roleRows]}:
 *            typed arrays / Buffers in the
 * layout of csrc/acs_layout.h (what acs_mi355x/encoder.py produces).
 */
#define NAPI_VERSION 8
#include <node_api.h>
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

static napi_value throw_acs(napi_env env, const char* what) {
  char msg[512];
  const char* e = acs_last_error();
  snprintf(msg, sizeof msg, "%s", e && *e ? e : what);
  napi_throw_error(env, NULL, msg);
  return NULL;
}

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

/* JS batch object -> acs_req_batch (pointers into the JS buffers; caller keeps them alive). */
static int read_batch(napi_env env, napi_value obj, acs_req_batch* b) {
  size_t len;
  void* p;
  memset(b, 0, sizeof *b);
  if (prop_u32(env, obj, "n", &b->n)) return -1;
  if (prop_bytes(env, obj, "hdr", &p, &len)) return -1;
  b->hdr = p;
  if (prop_bytes(env, obj, "res", &p, &len)) return -1;
  b->res = p;
  if (prop_bytes(env, obj, "subj", &p, &len)) return -1;
  b->subj = p;
  if (prop_bytes(env, obj, "act", &p, &len)) return -1;
  b->act = p;
  if (prop_bytes(env, obj, "roles", &p, &len)) return -1;
  b->roles = (const uint32_t*)p;
  if (prop_bytes(env, obj, "arena", &p, &len)) return -1;
  b->arena = (const uint32_t*)p;
  b->arena_words = len / 4;
  if (prop_bytes(env, obj, "rx", &p, &len)) return -1;
  b->rx = (const uint8_t*)p;
  if (prop_u32(env, obj, "rxCols", &b->rx_cols) || prop_u32(env, obj, "rxRows", &b->rx_rows)) return -1;
  if (prop_bytes(env, obj, "cand", &p, &len)) return -1;
  b->cand = (const uint32_t*)p;
  if (prop_u32(env, obj, "candWords", &b->cand_words) || prop_u32(env, obj, "candWp", &b->cand_wp) ||
      prop_u32(env, obj, "candWr", &b->cand_wr) || prop_u32(env, obj, "candRows", &b->cand_rows))
    return -1;
  /* optional role factor (large stores): roleKey [n] u32, roleRowsBits, roleRows */
  if (prop_bytes(env, obj, "roleKey", &p, &len)) return -1;
  b->role_key = (const uint32_t*)p;
  if (prop_bytes(env, obj, "roleRowsBits", &p, &len)) return -1;
  b->role_rows_bits = (const uint32_t*)p;
  if (prop_u32(env, obj, "roleRows", &b->role_rows)) return -1;
  if (!b->role_key) b->role_rows = 0;
  return 0;
}

static acs_tables* get_handle(napi_env env, napi_value v) {
  void* h = NULL;
  if (napi_get_value_external(env, v, &h) != napi_ok) return NULL;
  return (acs_tables*)h;
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

/* ------------------------------------------------------------------ compile / free */
static napi_value js_compile(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2], out;
  void* blob;
  size_t len;
  int32_t device = 0;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc < 1 || get_bytes(env, argv[0], &blob, &len) || !blob) {
    napi_throw_type_error(env, NULL, "compile(blob: Uint8Array, device?: number)");
    return NULL;
  }
  if (argc > 1) CHECK(env, napi_get_value_int32(env, argv[1], &device));
  acs_tables* t = acs_compile(blob, len, device);
  if (!t) return throw_acs(env, "acs_compile");
  CHECK(env, napi_create_external(env, t, NULL, NULL, &out));
  return out;
}

static napi_value js_free(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  if (argc > 0) acs_free(get_handle(env, argv[0]));
  return NULL;
}

/* ------------------------------------------------------------------ isAllowed (sync) */
static napi_value js_is_allowed(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  acs_req_batch b;
  void* out;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  acs_tables* t = argc == 2 ? get_handle(env, argv[0]) : NULL;
  if (!t || read_batch(env, argv[1], &b)) {
    napi_throw_type_error(env, NULL, "isAllowed(handle, batch)");
    return NULL;
  }
  napi_value arr = new_u8(env, (size_t)b.n * sizeof(acs_decision), &out);
  if (!arr) return NULL;
  if (acs_is_allowed(t, &b, (acs_decision*)out) != 0) return throw_acs(env, "acs_is_allowed");
  return arr;
}

/* ------------------------------------------------------------------ isAllowed (async) */
typedef struct {
  napi_async_work work;
  napi_deferred deferred;
  napi_ref keep_batch, keep_out;
  acs_tables* t;
  acs_req_batch b;
  acs_decision* out;
  int rc;
  char err[256];
} async_req;

static void exec_is_allowed(napi_env env, void* data) {
  (void)env;
  async_req* r = (async_req*)data;
  r->rc = acs_is_allowed(r->t, &r->b, r->out);
  if (r->rc) snprintf(r->err, sizeof r->err, "acs_is_allowed: %s", acs_last_error());
}

static void done_is_allowed(napi_env env, napi_status status, void* data) {
  async_req* r = (async_req*)data;
  napi_value out;
  napi_get_reference_value(env, r->keep_out, &out);
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
  async_req* r = (async_req*)calloc(1, sizeof *r);
  if (!r) {
    napi_throw_error(env, NULL, "out of memory");
    return NULL;
  }
  r->t = argc == 2 ? get_handle(env, argv[0]) : NULL;
  if (!r->t || read_batch(env, argv[1], &r->b)) {
    free(r);
    napi_throw_type_error(env, NULL, "isAllowedAsync(handle, batch)");
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
  CHECK(env, napi_queue_async_work(env, r->work));
  return promise;
}

/* ------------------------------------------------------------------ whatIsAllowed */
static napi_value js_what_is_allowed(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2], res;
  acs_req_batch b;
  void *bits, *obl, *obl_n, *out;
  CHECK(env, napi_get_cb_info(env, info, &argc, argv, NULL, NULL));
  acs_tables* t = argc == 2 ? get_handle(env, argv[0]) : NULL;
  if (!t || read_batch(env, argv[1], &b)) {
    napi_throw_type_error(env, NULL, "whatIsAllowed(handle, batch)");
    return NULL;
  }
  const size_t w = acs_wia_words_per_request(t);
  napi_value a_bits = new_u32(env, (size_t)b.n * w, &bits);
  napi_value a_obl = new_u32(env, (size_t)b.n * ACS_OBL_MAX * 2, &obl);
  napi_value a_obl_n = new_u32(env, b.n, &obl_n);
  napi_value a_out = new_u8(env, (size_t)b.n * sizeof(acs_decision), &out);
  if (!a_bits || !a_obl || !a_obl_n || !a_out) return NULL;
  if (acs_what_is_allowed(t, &b, (uint32_t*)bits, (uint32_t*)obl, (uint32_t*)obl_n, (acs_decision*)out) != 0)
    return throw_acs(env, "acs_what_is_allowed");
  CHECK(env, napi_create_object(env, &res));
  CHECK(env, napi_set_named_property(env, res, "bits", a_bits));
  CHECK(env, napi_set_named_property(env, res, "obl", a_obl));
  CHECK(env, napi_set_named_property(env, res, "oblN", a_obl_n));
  CHECK(env, napi_set_named_property(env, res, "out", a_out));
  return res;
}

/* whatIsAllowedObl(handle, batch, idx: Uint32Array, chunks, cap) -> {obl, oblN}: the
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
  acs_tables* t = argc == 5 ? get_handle(env, argv[0]) : NULL;
  if (!t || read_batch(env, argv[1], &b) || get_bytes(env, argv[2], &idx, &idx_len) || idx_len % 4 ||
      napi_get_value_uint32(env, argv[3], &chunks) != napi_ok || napi_get_value_uint32(env, argv[4], &cap) != napi_ok ||
      chunks == 0 || chunks > 64 || cap == 0 || cap > (1u << 20)) {
    napi_throw_type_error(env, NULL, "whatIsAllowedObl(handle, batch, idx: Uint32Array, chunks 1..64, cap 1..2^20)");
    return NULL;
  }
  const size_t m = idx_len / 4;
  napi_value a_obl = new_u32(env, m * chunks * (size_t)cap * 2, &obl);
  napi_value a_obl_n = new_u32(env, m * chunks, &obl_n);
  if (!a_obl || !a_obl_n) return NULL;
  if (acs_what_is_allowed_obl(t, &b, (const uint32_t*)idx, m, chunks, cap, (uint32_t*)obl, (uint32_t*)obl_n) != 0)
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
  acs_tables* t = argc ? get_handle(env, argv[0]) : NULL;
  CHECK(env, napi_create_uint32(env, t ? acs_wia_words_per_request(t) : 0, &v));
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
  const napi_property_descriptor d[] = {
      {"compile", NULL, js_compile, NULL, NULL, NULL, napi_enumerable, NULL},
      {"free", NULL, js_free, NULL, NULL, NULL, napi_enumerable, NULL},
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
