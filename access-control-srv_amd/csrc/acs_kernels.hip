// acs_kernels.hip — gfx950 kernels + C ABI of the MI355X access-control evaluator.
//
// K1 is_allowed_kernel      : one request per lane, 64-request tiles per wave64;
//                             table records via wave-uniform (scalar) loads, request
//                             SoA rows via coalesced vector loads; 8 B decision out.
// K2 what_is_allowed_kernel : same traversal without HR/ACL/condition/combine; writes
//                             the (sets|policies|rules) inclusion bitset + mask log.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/acs_mi355x.h"
#include "acs_eval.h"

using namespace acs;

namespace {

thread_local std::string g_err;

int fail(const std::string& msg) {
  g_err = msg;
  return -1;
}

#define HIP_OK(expr)                                                                        \
  do {                                                                                      \
    hipError_t e_ = (expr);                                                                 \
    if (e_ != hipSuccess) return fail(std::string(#expr ": ") + hipGetErrorString(e_));     \
  } while (0)

constexpr int BLOCK = 256;

__global__ __launch_bounds__(BLOCK) void is_allowed_kernel(Tables T, Batch B, Decision* __restrict__ out) {
  const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= B.n) return;
  out[i] = is_allowed(T, B, i);
}

__global__ __launch_bounds__(BLOCK) void what_is_allowed_kernel(Tables T, Batch B, uint32_t words,
                                                                uint32_t* __restrict__ bits,
                                                                uint32_t* __restrict__ obl,
                                                                uint32_t* __restrict__ obl_n,
                                                                Decision* __restrict__ out) {
  const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
  if (i >= B.n) return;
  uint32_t* my_bits = bits + (size_t)i * words;
  for (uint32_t w = 0; w < words; ++w) my_bits[w] = 0;
  out[i] = what_is_allowed(T, B, i, my_bits, obl + (size_t)i * 2 * OBL_MAX, obl_n + i);
}

size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

}  // namespace

struct acs_tables {
  int device = 0;
  void* dev = nullptr;  // one allocation holding every section
  Tables view{};
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  float last_ms = -1.f;
};

extern "C" {

const char* acs_last_error(void) { return g_err.c_str(); }

int acs_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int acs_layout_sizes(uint32_t* out, int n) {
  const uint32_t s[8] = {sizeof(TargetRec), sizeof(RuleResAttr), sizeof(SetRec), sizeof(PolicyRec),
                         sizeof(RuleRec), sizeof(ReqHdr), sizeof(ReqRes), sizeof(Decision)};
  for (int k = 0; k < n && k < 8; ++k) out[k] = s[k];
  return 8;
}

acs_tables* acs_compile(const void* blob, size_t n_bytes, int device) {
  if (!blob || n_bytes < sizeof(acs_blob_header)) {
    fail("acs_compile: blob too small");
    return nullptr;
  }
  acs_blob_header h;
  std::memcpy(&h, blob, sizeof h);
  if (h.magic != ACS_BLOB_MAGIC || h.version != ACS_ABI_VERSION) {
    fail("acs_compile: bad blob magic/version");
    return nullptr;
  }
  const size_t sz[7] = {h.n_sets * sizeof(SetRec),       h.n_pols * sizeof(PolicyRec), h.n_rules * sizeof(RuleRec),
                        h.n_targets * sizeof(TargetRec), h.n_rres * sizeof(RuleResAttr), h.n_pairs * sizeof(Pair),
                        h.n_u32pool * sizeof(uint32_t)};
  size_t off[7], total = 0, src = align16(sizeof h);
  for (int k = 0; k < 7; ++k) {
    off[k] = total;
    total += align16(sz[k]);
  }
  if (src + total > n_bytes + 0) {
    // the host writes each section 16-byte aligned after the header
    fail("acs_compile: blob shorter than its header declares");
    return nullptr;
  }
  auto* t = new acs_tables();
  t->device = device;
  if (hipSetDevice(device) != hipSuccess || hipMalloc(&t->dev, total ? total : 16) != hipSuccess ||
      hipMemcpy(t->dev, (const char*)blob + src, total, hipMemcpyHostToDevice) != hipSuccess ||
      hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&t->ev0) != hipSuccess || hipEventCreate(&t->ev1) != hipSuccess) {
    fail("acs_compile: device allocation / upload failed");
    acs_free(t);
    return nullptr;
  }
  char* base = (char*)t->dev;
  t->view.sets = (const SetRec*)(base + off[0]);
  t->view.pols = (const PolicyRec*)(base + off[1]);
  t->view.rules = (const RuleRec*)(base + off[2]);
  t->view.targets = (const TargetRec*)(base + off[3]);
  t->view.rres = (const RuleResAttr*)(base + off[4]);
  t->view.pairs = (const Pair*)(base + off[5]);
  t->view.u32pool = (const uint32_t*)(base + off[6]);
  t->view.n_sets = h.n_sets;
  t->view.n_pols = h.n_pols;
  t->view.n_rules = h.n_rules;
  t->view.id_user = h.id_user;
  return t;
}

void acs_free(acs_tables* t) {
  if (!t) return;
  (void)hipSetDevice(t->device);
  if (t->dev) (void)hipFree(t->dev);
  if (t->ev0) (void)hipEventDestroy(t->ev0);
  if (t->ev1) (void)hipEventDestroy(t->ev1);
  if (t->stream) (void)hipStreamDestroy(t->stream);
  delete t;
}

uint32_t acs_wia_words_per_request(const acs_tables* t) {
  return (t->view.n_sets + t->view.n_pols + t->view.n_rules + 31) / 32;
}

float acs_last_kernel_ms(const acs_tables* t) { return t ? t->last_ms : -1.f; }

static Batch to_batch(const acs_req_batch* b) {
  Batch B{};
  B.n = b->n;
  B.hdr = (const ReqHdr*)b->hdr;
  B.res = (const ReqRes*)b->res;
  B.subj = (const Pair*)b->subj;
  B.act = (const Pair*)b->act;
  B.roles = b->roles;
  B.arena = b->arena;
  B.rx = b->rx;
  B.rx_rows = b->rx_rows;
  return B;
}

int acs_is_allowed_device(acs_tables* t, const acs_req_batch* b, acs_decision* out, void* stream) {
  if (!t || !b) return fail("acs_is_allowed_device: null argument");
  if (b->n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  Batch B = to_batch(b);
  dim3 grid((b->n + BLOCK - 1) / BLOCK);
  hipLaunchKernelGGL(is_allowed_kernel, grid, dim3(BLOCK), 0, s, t->view, B, (Decision*)out);
  HIP_OK(hipGetLastError());
  return 0;
}

int acs_what_is_allowed_device(acs_tables* t, const acs_req_batch* b, uint32_t* bits, uint32_t* obl,
                               uint32_t* obl_n, acs_decision* out, void* stream) {
  if (!t || !b) return fail("acs_what_is_allowed_device: null argument");
  if (b->n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  Batch B = to_batch(b);
  dim3 grid((b->n + BLOCK - 1) / BLOCK);
  hipLaunchKernelGGL(what_is_allowed_kernel, grid, dim3(BLOCK), 0, s, t->view, B, acs_wia_words_per_request(t),
                     bits, obl, obl_n, (Decision*)out);
  HIP_OK(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------- host-buffer entry points
namespace {

struct DevBatch {
  std::vector<void*> bufs;
  acs_req_batch d{};
  ~DevBatch() {
    for (void* p : bufs) (void)hipFree(p);
  }
  int up(const void* src, size_t n, const void** dst, hipStream_t s) {
    void* p = nullptr;
    HIP_OK(hipMalloc(&p, n ? n : 16));
    bufs.push_back(p);
    if (n) HIP_OK(hipMemcpyAsync(p, src, n, hipMemcpyHostToDevice, s));
    *dst = p;
    return 0;
  }
  void* alloc(size_t n) {
    void* p = nullptr;
    if (hipMalloc(&p, n ? n : 16) != hipSuccess) return nullptr;
    bufs.push_back(p);
    return p;
  }
};

int upload_batch(DevBatch& D, const acs_req_batch* b, hipStream_t s) {
  D.d = *b;
  const size_t n = b->n;
  if (D.up(b->hdr, n * sizeof(ReqHdr), &D.d.hdr, s) || D.up(b->res, n * QMAX * sizeof(ReqRes), &D.d.res, s) ||
      D.up(b->subj, n * SMAX * sizeof(Pair), &D.d.subj, s) || D.up(b->act, n * AMAX * sizeof(Pair), &D.d.act, s) ||
      D.up(b->roles, n * RMAX * sizeof(uint32_t), (const void**)&D.d.roles, s) ||
      D.up(b->arena, b->arena_words * sizeof(uint32_t), (const void**)&D.d.arena, s) ||
      D.up(b->rx, (size_t)b->rx_cols * b->rx_rows, (const void**)&D.d.rx, s))
    return -1;
  return 0;
}

}  // namespace

int acs_is_allowed(acs_tables* t, const acs_req_batch* b, acs_decision* out) {
  if (!t || !b || !out) return fail("acs_is_allowed: null argument");
  if (b->n == 0) return 0;
  HIP_OK(hipSetDevice(t->device));
  DevBatch D;
  if (upload_batch(D, b, t->stream)) return -1;
  void* dout = D.alloc(b->n * sizeof(Decision));
  if (!dout) return fail("acs_is_allowed: hipMalloc failed");
  HIP_OK(hipEventRecord(t->ev0, t->stream));
  if (acs_is_allowed_device(t, &D.d, (acs_decision*)dout, t->stream)) return -1;
  HIP_OK(hipEventRecord(t->ev1, t->stream));
  HIP_OK(hipMemcpyAsync(out, dout, b->n * sizeof(Decision), hipMemcpyDeviceToHost, t->stream));
  HIP_OK(hipStreamSynchronize(t->stream));
  HIP_OK(hipEventElapsedTime(&t->last_ms, t->ev0, t->ev1));
  return 0;
}

int acs_what_is_allowed(acs_tables* t, const acs_req_batch* b, uint32_t* bits, uint32_t* obl, uint32_t* obl_n,
                        acs_decision* out) {
  if (!t || !b || !bits || !obl || !obl_n || !out) return fail("acs_what_is_allowed: null argument");
  if (b->n == 0) return 0;
  HIP_OK(hipSetDevice(t->device));
  DevBatch D;
  if (upload_batch(D, b, t->stream)) return -1;
  const size_t words = acs_wia_words_per_request(t);
  void* dbits = D.alloc(b->n * words * sizeof(uint32_t));
  void* dobl = D.alloc(b->n * 2 * OBL_MAX * sizeof(uint32_t));
  void* dobln = D.alloc(b->n * sizeof(uint32_t));
  void* dout = D.alloc(b->n * sizeof(Decision));
  if (!dbits || !dobl || !dobln || !dout) return fail("acs_what_is_allowed: hipMalloc failed");
  HIP_OK(hipEventRecord(t->ev0, t->stream));
  if (acs_what_is_allowed_device(t, &D.d, (uint32_t*)dbits, (uint32_t*)dobl, (uint32_t*)dobln,
                                 (acs_decision*)dout, t->stream))
    return -1;
  HIP_OK(hipEventRecord(t->ev1, t->stream));
  HIP_OK(hipMemcpyAsync(bits, dbits, b->n * words * sizeof(uint32_t), hipMemcpyDeviceToHost, t->stream));
  HIP_OK(hipMemcpyAsync(obl, dobl, b->n * 2 * OBL_MAX * sizeof(uint32_t), hipMemcpyDeviceToHost, t->stream));
  HIP_OK(hipMemcpyAsync(obl_n, dobln, b->n * sizeof(uint32_t), hipMemcpyDeviceToHost, t->stream));
  HIP_OK(hipMemcpyAsync(out, dout, b->n * sizeof(Decision), hipMemcpyDeviceToHost, t->stream));
  HIP_OK(hipStreamSynchronize(t->stream));
  HIP_OK(hipEventElapsedTime(&t->last_ms, t->ev0, t->ev1));
  return 0;
}

}  // extern "C"
