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
#include <mutex>
#include <string>
#include <vector>

#include "../../include/acs_mi355x.h"
#include "acs_eval.h"

#include <hipcub/hipcub.hpp>
#include <rocprim/device/device_radix_sort.hpp>

// Coherence-sort algorithm.  rocprim's default dispatch runs a block sort + ~10 merge
// passes for n <= 2^20 (c2's whole 1M batch: 0.17 ms); a merge-sort limit of 0 forces the
// onesweep radix passes over [0, end_bit).  Both are stable sorts of the same keys, so the
// permutation is identical.  -DACS_SORT_HIPCUB keeps the default dispatch (A/B variant).
using SortCfg = rocprim::radix_sort_config<rocprim::default_config, rocprim::default_config,
                                           rocprim::default_config, 0>;
static hipError_t sort_pairs(void* tmp, size_t& bytes, const uint32_t* kin, uint32_t* kout,
                             const uint32_t* vin, uint32_t* vout, int n, int end_bit, hipStream_t s) {
#if defined(ACS_SORT_HIPCUB)
  return hipcub::DeviceRadixSort::SortPairs(tmp, bytes, kin, kout, vin, vout, n, 0, end_bit, s);
#else
  return rocprim::radix_sort_pairs<SortCfg>(tmp, bytes, kin, kout, vin, vout, (size_t)n, 0u,
                                            (unsigned)end_bit, s);
#endif
}

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

// Sort key that makes a wave share its request class (one candidate row) and action — or,
// with a role factor, its role key — so table-driven branches are wave-uniform:
// [bucket:16 | action id or role key:16].  Class ids come heaviest-first from the host (most
// candidate nodes), and unfiltered requests (PCOL_ALL) take bucket 0, so the longest
// waves start first and the launch has no long tail.  Unfiltered requests group by
// their first entity id.
// The low field keeps `lowbits` bits (role keys are dense, so all of them; action ids and
// entity ids are folded mod 2^lowbits): fewer key bits, fewer onesweep passes.  A fold
// collision only merges two groups, which costs coherence, never correctness.
__global__ __launch_bounds__(BLOCK) void sort_keys_kernel(Batch B, uint32_t lowbits, uint32_t* __restrict__ keys,
                                                          uint32_t* __restrict__ idx) {
  const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
  if (k >= B.n) return;
  const ReqHdr h = B.hdr[k];
  const uint32_t cls = h.flags >> RQ_PCOL_SHIFT;
  uint32_t low = B.role_key ? B.role_key[k] : (h.nact ? B.act[k].value : 0u), bucket = cls + 1;
  if (cls >= B.cand_rows) {
    bucket = 0;
    for (uint32_t j = 0; j < h.nres; ++j) {
      const ReqRes q = B.res[(size_t)j * B.n + k];
      if (q.kind & K_ENT) {
        low = q.value;
        break;
      }
    }
  }
  keys[k] = (bucket << lowbits) | (low & ((1u << lowbits) - 1u));
  idx[k] = k;
}

// Dynamic LDS per wave: one W-word union row when W <= LDS_FILTER_WORDS; for longer rows
// (large stores) a LDS_PREFIX_WORDS union prefix (sets + policies at c5) and a 64-entry
// (class, role key) list for the rest — 8 KB per 256-thread block, so the block's LDS
// (32 KB attribute staging + filter) still allows 4 blocks per CU.
constexpr uint32_t LDS_FILTER_WORDS = 1024;
constexpr uint32_t LDS_PREFIX_WORDS = 448;
constexpr uint32_t LDS_LIST_WORDS = 64;
// Candidate filter of a wave, built with every lane present before any lane diverges.  A
// request's row is its class row, AND-ed with its role-factor row when the batch has one.
// With an LDS row (`lds` = this wave's W-word region, W <= LDS_FILTER_WORDS) the filter is
// the OR of the rows of all the wave's active requests, however many (class, role key)
// pairs the wave spans.  With rows too long for LDS (large stores) it keeps up to 4 row
// pointer pairs, or — a more mixed wave — the pairs in this wave's LDS list, OR-ed word by
// word.  An unfiltered request (PCOL_ALL) disables filtering for its wave.
__device__ inline Filter wave_filter(const Batch& B, bool valid, uint32_t cls, uint32_t rk, uint32_t* lds,
                                     uint32_t* list) {
  Filter F{};
  F.wp = B.cand_wp;
  F.wr = B.cand_wr;
  F.cand = B.cand;
  F.rbits = B.role_bits;
  F.nroles = B.role_key ? B.role_rows : 0u;
  F.W = B.cand_words;
  F.all = B.cand == nullptr;
  const uint32_t lane = threadIdx.x & 63u, W = B.cand_words;
  // the LDS union covers the whole row, or (long rows) the set + policy prefix
  const uint32_t LW = W <= LDS_FILTER_WORDS ? W : (W < LDS_PREFIX_WORDS ? W : LDS_PREFIX_WORDS);
  F.lds_n = LW;
  if (lds && !F.all)
    for (uint32_t w = lane; w < LW; w += 64) lds[w] = 0u;
  const uint32_t key = cls << 16 | (rk < F.nroles ? rk : 0xFFFFu);
  uint32_t n = 0;
  uint64_t pending = __ballot(valid);
  while (pending && !F.all) {
    const int leader = __builtin_ctzll(pending);
    const uint32_t k = __builtin_amdgcn_readlane(key, leader), c = k >> 16, r = k & 0xFFFFu;
    if (c == PCOL_ALL || c >= B.cand_rows) {
      F.all = true;
      break;
    }
    const uint32_t* row = B.cand + (size_t)c * W;
    const uint32_t* rrow = r < F.nroles ? B.role_bits + (size_t)r * W : nullptr;
    if (lds)
      for (uint32_t w = lane; w < LW; w += 64) lds[w] |= row[w] & (rrow ? rrow[w] : ~0u);
    if (list) {
      if (lane == 0) list[n] = k;  // at most 64 distinct (class, role key) pairs per wave
      if (n < 4) {
        if (n == 0) { F.row[0] = row; F.rrow[0] = rrow; }
        else if (n == 1) { F.row[1] = row; F.rrow[1] = rrow; }
        else if (n == 2) { F.row[2] = row; F.rrow[2] = rrow; }
        else { F.row[3] = row; F.rrow[3] = rrow; }
      }
    }
    ++n;
    pending &= ~__ballot(valid && key == k);
  }
  if (!F.all && n == 0) F.all = true;  // no active lane: nothing is evaluated anyway
  if (!F.all && lds) F.lds = lds;
  if (!F.all && list && n > 4) {
    F.list = list;
    F.nlist = n;
  }
  return F;
}

extern __shared__ uint32_t acs_dyn_lds[];

__device__ inline uint32_t lds_wave_words(const Batch& B) {
  return B.cand_words <= LDS_FILTER_WORDS ? B.cand_words : LDS_PREFIX_WORDS + LDS_LIST_WORDS;
}

__device__ inline uint32_t* wave_lds_row(const Batch& B) {
  if (!B.cand) return nullptr;
  return acs_dyn_lds + (threadIdx.x >> 6) * lds_wave_words(B);
}

__device__ inline uint32_t* wave_lds_list(const Batch& B) {
  if (!B.cand || B.cand_words <= LDS_FILTER_WORDS) return nullptr;
  return acs_dyn_lds + (threadIdx.x >> 6) * lds_wave_words(B) + LDS_PREFIX_WORDS;
}

__device__ inline uint32_t request_pcol(const ReqHdr& h) {
  return (h.flags & RQ_NO_TARGET) ? PCOL_ALL : (h.flags >> RQ_PCOL_SHIFT);
}

#if defined(ACS_PHASE_PROF)
__device__ unsigned long long acs_phase_acc[PH_N];
#endif

// XCD-aware block order.  The dispatcher deals workgroups to the 8 XCDs round-robin
// (block b -> XCD b % 8), and each XCD has its own L2.  After the coherence sort, runs of
// neighbouring blocks share a request class and so the same candidate nodes; remapping
// each group of 8*G consecutive blocks so that XCD x takes the logical blocks
// [x*G, x*G+G) of the group keeps a class's table reads in one L2 instead of eight.
// Groups stay in launch order (heaviest classes first); the partial last group is
// identity-mapped.  G = 0 disables the remap.
#ifndef ACS_XCD_GROUP
#define ACS_XCD_GROUP 0
#endif
__device__ inline uint32_t xcd_block(uint32_t b, uint32_t nb) {
  constexpr uint32_t G = ACS_XCD_GROUP, NX = 8;
  if (G == 0) return b;
  const uint32_t span = NX * G;
  if (b >= nb / span * span) return b;
  const uint32_t r = b % span;
  return b - r + (r % NX) * G + r / NX;
}

// K1: one request per lane; its resource attributes are staged in this lane's LDS column.
#ifndef ACS_K1_WAVES_PER_EU
#define ACS_K1_WAVES_PER_EU 4  // measured: 4 waves/SIMD (VGPR <= 128) beats 3 (+12% c2, +13% c3), 5+ spill
#endif
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(ACS_K1_WAVES_PER_EU))) void is_allowed_kernel(Tables T, Batch B, const uint32_t* __restrict__ perm,
                                                           Decision* __restrict__ out) {
  __shared__ ReqRes stage[LDS_SLOTS * BLOCK];
  const uint32_t k = xcd_block(blockIdx.x, gridDim.x) * BLOCK + threadIdx.x;
  const bool in = k < B.n;
  const uint32_t i = in ? (perm ? perm[k] : k) : 0u;
  ReqHdr h{};
  if (in) h = B.hdr[i];
  bool done = true;
  Decision d{};
  if (in) d = early_decision(h, &done);
  const Filter F = wave_filter(B, in && !done, request_pcol(h), B.role_key && in ? B.role_key[i] : 0xFFFFu, wave_lds_row(B),
                               wave_lds_list(B));
#if defined(ACS_PHASE_PROF)
  uint64_t prof_lane[PH_N] = {};
  if (!in) done = true;
#else
  if (!in) return;
#endif
  if (!done) {
    ReqRes* col = stage + threadIdx.x;
    const uint32_t nq = h.nres < LDS_SLOTS ? h.nres : LDS_SLOTS;
    for (uint32_t j = 0; j < nq; ++j) col[j * BLOCK] = B.res[(size_t)j * B.n + i];
#if defined(ACS_PHASE_PROF)
    const ReqLds R(T, B, i, h, col, BLOCK);
    d = is_allowed_t(R, F);
    for (int k = 0; k < PH_N; ++k) prof_lane[k] = R.prof[k];
#else
    d = is_allowed_t(ReqLds(T, B, i, h, col, BLOCK), F);
#endif
  }
#if !defined(ACS_PHASE_PROF)
  out[i] = d;
#else
  if (in) out[i] = d;
  for (int k = 0; k < PH_N; ++k) {  // lane-cycles per phase, one atomic per wave
    uint64_t v = prof_lane[k];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63u) == 0) atomicAdd(&acs_phase_acc[k], (unsigned long long)v);
  }
#endif
}

// K2: whatIsAllowed inclusion bitset + maskedProperty log, one request per lane (perm
// order k).  The bitset goes to a word-major scratch buffer tmp[words][n] at column k, so a
// wave's zeroing and bit updates are coalesced 256-B accesses; bitset_transpose_kernel
// then writes each column to its request's row of the [n][words] output.
__global__ __launch_bounds__(BLOCK) void what_is_allowed_kernel(Tables T, Batch B, const uint32_t* __restrict__ perm,
                                                                uint32_t words, uint32_t* __restrict__ tmp,
                                                                uint32_t* __restrict__ obl,
                                                                uint32_t* __restrict__ obl_n,
                                                                Decision* __restrict__ out) {
  __shared__ ReqRes stage[LDS_SLOTS * BLOCK];
  const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
  const bool in = k < B.n;
  const uint32_t i = in ? (perm ? perm[k] : k) : 0u;
  ReqHdr h{};
  if (in) h = B.hdr[i];
  const bool host = (h.flags & RQ_HOST) != 0;
  const Filter F = wave_filter(B, in && !host, request_pcol(h), B.role_key && in ? B.role_key[i] : 0xFFFFu,
                               wave_lds_row(B), wave_lds_list(B));
  if (!in) return;
  uint32_t* col = tmp + k;
  for (uint32_t w = 0; w < words; ++w) col[(size_t)w * B.n] = 0;
  OblLog log{obl + (size_t)i * 2 * OBL_MAX, 0, false};
  Decision d{};
  if (host) {
    d.flags = OF_HOST_REQ;
  } else {
    ReqRes* scol = stage + threadIdx.x;
    const uint32_t nq = h.nres < LDS_SLOTS ? h.nres : LDS_SLOTS;
    for (uint32_t j = 0; j < nq; ++j) scol[j * BLOCK] = B.res[(size_t)j * B.n + i];
    d = what_is_allowed_t(ReqLds(T, B, i, h, scol, BLOCK), F, col, B.n, log);
  }
  obl_n[i] = (d.flags & OF_ERR) ? 0u : log.n;
  out[i] = d;
}

// Obligation-only pass for requests idx[0..m) — those whose K2 log
// overflowed (OF_OBL_OVERFLOW) — with a cap-entry maskedProperty log and no bitset, so long
// obligation lists stay on the GPU instead of the host path.  whatIsAllowed keeps no state
// across policy sets except the log, so the sets are cut into `chunks` contiguous ranges
// and lane k evaluates range c = k / m of request idx[k % m]: chunks x more waves, each
// 1/chunks as long (the pass is one wave's traversal deep: 461 waves at c4).
// obl[c][j] / obl_n[c][j]: range c's log and total push count (> cap: re-run with that
// cap); a request's log is the concatenation over c.  An index outside the batch writes
// 0xFFFFFFFF and reads nothing.
__global__ __launch_bounds__(BLOCK) void what_is_allowed_obl_kernel(Tables T, Batch B, const uint32_t* __restrict__ idx,
                                                                    uint32_t m, uint32_t chunks, uint32_t cap,
                                                                    uint32_t* __restrict__ obl,
                                                                    uint32_t* __restrict__ obl_n) {
  __shared__ ReqRes stage[LDS_SLOTS * BLOCK];
  // each range's lanes start on a wave boundary (m padded to 64): the set range, and with it
  // the candidate iteration, is wave-uniform
  const uint64_t mp = ((uint64_t)m + 63u) & ~(uint64_t)63u;
  const uint64_t t = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  const uint32_t c = (uint32_t)(t / mp), j = (uint32_t)(t % mp);
  const bool live = c < chunks && j < m;
  const uint64_t k = (uint64_t)c * m + j;  // output slot [c][j]
  const uint32_t i = live ? idx[j] : 0u;
  const bool in = live && i < B.n;
  ReqHdr h{};
  if (in) h = B.hdr[i];
  const bool host = (h.flags & RQ_HOST) != 0;
  const Filter F = wave_filter(B, in && !host, request_pcol(h), B.role_key && in ? B.role_key[i] : 0xFFFFu,
                               wave_lds_row(B), wave_lds_list(B));
  if (!live) return;
  if (!in) {
    obl_n[k] = 0xFFFFFFFFu;
    return;
  }
  uint32_t total = 0;
  if (!host) {
    OblLog log{obl + k * 2 * cap, 0, false, cap, 0};
    ReqRes* scol = stage + threadIdx.x;
    const uint32_t nq = h.nres < LDS_SLOTS ? h.nres : LDS_SLOTS;
    for (uint32_t q = 0; q < nq; ++q) scol[q * BLOCK] = B.res[(size_t)q * B.n + i];
    const uint32_t s0 = (uint32_t)((uint64_t)T.n_sets * c / chunks), s1 = (uint32_t)((uint64_t)T.n_sets * (c + 1) / chunks);
    const Decision d = what_is_allowed_t(ReqLds(T, B, i, h, scol, BLOCK), F, nullptr, 0, log, s0, s1);
    total = (d.flags & OF_ERR) ? 0u : log.total;
  }
  obl_n[k] = total;
}

// tmp[words][n] (column k = the k-th request in perm order) -> bits[perm[k]][words].  A
// 256-thread block moves a 64-column x 64-word tile through LDS: every load instruction
// reads 256 contiguous bytes of a tmp row, every store instruction writes 256 contiguous
// bytes (64 words) of one output row — both fully coalesced (the previous 32-word tile
// stored 4-byte pieces of 16 rows per instruction: 1.29 ms for 1M c4 rows).
// Tile order (ACS_TP_MODE): output rows are `words` u32 long (c4: 1400 B), so a row's
// 256-B segments are not line-aligned and neighbouring segments share cache lines.
//   0: grid (column tiles, word tiles) — a row's segments are written far apart in time;
//   1: grid (word tiles, column tiles) — a row's segments are written by consecutive blocks;
//   2: one block per column tile walks all word tiles — each row written by one block.
#ifndef ACS_TP_MODE
#define ACS_TP_MODE 0
#endif
constexpr uint32_t TP_COLS = 64, TP_WORDS = 64;
__device__ inline void transpose_tile(uint32_t (*tile)[TP_COLS + 1], const uint32_t* __restrict__ tmp, uint32_t n,
                                      uint32_t words, const uint32_t* __restrict__ perm, uint32_t* __restrict__ bits,
                                      uint32_t k0, uint32_t w0) {
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  for (uint32_t r = wave; r < TP_WORDS; r += BLOCK / 64) {
    const uint32_t w = w0 + r, k = k0 + lane;
    tile[r][lane] = (w < words && k < n) ? tmp[(size_t)w * n + k] : 0u;
  }
  __syncthreads();
  const uint32_t w = w0 + lane;
  for (uint32_t r = wave; r < TP_COLS; r += BLOCK / 64) {
    const uint32_t k = k0 + r;
    if (k >= n) break;
    if (w < words) bits[(size_t)(perm ? perm[k] : k) * words + w] = tile[lane][r];
  }
}
__global__ __launch_bounds__(BLOCK) void bitset_transpose_kernel(const uint32_t* __restrict__ tmp, uint32_t n,
                                                                 uint32_t words, const uint32_t* __restrict__ perm,
                                                                 uint32_t* __restrict__ bits) {
  __shared__ uint32_t tile[TP_WORDS][TP_COLS + 1];
#if ACS_TP_MODE == 2
  for (uint32_t w0 = 0; w0 < words; w0 += TP_WORDS) {
    transpose_tile(tile, tmp, n, words, perm, bits, blockIdx.x * TP_COLS, w0);
    __syncthreads();  // the tile is reused by the next word range
  }
#elif ACS_TP_MODE == 1
  transpose_tile(tile, tmp, n, words, perm, bits, blockIdx.y * TP_COLS, blockIdx.x * TP_WORDS);
#else
  transpose_tile(tile, tmp, n, words, perm, bits, blockIdx.x * TP_COLS, blockIdx.y * TP_WORDS);
#endif
}
static dim3 transpose_grid(uint32_t n, uint32_t words) {
  const uint32_t ct = (n + TP_COLS - 1) / TP_COLS, wt = (words + TP_WORDS - 1) / TP_WORDS;
#if ACS_TP_MODE == 2
  (void)wt;
  return dim3(ct);
#elif ACS_TP_MODE == 1
  return dim3(wt, ct);
#else
  return dim3(ct, wt);
#endif
}

__global__ __launch_bounds__(BLOCK) void shard_key_kernel(Tables T, const Decision* __restrict__ d, uint32_t n,
                                                          ShardBase b, uint64_t* __restrict__ keys) {
  const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
  if (i < n) keys[i] = shard_key(T, d[i], b);
}

__global__ __launch_bounds__(BLOCK) void shard_decode_kernel(const uint64_t* __restrict__ keys, uint32_t n,
                                                             Decision* __restrict__ out) {
  const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
  if (i < n) out[i] = shard_decode(keys[i]);
}

size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

size_t filter_lds_bytes(const Batch& B) {
  if (!B.cand) return 0;
  return (size_t)(BLOCK / 64) * (B.cand_words <= LDS_FILTER_WORDS ? B.cand_words : LDS_PREFIX_WORDS + LDS_LIST_WORDS) * 4;
}

}  // namespace

struct acs_tables {
  int device = 0;
  void* dev = nullptr;  // one allocation holding every section
  Tables view{};
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  float last_ms = -1.f;
  int sort = 1;         // coherence sort of each batch (ACS_OPT_SORT)
  // ACS_OPT_TIMING: HIP events recorded on the launch stream around every eval kernel
  static constexpr int RING = 256;
  int timing = 0;
  hipEvent_t tev[2 * RING] = {};
  uint64_t launches = 0;
  // sort workspace, grown on demand: keys/idx double buffers + hipcub temp storage
  void* ws = nullptr;
  size_t ws_bytes = 0;
  // K2 word-major bitset scratch ([words][n] u32), grown on demand
  void* wbuf = nullptr;
  size_t wbuf_bytes = 0;
  // host-buffer entry points (internal stream, events, workspace) may be called from
  // several host threads at once (e.g. the N-API addon's libuv pool): one at a time
  std::mutex mu;
};

extern "C" {

const char* acs_last_error(void) { return g_err.c_str(); }

#if defined(ACS_PHASE_PROF)
// Profiling build only: read and reset the per-phase lane-cycle sums.
int acs_phase_read(unsigned long long* out, int n) {
  unsigned long long h[PH_N] = {}, z[PH_N] = {};
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpyFromSymbol(h, HIP_SYMBOL(acs_phase_acc), sizeof h));
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(acs_phase_acc), z, sizeof z));
  for (int k = 0; k < n && k < PH_N; ++k) out[k] = h[k];
  return PH_N;
}
#endif

#if defined(ACS_CHECK_UNIFORM)
// Debug build only: read and reset the non-uniform table-load counters.
int acs_debug_read(unsigned long long* out, int n) {
  unsigned long long h[4] = {}, z[4] = {};
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpyFromSymbol(h, HIP_SYMBOL(acs_nonuniform), sizeof h));
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(acs_nonuniform), z, sizeof z));
  for (int k = 0; k < n && k < 4; ++k) out[k] = h[k];
  return 4;
}
#endif

int acs_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int acs_layout_sizes(uint32_t* out, int n) {
  const uint32_t s[5] = {sizeof(NodeRec), sizeof(RuleResAttr), sizeof(ReqHdr), sizeof(ReqRes), sizeof(Decision)};
  for (int k = 0; k < n && k < 5; ++k) out[k] = s[k];
  return 5;
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
  const size_t sz[6] = {h.n_sets * sizeof(NodeRec), h.n_pols * sizeof(NodeRec), h.n_rules * sizeof(NodeRec),
                        h.n_rres * sizeof(RuleResAttr), h.n_pairs * sizeof(Pair), h.n_u32pool * sizeof(uint32_t)};
  size_t off[6], total = 0, src = align16(sizeof h);
  for (int k = 0; k < 6; ++k) {
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
  const size_t alloc = total + 64;  // clamp window [base, base + total] for 64-B record loads
  if (hipSetDevice(device) != hipSuccess || hipMalloc(&t->dev, alloc) != hipSuccess ||
      hipMemcpy(t->dev, (const char*)blob + src, total, hipMemcpyHostToDevice) != hipSuccess ||
      hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&t->ev0) != hipSuccess || hipEventCreate(&t->ev1) != hipSuccess) {
    fail("acs_compile: device allocation / upload failed");
    acs_free(t);
    return nullptr;
  }
  char* base = (char*)t->dev;
  t->view.sets = (const NodeRec*)(base + off[0]);
  t->view.pols = (const NodeRec*)(base + off[1]);
  t->view.rules = (const NodeRec*)(base + off[2]);
  t->view.rres = (const RuleResAttr*)(base + off[3]);
  t->view.pairs = (const Pair*)(base + off[4]);
  t->view.u32pool = (const uint32_t*)(base + off[5]);
  t->view.n_sets = h.n_sets;
  t->view.n_pols = h.n_pols;
  t->view.n_rules = h.n_rules;
  t->view.id_user = h.id_user;
  t->view.lo = (uint64_t)(uintptr_t)base;
  t->view.hi = (uint64_t)(uintptr_t)base + alloc - 64;
  return t;
}

void acs_free(acs_tables* t) {
  if (!t) return;
  (void)hipSetDevice(t->device);
  if (t->dev) (void)hipFree(t->dev);
  if (t->ev0) (void)hipEventDestroy(t->ev0);
  if (t->ev1) (void)hipEventDestroy(t->ev1);
  if (t->stream) (void)hipStreamDestroy(t->stream);
  if (t->ws) (void)hipFree(t->ws);
  if (t->wbuf) (void)hipFree(t->wbuf);
  for (hipEvent_t e : t->tev)
    if (e) (void)hipEventDestroy(e);
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
  B.cand = b->cand;
  B.cand_words = b->cand_words;
  B.cand_wp = b->cand_wp;
  B.cand_wr = b->cand_wr;
  B.cand_rows = b->cand ? b->cand_rows : 0u;
  B.role_key = b->cand ? b->role_key : nullptr;
  B.role_bits = b->role_rows_bits;
  B.role_rows = b->role_key ? b->role_rows : 0u;
  return B;
}

int acs_set_option(acs_tables* t, int option, int value) {
  if (!t) return fail("acs_set_option: null tables");
  if (option == ACS_OPT_SORT) {
    t->sort = value ? 1 : 0;
    return 0;
  }
  if (option == ACS_OPT_TIMING) {
    if (value && !t->tev[0]) {
      HIP_OK(hipSetDevice(t->device));
      for (hipEvent_t& e : t->tev) HIP_OK(hipEventCreate(&e));
    }
    t->timing = value ? 1 : 0;
    t->launches = 0;
    return 0;
  }
  return fail("acs_set_option: unknown option");
}

// Coherence sort: permutation of request indices ordered by (class, action).
static int coherence_perm(acs_tables* t, const Batch& B, hipStream_t s, const uint32_t** perm) {
  *perm = nullptr;
  if (!t->sort || B.n < 2 * BLOCK) return 0;
  const size_t n = B.n;
#ifndef ACS_SORT_LOWBITS
#define ACS_SORT_LOWBITS 4
#endif
  uint32_t lowbits = ACS_SORT_LOWBITS;  // action / entity ids folded to 4 bits (c2: 16-bit keys, 2 passes)
  if (B.role_key) {
    lowbits = 1;
    while (lowbits < 16 && (B.role_rows - 1) >> lowbits) ++lowbits;
  }
#if defined(ACS_SORT_KEY16)
  lowbits = 16;  // A/B variant: the unfolded 16-bit low field
#endif
  int end_bit = (int)lowbits;  // keys < (cand_rows + 1) << lowbits
  while (end_bit < 32 && (uint64_t(B.cand_rows) >> (end_bit - lowbits)) != 0) ++end_bit;
  if (end_bit < 1) end_bit = 1;
  size_t temp = 0;
  HIP_OK(sort_pairs(nullptr, temp, nullptr, nullptr, nullptr, nullptr, (int)n, end_bit, s));
  const size_t need = 4 * n * sizeof(uint32_t) + temp + 256;
  if (need > t->ws_bytes) {
    if (t->ws) HIP_OK(hipFree(t->ws));
    t->ws = nullptr;
    t->ws_bytes = 0;
    HIP_OK(hipMalloc(&t->ws, need));
    t->ws_bytes = need;
  }
  uint32_t* keys_in = (uint32_t*)t->ws;
  uint32_t* keys_out = keys_in + n;
  uint32_t* idx_in = keys_out + n;
  uint32_t* idx_out = idx_in + n;
  void* tmp = (void*)(((uintptr_t)(idx_out + n) + 255) & ~uintptr_t(255));
  hipLaunchKernelGGL(sort_keys_kernel, dim3((n + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, B, lowbits, keys_in, idx_in);
  HIP_OK(hipGetLastError());
  HIP_OK(sort_pairs(tmp, temp, keys_in, keys_out, idx_in, idx_out, (int)n, end_bit, s));
  *perm = idx_out;
  return 0;
}

int acs_is_allowed_device(acs_tables* t, const acs_req_batch* b, acs_decision* out, void* stream) {
  if (!t || !b) return fail("acs_is_allowed_device: null argument");
  if (b->n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  Batch B = to_batch(b);
  const uint32_t* perm = nullptr;
  if (coherence_perm(t, B, s, &perm)) return -1;
  dim3 grid((b->n + BLOCK - 1) / BLOCK);
  const int slot = (int)(t->launches % acs_tables::RING);
  if (t->timing) HIP_OK(hipEventRecord(t->tev[2 * slot], s));
  hipLaunchKernelGGL(is_allowed_kernel, grid, dim3(BLOCK), filter_lds_bytes(B), s, t->view, B, perm, (Decision*)out);
  HIP_OK(hipGetLastError());
  if (t->timing) {
    HIP_OK(hipEventRecord(t->tev[2 * slot + 1], s));
    t->launches++;
  }
  return 0;
}

int acs_kernel_times(acs_tables* t, float* ms, int n) {
  if (!t || !t->timing) return fail("acs_kernel_times: timing not enabled");
  const int avail = (int)(t->launches < (uint64_t)acs_tables::RING ? t->launches : acs_tables::RING);
  const int m = n < avail ? n : avail;
  for (int k = 0; k < m; ++k) {
    const int slot = (int)((t->launches - m + k) % acs_tables::RING);
    HIP_OK(hipEventSynchronize(t->tev[2 * slot + 1]));
    HIP_OK(hipEventElapsedTime(&ms[k], t->tev[2 * slot], t->tev[2 * slot + 1]));
  }
  return m;
}

int acs_what_is_allowed_device(acs_tables* t, const acs_req_batch* b, uint32_t* bits, uint32_t* obl,
                               uint32_t* obl_n, acs_decision* out, void* stream) {
  if (!t || !b) return fail("acs_what_is_allowed_device: null argument");
  if (b->n == 0) return 0;
  hipStream_t s = (hipStream_t)stream;
  Batch B = to_batch(b);
  const uint32_t* perm = nullptr;
  if (coherence_perm(t, B, s, &perm)) return -1;
  dim3 grid((b->n + BLOCK - 1) / BLOCK);
  const uint32_t words = acs_wia_words_per_request(t);
  const size_t need = (size_t)words * b->n * sizeof(uint32_t);
  if (need > t->wbuf_bytes) {
    if (t->wbuf) HIP_OK(hipFree(t->wbuf));
    t->wbuf = nullptr;
    t->wbuf_bytes = 0;
    HIP_OK(hipMalloc(&t->wbuf, need ? need : 16));
    t->wbuf_bytes = need;
  }
  const int slot = (int)(t->launches % acs_tables::RING);
  if (t->timing) HIP_OK(hipEventRecord(t->tev[2 * slot], s));
  hipLaunchKernelGGL(what_is_allowed_kernel, grid, dim3(BLOCK), filter_lds_bytes(B), s, t->view, B, perm, words,
                     (uint32_t*)t->wbuf, obl, obl_n, (Decision*)out);
  HIP_OK(hipGetLastError());
  if (words) {
    hipLaunchKernelGGL(bitset_transpose_kernel, transpose_grid(b->n, words), dim3(BLOCK), 0, s, (const uint32_t*)t->wbuf, b->n, words, perm, bits);
    HIP_OK(hipGetLastError());
  }
  if (t->timing) {
    HIP_OK(hipEventRecord(t->tev[2 * slot + 1], s));
    t->launches++;
  }
  return 0;
}

constexpr uint32_t OBL_CAP_LIMIT = 1u << 20;

int acs_what_is_allowed_obl_device(acs_tables* t, const acs_req_batch* b, const uint32_t* idx, size_t m,
                                   uint32_t chunks, uint32_t cap, uint32_t* obl, uint32_t* obl_n, void* stream) {
  if (!t || !b || (m && (!idx || !obl || !obl_n))) return fail("acs_what_is_allowed_obl_device: null argument");
  if (cap == 0 || cap > OBL_CAP_LIMIT) return fail("acs_what_is_allowed_obl_device: cap must be in [1, 2^20]");
  if (chunks == 0 || chunks > 64) return fail("acs_what_is_allowed_obl_device: chunks must be in [1, 64]");
  if (m > 0xFFFFFFFFull || m * chunks > 0xFFFFFFFFull) return fail("acs_what_is_allowed_obl_device: too many requests");
  if (m == 0 || b->n == 0) return 0;
  Batch B = to_batch(b);
  const size_t lanes = ((m + 63) & ~(size_t)63) * chunks;  // each range padded to whole waves
  hipLaunchKernelGGL(what_is_allowed_obl_kernel, dim3((unsigned)((lanes + BLOCK - 1) / BLOCK)), dim3(BLOCK),
                     filter_lds_bytes(B), (hipStream_t)stream, t->view, B, idx, (uint32_t)m, chunks, cap, obl, obl_n);
  HIP_OK(hipGetLastError());
  return 0;
}

int acs_shard_keys_device(acs_tables* t, const acs_decision* dec, size_t n, const acs_shard* shard, uint64_t* keys,
                          void* stream) {
  if (!t || !shard || (n && (!dec || !keys))) return fail("acs_shard_keys_device: null argument");
  if (n > 0xFFFFFFFFull) return fail("acs_shard_keys_device: batch too large");
  if (n == 0) return 0;
  const ShardBase b{shard->set_base, shard->pol_base, shard->rule_base};
  hipLaunchKernelGGL(shard_key_kernel, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0,
                     (hipStream_t)stream, t->view, (const Decision*)dec, (uint32_t)n, b, keys);
  HIP_OK(hipGetLastError());
  return 0;
}

int acs_shard_decode_device(const uint64_t* keys, size_t n, acs_decision* out, void* stream) {
  if (n && (!keys || !out)) return fail("acs_shard_decode_device: null argument");
  if (n > 0xFFFFFFFFull) return fail("acs_shard_decode_device: batch too large");
  if (n == 0) return 0;
  hipLaunchKernelGGL(shard_decode_kernel, dim3((unsigned)((n + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0,
                     (hipStream_t)stream, keys, (uint32_t)n, (Decision*)out);
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
  if (b->cand && D.up(b->cand, (size_t)b->cand_rows * b->cand_words * sizeof(uint32_t),
                      (const void**)&D.d.cand, s))
    return -1;
  if (b->role_key && (D.up(b->role_key, n * sizeof(uint32_t), (const void**)&D.d.role_key, s) ||
                      D.up(b->role_rows_bits, (size_t)b->role_rows * b->cand_words * sizeof(uint32_t),
                           (const void**)&D.d.role_rows_bits, s)))
    return -1;
  return 0;
}

}  // namespace

int acs_is_allowed(acs_tables* t, const acs_req_batch* b, acs_decision* out) {
  if (!t || !b || !out) return fail("acs_is_allowed: null argument");
  if (b->n == 0) return 0;
  std::lock_guard<std::mutex> lock(t->mu);
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
  std::lock_guard<std::mutex> lock(t->mu);
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

int acs_what_is_allowed_obl(acs_tables* t, const acs_req_batch* b, const uint32_t* idx, size_t m, uint32_t chunks,
                            uint32_t cap, uint32_t* obl, uint32_t* obl_n) {
  if (!t || !b || (m && (!idx || !obl || !obl_n))) return fail("acs_what_is_allowed_obl: null argument");
  if (cap == 0 || cap > OBL_CAP_LIMIT) return fail("acs_what_is_allowed_obl: cap must be in [1, 2^20]");
  if (chunks == 0 || chunks > 64) return fail("acs_what_is_allowed_obl: chunks must be in [1, 64]");
  if (m == 0) return 0;
  for (size_t k = 0; k < m; ++k)
    if (idx[k] >= b->n) return fail("acs_what_is_allowed_obl: request index outside the batch");
  std::lock_guard<std::mutex> lock(t->mu);
  HIP_OK(hipSetDevice(t->device));
  DevBatch D;
  if (upload_batch(D, b, t->stream)) return -1;
  const size_t lanes = m * chunks;
  void* didx = D.alloc(m * sizeof(uint32_t));
  void* dobl = D.alloc(lanes * 2 * (size_t)cap * sizeof(uint32_t));
  void* dobln = D.alloc(lanes * sizeof(uint32_t));
  if (!didx || !dobl || !dobln) return fail("acs_what_is_allowed_obl: hipMalloc failed");
  HIP_OK(hipMemcpyAsync(didx, idx, m * sizeof(uint32_t), hipMemcpyHostToDevice, t->stream));
  if (acs_what_is_allowed_obl_device(t, &D.d, (const uint32_t*)didx, m, chunks, cap, (uint32_t*)dobl,
                                     (uint32_t*)dobln, t->stream))
    return -1;
  HIP_OK(hipMemcpyAsync(obl, dobl, lanes * 2 * (size_t)cap * sizeof(uint32_t), hipMemcpyDeviceToHost, t->stream));
  HIP_OK(hipMemcpyAsync(obl_n, dobln, lanes * sizeof(uint32_t), hipMemcpyDeviceToHost, t->stream));
  HIP_OK(hipStreamSynchronize(t->stream));
  return 0;
}

}  // extern "C"
