// acs_kernels.hip — gfx950 kernels + C ABI of the MI355X access-control evaluator.
//
// K1 is_allowed_kernel      : one request per lane, 64-request tiles per wave64;
//                             table records via wave-uniform (scalar) loads, request
//                             SoA rows via coalesced vector loads; 8 B decision out.
// K2 what_is_allowed_kernel : same traversal without HR/ACL/condition/combine; writes
//                             each request's (sets|policies|rules) inclusion bitset row
//                             once, 16 B at a time, + the maskedProperty log.
// Coherence sort            : hand-written LSD radix sort (8-bit digits) of the
//                             (class, low) keys -> the permutation K1 / K2 run in.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <atomic>
#include <sys/mman.h>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "../../include/acs_mi355x.h"
#include "acs_eval.h"
#include "acs_pool.h"

using namespace acs;

#if defined(ACS_SCAN_COUNT)  // the counting build's kernels carry their own names in traces / PMC passes
#define is_allowed_kernel is_allowed_kernel_scan_count
#define what_is_allowed_kernel what_is_allowed_kernel_scan_count
#endif

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

// A/B switches of experiment builds (acs_mi355x/build.build_variant, `bench.py --lib`), fixed
// at compile time: the product library defines none of them, so no environment variable can
// change how a service evaluates.  (Forms that measured no gain — table replicas over L2
// channels, scalar / one-lane record loads, K2 occupancy and rule prefetch, SoA-instantiated
// compact kernels, unscattered records — were removed after their A/Bs: DESIGN.md §3.)
#ifndef ACS_AB_NO_CUT          // combining loops and the set walk always run to their end
#define ACS_AB_NO_CUT 0
#endif
#ifndef ACS_AB_NO_USEFUL       // walk the candidate sections instead of the useful ones
#define ACS_AB_NO_USEFUL 0
#endif
#ifndef ACS_AB_NO_VERDICTS     // ignore the per-class target verdicts
#define ACS_AB_NO_VERDICTS 0
#endif
#ifndef ACS_AB_NO_PAD          // device sort: waves may mix classes (no wave-aligned class runs)
#define ACS_AB_NO_PAD 0
#endif
#ifndef ACS_AB_DEVICE_SORT     // ignore the encoder's coherence order (the device sorts, round-3 form)
#define ACS_AB_DEVICE_SORT 0
#endif

// Sort key that makes a wave share its request class (one candidate row) and action — or,
// with a role factor, its role key — so table-driven branches are wave-uniform:
// [bucket | low field].  Class ids come heaviest-first from the host (most candidate
// nodes), and unfiltered requests (PCOL_ALL) take bucket 0, so the longest waves start
// first and the launch has no long tail.  Unfiltered requests group by their first entity
// id.  The low field keeps `lowbits` bits (role keys are dense, so all of them; action and
// entity ids are folded mod 2^lowbits): fewer key bits, fewer radix passes.  A fold
// collision only merges two groups, which costs coherence, never correctness: results are
// written to out[perm[k]], so any permutation gives the same records.  With a role factor
// and B.role_major the fields swap ([role key | bucket], `cbits` bucket bits): a wave then
// spans few role keys, and the role rows prune rules hardest (large stores).
__device__ inline uint32_t sort_key(const Batch& B, uint32_t k, uint32_t lowbits, uint32_t cbits) {
  const ReqLine* ln = B.hdr ? nullptr : B.lines + k;  // compact batch: the line holds the rows read here
  const ReqHdr h = ln ? ln->h : B.hdr[k];
  const uint32_t cls = h.flags >> RQ_PCOL_SHIFT;
  // the action is read only when it is the low field (a 4-B read of a 128-B line still
  // moves a sector: with lowbits == 0 the key kernel reads the header alone)
  uint32_t low = 0, bucket = cls + 1;
  if (B.role_key) low = B.role_key[k] & 0xFFFFu;  // the first role row
  else if (lowbits && h.nact) low = ln ? ln->a0.value : B.act[k].value;
  if (cls >= B.cand_rows) {
    bucket = 0;
    const uint32_t* ex = ln && ln->ext ? B.ext + (size_t)(ln->ext - 1u) * 4u : nullptr;
    for (uint32_t j = 0; j < h.nres; ++j) {
      const ReqRes q = !ln ? B.res[(size_t)j * B.n + k]
                       : j < (uint32_t)LINE_RES ? ln->res[j] : *(const ReqRes*)(ex + 4u * (j - LINE_RES));
      if (q.kind & K_ENT) {
        low = q.value;
        break;
      }
    }
  }
  low &= (1u << lowbits) - 1u;
  return B.role_major ? (low << cbits) | bucket : (bucket << lowbits) | low;
}

// ---------------------------------------------------------------- LSD radix sort
// Keys of up to 32 bits, 8-bit digits, ceil(end_bit / 8) passes.  Each pass:
//   histogram  per 2048-key tile, counts[tile][digit] (written whole — no memset);
//   tile scan  per group of 64 tiles, one thread per digit: the exclusive prefix over the
//              group's tiles (in place) and the group total gsum[group][digit];
//   group scan one block: per digit, the exclusive prefix over groups, then the digit
//              bases (exclusive scan of the 256 digit totals) folded in;
//   scatter    stable: a tile is ranked 256 keys per round in index order; inside a wave,
//              lanes with equal digits are found with 8 ballots (one per digit bit) and
//              ranked by the popcount of the lower lanes; the waves' per-digit counts go
//              through LDS.  Position = gbase[group][d] + counts[tile][d] + rank.
// Pass 0's histogram is fused into the key kernel.
constexpr uint32_t SORT_ITEMS = 8;                    // keys per thread per tile
constexpr uint32_t SORT_TILE = BLOCK * SORT_ITEMS;    // 2048
constexpr uint32_t RADIX = 256;
constexpr uint32_t SCAN_GROUP = 64;                   // tiles per tile-scan group

__device__ inline void tile_histogram(uint32_t* hist, const uint32_t* keys_or_null, const Batch* B,
                                      uint32_t lowbits, uint32_t cbits, uint32_t* keys_out, uint32_t* idx_out, uint32_t n,
                                      uint32_t shift, uint32_t* counts) {
  hist[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t t0 = blockIdx.x * SORT_TILE;
  for (uint32_t r = 0; r < SORT_ITEMS; ++r) {
    const uint32_t i = t0 + r * BLOCK + threadIdx.x;
    if (i >= n) break;
    uint32_t key;
    if (B) {
      key = sort_key(*B, i, lowbits, cbits);
      keys_out[i] = key;
      idx_out[i] = i;
    } else {
      key = keys_or_null[i];
    }
    atomicAdd(&hist[(key >> shift) & (RADIX - 1)], 1u);
  }
  __syncthreads();
  counts[(size_t)blockIdx.x * RADIX + threadIdx.x] = hist[threadIdx.x];
}

__global__ __launch_bounds__(BLOCK) void sort_keys_kernel(Batch B, uint32_t lowbits, uint32_t cbits,
                                                          uint32_t* __restrict__ keys, uint32_t* __restrict__ idx,
                                                          uint32_t* __restrict__ counts) {
  __shared__ uint32_t hist[RADIX];
  tile_histogram(hist, nullptr, &B, lowbits, cbits, keys, idx, B.n, 0, counts);
}

__global__ __launch_bounds__(BLOCK) void radix_histogram_kernel(const uint32_t* __restrict__ keys, uint32_t n,
                                                                uint32_t shift, uint32_t* __restrict__ counts) {
  __shared__ uint32_t hist[RADIX];
  tile_histogram(hist, keys, nullptr, 0, 0, nullptr, nullptr, n, shift, counts);
}

__global__ __launch_bounds__(RADIX) void radix_tile_scan_kernel(uint32_t* __restrict__ counts, uint32_t nt,
                                                                uint32_t* __restrict__ gsum) {
  const uint32_t d = threadIdx.x, b0 = blockIdx.x * SCAN_GROUP;
  const uint32_t b1 = b0 + SCAN_GROUP < nt ? b0 + SCAN_GROUP : nt;
  uint32_t c[SCAN_GROUP];
#pragma unroll
  for (uint32_t k = 0; k < SCAN_GROUP; ++k) c[k] = b0 + k < b1 ? counts[(size_t)(b0 + k) * RADIX + d] : 0u;
  uint32_t run = 0;
#pragma unroll
  for (uint32_t k = 0; k < SCAN_GROUP; ++k) {
    if (b0 + k < b1) counts[(size_t)(b0 + k) * RADIX + d] = run;
    run += c[k];
  }
  gsum[(size_t)blockIdx.x * RADIX + d] = run;
}

__global__ __launch_bounds__(RADIX) void radix_group_scan_kernel(uint32_t* __restrict__ gsum, uint32_t ng) {
  __shared__ uint32_t tot[RADIX];
  const uint32_t d = threadIdx.x;
  uint32_t run = 0;
  for (uint32_t g = 0; g < ng; ++g) {
    const uint32_t v = gsum[(size_t)g * RADIX + d];
    gsum[(size_t)g * RADIX + d] = run;
    run += v;
  }
  tot[d] = run;
  __syncthreads();
  for (uint32_t off = 1; off < RADIX; off <<= 1) {  // inclusive scan of the digit totals
    const uint32_t v = d >= off ? tot[d - off] : 0u;
    __syncthreads();
    tot[d] += v;
    __syncthreads();
  }
  const uint32_t base = tot[d] - run;
  for (uint32_t g = 0; g < ng; ++g) gsum[(size_t)g * RADIX + d] += base;
}

__global__ __launch_bounds__(BLOCK) void radix_scatter_kernel(const uint32_t* __restrict__ kin,
                                                              const uint32_t* __restrict__ vin,
                                                              uint32_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                              const uint32_t* __restrict__ counts,
                                                              const uint32_t* __restrict__ gbase, uint32_t n,
                                                              uint32_t shift, uint32_t write_keys) {
  __shared__ uint32_t base[RADIX];
  __shared__ uint32_t wcnt[BLOCK / 64][RADIX];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  base[threadIdx.x] = counts[(size_t)blockIdx.x * RADIX + threadIdx.x] +
                      gbase[(size_t)(blockIdx.x / SCAN_GROUP) * RADIX + threadIdx.x];
  const uint32_t t0 = blockIdx.x * SORT_TILE;
  for (uint32_t r = 0; r < SORT_ITEMS; ++r) {
    if (t0 + r * BLOCK >= n) break;  // block-uniform
#pragma unroll
    for (uint32_t w = 0; w < BLOCK / 64; ++w) wcnt[w][threadIdx.x] = 0;
    __syncthreads();
    const uint32_t i = t0 + r * BLOCK + threadIdx.x;
    const bool valid = i < n;
    const uint32_t key = valid ? kin[i] : 0u, val = valid ? vin[i] : 0u;
    const uint32_t d = (key >> shift) & (RADIX - 1);
    uint64_t same = __ballot(valid);
#pragma unroll
    for (uint32_t bit = 0; bit < 8; ++bit) {
      const uint64_t bb = __ballot((d >> bit) & 1u);
      same &= ((d >> bit) & 1u) ? bb : ~bb;
    }
    const uint32_t rank = (uint32_t)__popcll(same & lt);
    if (valid && rank == 0) wcnt[wave][d] = (uint32_t)__popcll(same);
    __syncthreads();
    uint32_t pos = base[d] + rank;
    for (uint32_t w = 0; w < wave; ++w) pos += wcnt[w][d];
    __syncthreads();  // every lane has read base[] before it advances
    uint32_t tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < BLOCK / 64; ++w) tot += wcnt[w][threadIdx.x];
    base[threadIdx.x] += tot;
    if (valid) {
      vout[pos] = val;
      if (write_keys) kout[pos] = key;
    }
    __syncthreads();  // wcnt is cleared by the next round
  }
}

// ---------------------------------------------------------------- class counting sort
// The coherence sort only has to GROUP equal keys (any permutation gives the same records),
// and a batch's key space is small (c3: 31k classes), so when it has at most CS_BINS keys one
// counting pass replaces the radix passes:
//   count    block b takes a contiguous chunk (< 2^16 keys) of the batch: extracts each key
//            from the request line (written to keys[] for the scatter), counts it in LDS
//            (16-bit counters, two per word: 64k bins in 128 KB) and writes its count row
//            counts[b][0..K) whole (no memset);
//   columns  per bin: exclusive prefix over the blocks (in place) and the bin total;
//   bases    one block: exclusive scan of the K bin totals;
//   scatter  block b again: a key's LDS atomic returns its rank inside the block, and
//            perm[base[key] + counts[b][key] + rank] = i.  Ranks follow the LDS atomic order,
//            so equal keys are grouped but not kept in index order (not needed).
// Traffic: the line headers once, 4 B of key written and read back, K x blocks count words
// twice, 4 B of perm per request — against ~8 passes of 8-B keys + values for the radix sort.
constexpr uint32_t CS_BINS = 65536;
constexpr uint32_t CS_THREADS = 1024;
constexpr uint32_t CS_MAX_CHUNK = 65535;  // per-block counts fit 16 bits
constexpr uint32_t CS_ITEMS = 8;          // keys per thread per round

__device__ inline void cs_zero(uint32_t* h, uint32_t K) {
  for (uint32_t w = threadIdx.x; w < (K + 1) / 2; w += CS_THREADS) h[w] = 0;
  __syncthreads();
}

__global__ __launch_bounds__(CS_THREADS) void class_count_kernel(Batch B, uint32_t lowbits, uint32_t cbits,
                                                                 uint32_t chunk, uint32_t K,
                                                                 uint32_t* __restrict__ keys,
                                                                 uint32_t* __restrict__ counts) {
  __shared__ uint32_t h[CS_BINS / 2];
  cs_zero(h, K);
  const uint32_t i0 = blockIdx.x * chunk, i1 = i0 + chunk < B.n ? i0 + chunk : B.n;
  // CS_ITEMS keys per thread per round, their header reads all in flight before the atomics
  for (uint32_t r0 = i0; r0 < i1; r0 += CS_ITEMS * CS_THREADS) {
    uint32_t key[CS_ITEMS];
#pragma unroll
    for (uint32_t j = 0; j < CS_ITEMS; ++j) {
      const uint32_t i = r0 + j * CS_THREADS + threadIdx.x;
      key[j] = i < i1 ? sort_key(B, i, lowbits, cbits) : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < CS_ITEMS; ++j) {
      const uint32_t i = r0 + j * CS_THREADS + threadIdx.x;
      if (i < i1) {
        keys[i] = key[j];
        atomicAdd(&h[key[j] >> 1], 1u << ((key[j] & 1u) * 16u));
      }
    }
  }
  __syncthreads();
  uint32_t* row = counts + (size_t)blockIdx.x * K;
  for (uint32_t k = threadIdx.x; k < K; k += CS_THREADS) row[k] = (h[k >> 1] >> ((k & 1u) * 16u)) & 0xFFFFu;
}

__global__ __launch_bounds__(BLOCK) void class_columns_kernel(uint32_t* __restrict__ counts, uint32_t nb, uint32_t K,
                                                              uint32_t* __restrict__ tot) {
  const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
  if (k >= K) return;
  uint32_t run = 0;
  constexpr uint32_t G = 32;  // rows loaded per round, all in flight (a serial load per row is latency-bound)
  for (uint32_t b0 = 0; b0 < nb; b0 += G) {
    uint32_t c[G];
#pragma unroll
    for (uint32_t j = 0; j < G; ++j) c[j] = b0 + j < nb ? counts[(size_t)(b0 + j) * K + k] : 0u;
#pragma unroll
    for (uint32_t j = 0; j < G; ++j) {
      if (b0 + j < nb) counts[(size_t)(b0 + j) * K + k] = run;
      run += c[j];
    }
  }
  tot[k] = run;
}

// pad: each key's run starts on a wave boundary (runs rounded up to 64 lanes; the holes stay
// 0xFFFFFFFF), so no wave mixes keys (whatIsAllowed, where a wave walks the union of its
// lanes' candidates).
__global__ __launch_bounds__(CS_THREADS) void class_bases_kernel(uint32_t* __restrict__ tot, uint32_t K, uint32_t pad) {
  __shared__ uint32_t part[CS_THREADS];
  constexpr uint32_t PER_MAX = CS_BINS / CS_THREADS;  // 64: this thread's bins, loaded at once
  const uint32_t per = (K + CS_THREADS - 1) / CS_THREADS, k0 = threadIdx.x * per;
  uint32_t v[PER_MAX];
  uint32_t s = 0;
#pragma unroll
  for (uint32_t j = 0; j < PER_MAX; ++j) {
    v[j] = j < per && k0 + j < K ? tot[k0 + j] : 0u;
    if (pad) v[j] = (v[j] + 63u) & ~63u;
    s += v[j];
  }
  part[threadIdx.x] = s;
  __syncthreads();
  for (uint32_t off = 1; off < CS_THREADS; off <<= 1) {  // inclusive scan of the thread sums
    const uint32_t v = threadIdx.x >= off ? part[threadIdx.x - off] : 0u;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint32_t run = part[threadIdx.x] - s;
#pragma unroll
  for (uint32_t j = 0; j < PER_MAX; ++j) {
    if (j < per && k0 + j < K) tot[k0 + j] = run;
    run += v[j];
  }
}

__global__ __launch_bounds__(CS_THREADS) void class_scatter_kernel(const uint32_t* __restrict__ keys, uint32_t n,
                                                                   uint32_t chunk, uint32_t K,
                                                                   const uint32_t* __restrict__ counts,
                                                                   const uint32_t* __restrict__ base,
                                                                   uint32_t* __restrict__ perm) {
  __shared__ uint32_t h[CS_BINS / 2];
  cs_zero(h, K);
  const uint32_t i0 = blockIdx.x * chunk, i1 = i0 + chunk < n ? i0 + chunk : n;
  const uint32_t* row = counts + (size_t)blockIdx.x * K;
  for (uint32_t r0 = i0; r0 < i1; r0 += CS_ITEMS * CS_THREADS) {
    uint32_t key[CS_ITEMS], at[CS_ITEMS];
#pragma unroll
    for (uint32_t j = 0; j < CS_ITEMS; ++j) {
      const uint32_t i = r0 + j * CS_THREADS + threadIdx.x;
      key[j] = i < i1 ? keys[i] : 0u;
    }
#pragma unroll
    for (uint32_t j = 0; j < CS_ITEMS; ++j) at[j] = base[key[j]] + row[key[j]];  // all in flight
#pragma unroll
    for (uint32_t j = 0; j < CS_ITEMS; ++j) {
      const uint32_t i = r0 + j * CS_THREADS + threadIdx.x;
      if (i < i1) {
        const uint32_t sh = (key[j] & 1u) * 16u;
        const uint32_t rank = (atomicAdd(&h[key[j] >> 1], 1u << sh) >> sh) & 0xFFFFu;
        perm[at[j] + rank] = i;
      }
    }
  }
}

// Dynamic LDS per wave: one W-word union row when W <= LDS_FILTER_WORDS (the FilterLds
// form); for longer rows (large stores) a B.lds_pref-word union prefix — the set and policy
// sections, at most LDS_FILTER_WORDS — while rule words come from the lanes' own rows.
constexpr uint32_t LDS_FILTER_WORDS = 1024;
// OR the second class rows of the wave's composed lanes (ReqLine.cls2 = c2, 1 + class) into
// its LDS row, words [0, LW); *any: the wave holds a composed lane.  False when one names a row
// outside the batch (the wave then runs unfiltered).
// lds[w] |= row[w] for w = lane, lane + 64, ... < LW.  (Rejected A/B, r05_x: eight loads in flight
// per lane before the ORs — c3 10M K1 3.08 vs 2.93 ms, c3 131,072 0.387 vs 0.368.)
__device__ inline void lds_or_row(uint32_t* lds, const uint32_t* __restrict__ row, uint32_t LW, uint32_t lane) {
  for (uint32_t w = lane; w < LW; w += 64u) lds[w] |= row[w];
}

// the same with the row AND-ed with a role-factor row (or the OR of two)
__device__ inline void lds_or_row_roles(uint32_t* lds, const uint32_t* __restrict__ row, const uint32_t* q1,
                                        const uint32_t* q2, uint32_t LW, uint32_t lane) {
  for (uint32_t w = lane; w < LW; w += 64u) lds[w] |= row[w] & role_word(q1, q2, w);
}

__device__ inline bool or_second_rows(const Batch& B, bool valid, uint32_t c2, uint32_t* lds, uint32_t LW, bool* any) {
  const uint32_t lane = threadIdx.x & 63u, W = B.cand_words;
  uint64_t pending = __ballot(valid && c2 != 0u);
  *any = pending != 0;
  while (pending) {
    const int leader = __builtin_ctzll(pending);
    const uint32_t k = __builtin_amdgcn_readlane(c2, leader);
    if (k - 1u >= B.cand_rows) return false;
    const uint32_t* row = B.cand + (size_t)(k - 1u) * W;
    lds_or_row(lds, row, LW, lane);
    ACS_SCAN(LW * 4u);
    ACS_OPC(OP_ROWS2);
    pending &= ~__ballot(valid && c2 == k);
  }
  return true;
}

constexpr uint32_t NO_ROLE_KEY = 0xFFFFFFFFu;  // a lane without role filtering (wave_filter keys)

// Candidate filter of a wave, built with every lane present before any lane diverges.  A
// request's row is its class row (OR its second class row: composed rows), AND-ed with its
// role-factor row when the batch has one.  The LDS part is the OR of the rows of all the
// wave's active requests over the first lds_n words, however many (class, role key) pairs the
// wave spans; Filter::word ORs the active lanes' own rows past it.  An unfiltered request
// (PCOL_ALL) disables filtering for its wave.
__device__ inline Filter wave_filter(const Batch& B, bool valid, uint32_t cls, uint32_t rk, uint32_t c2, uint32_t* lds) {
  Filter F{};
  F.wp = B.cand_wp;
  F.wr = B.cand_wr;
  F.wsu = B.cand_wsu;
  F.wpu = B.cand_wpu ? B.cand_wpu : B.cand_wp;
  F.wv = B.cand_wv;
  F.vok = false;  // waves mix classes: the general form keeps no per-class verdicts
  F.all = B.cand == nullptr;
  F.lds = lds;
  const uint32_t lane = threadIdx.x & 63u, W = B.cand_words;
  const uint32_t LW = W <= LDS_FILTER_WORDS ? W : B.lds_pref;
  F.lds_n = LW;
  // this lane's own rows (any valid row for a lane that evaluates nothing)
  const bool own = valid && cls < B.cand_rows;
  F.row = B.cand ? B.cand + (size_t)(own ? cls : 0u) * W : nullptr;
  F.row2 = own && c2 && c2 - 1u < B.cand_rows ? B.cand + (size_t)(c2 - 1u) * W : nullptr;
  const uint32_t *r1, *r2;
  role_rows_of(B, rk, &r1, &r2);
  F.rrow = own ? r1 : nullptr;
  F.rrow2 = own ? r2 : nullptr;
  if (F.all) return F;
  for (uint32_t w = lane; w < LW; w += 64) lds[w] = 0u;
  const uint32_t rkey = r1 ? rk : NO_ROLE_KEY;
  uint64_t pending = __ballot(valid);
  if (!pending) F.all = true;  // no active lane: nothing is evaluated anyway
  while (pending) {  // once per distinct (class, role key) of the wave
    const int leader = __builtin_ctzll(pending);
    const uint32_t c = __builtin_amdgcn_readlane(cls, leader), r = __builtin_amdgcn_readlane(rkey, leader);
    if (c == PCOL_ALL || c >= B.cand_rows) {
      F.all = true;
      break;
    }
    const uint32_t* row = B.cand + (size_t)c * W;
    const uint32_t *q1 = nullptr, *q2 = nullptr;
    if (r != NO_ROLE_KEY) role_rows_of(B, r, &q1, &q2);
    if (q1)
      lds_or_row_roles(lds, row, q1, q2, LW, lane);
    else
      lds_or_row(lds, row, LW, lane);
    ACS_SCAN(LW * (q1 ? (q2 ? 12u : 8u) : 4u));
    pending &= ~__ballot(valid && cls == c && rkey == r);
  }
  bool any2;
  if (!F.all && !or_second_rows(B, valid, c2, lds, LW, &any2)) F.all = true;
  return F;
}

// The LDS form (FilterLds): the wave's OR row over its (class & role) rows in this wave's
// W-word LDS region, all ones when the wave holds an unfiltered request.
__device__ inline FilterLds wave_filter_lds(const Batch& B, bool valid, uint32_t cls, uint32_t rk, uint32_t c2,
                                            uint32_t* lds) {
  FilterLds F{lds, B.cand_wp, B.cand_wr, B.cand_wsu, B.cand_wpu ? B.cand_wpu : B.cand_wp, B.cand_wv, nullptr, nullptr,
              false, false};
  const uint32_t lane = threadIdx.x & 63u, W = B.cand_words;
  const uint32_t *r1, *r2;
  role_rows_of(B, rk, &r1, &r2);
  const uint32_t rkey = r1 ? rk : NO_ROLE_KEY;
  bool all = false, any2 = false;
  uint32_t first_cls = PCOL_ALL, classes = 0;
  for (uint32_t w = lane; w < W; w += 64) lds[w] = 0u;
  uint64_t pending = __ballot(valid);
  while (pending) {  // once per distinct (class, role key) of the wave
    const int leader = __builtin_ctzll(pending);
    const uint32_t c = __builtin_amdgcn_readlane(cls, leader), r = __builtin_amdgcn_readlane(rkey, leader);
    if (c == PCOL_ALL || c >= B.cand_rows) {
      all = true;
      break;
    }
    const uint32_t* row = B.cand + (size_t)c * W;
    const uint32_t *q1 = nullptr, *q2 = nullptr;
    if (r != NO_ROLE_KEY) role_rows_of(B, r, &q1, &q2);
    if (q1)
      lds_or_row_roles(lds, row, q1, q2, W, lane);
    else
      lds_or_row(lds, row, W, lane);
    ACS_SCAN(W * (q1 ? (q2 ? 12u : 8u) : 4u));
    ACS_OPC(OP_ROWS);
    if (c != first_cls) {
      first_cls = c;
      ++classes;
    }
    pending &= ~__ballot(valid && cls == c && rkey == r);
  }
  // a wave of one class keeps that class's verdict sections in LDS: second rows are OR-ed into
  // the candidate sections only
  if (!all && !or_second_rows(B, valid, c2, lds, classes == 1 ? B.cand_wv : W, &any2)) all = true;
  if (all)
    for (uint32_t w = lane; w < W; w += 64) lds[w] = ~0u;
  // the verdicts are the class's (role keys may differ: role rows keep the verdict sections
  // whole): a wave of one class reads them from LDS — a composed lane composing them with its
  // second row's — any other lane from its own class row(s) (the LDS form is only chosen for
  // batches that carry verdict sections)
  F.single = !all && classes == 1 && !B.no_verdicts;
  const bool c2ok = c2 == 0u || c2 - 1u < B.cand_rows;
  F.own = valid && cls < B.cand_rows && c2ok && !B.no_verdicts ? B.cand + (size_t)cls * W : nullptr;
  F.own2 = F.own && c2 ? B.cand + (size_t)(c2 - 1u) * W : nullptr;
  F.ownc = F.own != nullptr && B.role_key == nullptr;
  return F;
}

__device__ inline FilterAll wave_filter_all(const Batch& B) {
  return FilterAll{B.cand_wp, B.cand_wr, B.cand_wsu, B.cand_wpu ? B.cand_wpu : B.cand_wp};
}

// One maker per filter form, selected by the kernel's template argument.
template <class FL> struct FilterMaker;
template <> struct FilterMaker<Filter> {
  static __device__ Filter make(const Batch& B, bool valid, uint32_t cls, uint32_t rk, uint32_t c2, uint32_t* lds) {
    return wave_filter(B, valid, cls, rk, c2, lds);
  }
};
template <> struct FilterMaker<FilterLds> {
  static __device__ FilterLds make(const Batch& B, bool valid, uint32_t cls, uint32_t rk, uint32_t c2, uint32_t* lds) {
    return wave_filter_lds(B, valid, cls, rk, c2, lds);
  }
};
template <> struct FilterMaker<FilterAll> {
  static __device__ FilterAll make(const Batch& B, bool, uint32_t, uint32_t, uint32_t, uint32_t*) {
    return wave_filter_all(B);
  }
};

extern __shared__ uint32_t acs_dyn_lds[];

__host__ __device__ inline uint32_t lds_wave_words(const Batch& B) {
  return B.cand_words <= LDS_FILTER_WORDS ? B.cand_words : B.lds_pref;
}

__device__ inline uint32_t* wave_lds_row(const Batch& B) {
  if (!B.cand) return nullptr;
  return acs_dyn_lds + (threadIdx.x >> 6) * lds_wave_words(B);
}

__device__ inline uint32_t request_pcol(const ReqHdr& h) {
  return (h.flags & RQ_NO_TARGET) ? PCOL_ALL : (h.flags >> RQ_PCOL_SHIFT);
}

#if defined(ACS_WAVE_TIMES)
// Diagnostic build only: per-wave first-start / last-end wall clock of K1 / K2 and the smallest
// class of the wave's lanes (tools/wave_times.py, tools/wave_times_k1.py).  Every lane folds its own times in (vector atomics).
constexpr uint32_t WT_MAX = 1u << 16;
__device__ unsigned long long acs_wt0[WT_MAX], acs_wt1[WT_MAX];
__device__ unsigned int acs_wt_cls[WT_MAX], acs_wt_lanes[WT_MAX];
#endif
#if defined(ACS_PHASE_PROF)
__device__ unsigned long long acs_phase_acc[PH_N];
#endif

// A lane's first NS resource attributes into its LDS column (stride BLOCK): the line's, then
// past the line the extension record's (compact batches) or the SoA rows.
template <int NS, bool CB>
__device__ inline void stage_attrs(ReqRes* col, const Batch& B, const ReqLine* ln, uint32_t i, uint32_t nres) {
  const uint32_t nq = nres < (uint32_t)LINE_RES ? nres : (uint32_t)LINE_RES;
  for (uint32_t j = 0; j < nq; ++j) col[j * BLOCK] = ln ? ln->res[j] : B.res[(size_t)j * B.n + i];
  for (uint32_t j = LINE_RES; j < nres && j < (uint32_t)NS; ++j) {
    if (ln && CB) {
      ReqRes q;
      __builtin_memcpy(&q, B.ext + (size_t)(ln->ext - 1u) * 4u + 4u * (j - LINE_RES), sizeof q);
      col[j * BLOCK] = q;
    } else {
      col[j * BLOCK] = B.res[(size_t)j * B.n + i];
    }
  }
}

#ifndef ACS_AB_PROBE_K1_NOWALK
#define ACS_AB_PROBE_K1_NOWALK 0
#endif
#ifndef ACS_AB_PROBE_K1_NOROWS
#define ACS_AB_PROBE_K1_NOROWS 0
#endif
// K1 stages the line's 4 attributes (LDS_SLOTS).  (Rejected A/B, r06_p: a fifth slot for the first
// extension attribute, which leaves 4 blocks per CU — c3 10M 3.34 ms at 5 waves/SIMD with spills,
// 3.19 at 4 without, vs 2.95; c3adv, already at 4 waves, 1.639 vs 1.646.)

// K1: one request per lane; its resource attributes are staged in this lane's LDS column.
#ifndef ACS_K1_WAVES_PER_EU
// 5 waves/SIMD (VGPR <= 96, with 4 LDS attribute slots so 5 blocks fit a CU's LDS): c3 K1
// 1.98 -> 1.87 ms in a same-call A/B (r02_q; c2 0.180 -> 0.190 ms), 4 slots alone 1.95 ms
#define ACS_K1_WAVES_PER_EU 5
#endif
// CB: a compact batch (request lines + extension records, no SoA rows): the kernels are
// instantiated for it separately so that its row accessors carry no SoA paths (fewer live
// registers; acs_eval.h ReqCtx::soa; A/B c3 K1 1.94 -> 1.85 ms, r03_g).
template <bool CB>
__device__ inline const ReqLine* lane_line(const Batch& B, bool in, uint32_t i) {
  return CB ? B.lines + i : (in && B.lines ? B.lines + i : nullptr);  // one gather for the first rows
}


// 1 + the lane's second class (composed class rows; 0: none)
__device__ inline uint32_t lane_cls2(const ReqLine* ln, bool in) { return in && ln ? ln->cls2 : 0u; }

// AN: the batch holds ACL_NONE requests (acs_req_batch.hints): instantiate the skips for them
// (acs_eval.h is_allowed_t; they cost c3's plain batches registers: K1 3.12 -> 3.44 ms, r04_n).
// With the ACL_NONE skips K1 runs at 4 waves/SIMD (no VGPR spills; same-call A/B c3adv 1.98 ->
// 1.90 ms, while the plain c3 K1 is faster at 5: 3.11 vs 3.23 ms, r04_o).
#ifndef ACS_K1_AN_WAVES_PER_EU
#define ACS_K1_AN_WAVES_PER_EU 4
#endif
// SK: the lanes skip the sets, policies and rules outside their own class rows (acs_eval.h
// is_allowed_t) — the instantiation for batches whose waves mix classes: spread small batches and
// batches without wave-aligned class runs (c3 131,072 requests: K1 0.670 -> 0.578 ms with 32
// lanes per wave, r05_e; c3 524,288 unpadded 0.905 -> 0.790; c5 1M 8.64 -> 3.05 ms, r05_i).
// Batches of long class runs keep the plain form (c3 1M padded: 0.770 vs 0.789 ms, r05_i; c3 10M
// unpadded, ~300 requests per class: 3.02 vs 3.10 ms, r05_j)
#ifndef ACS_K1_SK_WAVES_PER_EU
// c3 131,072: 0.448 ms at 5, 0.437 at 4 with 16-request spread waves (r05_g); with 8-request waves
// 0.359 at 5 vs 0.375 at 4, c3 524,288 0.592 vs 0.595, c5 1M 3.150 vs 3.178 (r05_af)
#define ACS_K1_SK_WAVES_PER_EU 5
#endif
template <class FL, bool CB, bool AN, bool SK = false>
__global__ __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(
    AN ? ACS_K1_AN_WAVES_PER_EU : (SK ? ACS_K1_SK_WAVES_PER_EU : ACS_K1_WAVES_PER_EU)))) void is_allowed_kernel(
    Tables T, Batch B, const uint32_t* __restrict__ perm, uint32_t lanes, Decision* __restrict__ out) {
  __shared__ ReqRes stage[LDS_SLOTS * BLOCK];
  const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
  const uint32_t pk = k < lanes ? (perm ? perm[k] : k) : 0xFFFFFFFFu;  // padded perm: holes
  const bool in = pk < B.n;
  const uint32_t i = in ? pk : 0u;
  const ReqLine* ln = lane_line<CB>(B, in, i);
  ReqHdr h{};
  if (in) h = ln ? ln->h : B.hdr[i];
  bool done = true;
  Decision d{};
  if (in) d = early_decision(h, &done);
#if defined(ACS_WAVE_TIMES)
  const uint32_t wt = k >> 6;
  if (wt < WT_MAX) {
    atomicMin(&acs_wt0[wt], (unsigned long long)wall_clock64());
    if (in) {
      atomicAdd(&acs_wt_lanes[wt], 1u);
      atomicMin(&acs_wt_cls[wt], request_pcol(h));
    }
  }
#endif
#if ACS_AB_PROBE_K1_NOROWS  // timing probe: no filter rows, no walk (the prologue's line and attribute reads)
  if (in) out[i] = d;
  return;
#endif
  const FL F = FilterMaker<FL>::make(B, in && !done, request_pcol(h), B.role_key && in ? B.role_key[i] : 0xFFFFu,
                                     lane_cls2(ln, in), wave_lds_row(B));
#if ACS_AB_PROBE_K1_NOWALK  // timing probe: the prologue without the walk
  if (in) out[i] = d;
  (void)F;
  return;
#endif
#if defined(ACS_PHASE_PROF)
  uint64_t prof_lane[PH_N] = {};
  if (!in) done = true;
#else
  if (!in) return;
#endif
  if (!done) {
    ReqRes* col = stage + threadIdx.x;
    stage_attrs<LDS_SLOTS, CB>(col, B, ln, i, h.nres);
#if defined(ACS_PHASE_PROF)
    const ReqLds<> R(T, B, i, h, col, BLOCK, ln, !CB);
    d = is_allowed_t<AN, SK>(R, F);
    for (int k = 0; k < PH_N; ++k) prof_lane[k] = R.prof[k];
#else
    d = is_allowed_t<AN, SK>(ReqLds<>(T, B, i, h, col, BLOCK, ln, !CB), F);
#endif
  }
#if !defined(ACS_PHASE_PROF)
  out[i] = d;
#if defined(ACS_WAVE_TIMES)
  if (wt < WT_MAX) atomicMax(&acs_wt1[wt], (unsigned long long)wall_clock64());
#endif
#else
  if (in) out[i] = d;
  for (int k = 0; k < PH_N; ++k) {  // lane-cycles per phase, one atomic per wave
    uint64_t v = prof_lane[k];
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    if ((threadIdx.x & 63u) == 0) atomicAdd(&acs_phase_acc[k], (unsigned long long)v);
  }
#endif
}

// whatIsAllowed templates (acs_eval.h wia_template_set): one wave per class row of the batch; its
// lanes take the row's candidate sets in turn (sets are independent in whatIsAllowed), OR their
// bits into the wave's record in LDS, and the wave writes the record.  A set that makes the class
// untemplated clears the record's flags (the class's requests take the full walk).
struct LdsAcc {
  uint32_t* rec;
  __device__ void or_bits(uint32_t w, uint32_t bit) { atomicOr(rec + w, bit); }
};
// LDS writes of this wave's lanes visible to its other lanes (waves that share no LDS)
__device__ inline void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

// Every class row of the batch gets a template.  (Rejected A/B, r05_i: a request-count gate, rows
// of fewer than 32 / 128 requests untemplated — c4 1M K2 8.75 vs 4.01 ms: most waves then hold a
// lane whose class went untemplated and pay the full walk besides.)
__global__ __launch_bounds__(BLOCK) void wia_template_kernel(Tables T, Batch B, TplLayout TL, BitsLayout BL,
                                                             uint32_t* __restrict__ out) {
  const uint32_t wave = threadIdx.x >> 6, lane = threadIdx.x & 63u;
  const uint32_t c = blockIdx.x * (BLOCK / 64) + wave;
  if (c >= B.cand_rows) return;  // the waves share no LDS: they sync alone (wave_sync)
  uint32_t* rec = acs_dyn_lds + wave * TL.stride;
  for (uint32_t w = lane; w < TL.stride; w += 64) rec[w] = 0u;
  wave_sync();
  bool ok = true, role_free = true;
  {
    // rounds of 64 candidate sets, all lanes at once: in round r lane j takes the row's set of
    // rank 64 r + j.  The wave-uniform cursor (w, before) walks the row's words; a word that also
    // holds ranks of the next round is read again then.  (Set by set, one lane active, the pass
    // cost 5.0 ms at c4's 1M requests, r05_g.)
    const uint32_t* row = B.cand + (size_t)c * B.cand_words;
    const uint32_t nw = (T.n_sets + 31u) / 32u;
    LdsAcc acc{rec};
    uint32_t w = 0, before = 0;  // words consumed, candidate sets in them
    for (uint32_t r0 = 0;; r0 += 64u) {
      const uint32_t want = r0 + lane;
      uint32_t set = 0xFFFFFFFFu;
      for (; w < nw; ++w) {
        uint32_t x = row[w];
        // bits past n_sets in the last word are not sets (a caller's row may carry them): dropped
        if (w == nw - 1u && (T.n_sets & 31u)) x &= (1u << (T.n_sets & 31u)) - 1u;
        const uint32_t pc = (uint32_t)__builtin_popcount(x);
        if (want >= before && want < before + pc) {
          for (uint32_t q = want - before; q; --q) x &= x - 1u;
          set = 32u * w + (uint32_t)__builtin_ctz(x);
        }
        if (before + pc > r0 + 63u) break;  // the word holds next-round ranks too
        before += pc;
      }
      if (!__ballot(set != 0xFFFFFFFFu)) break;
      if (set != 0xFFFFFFFFu)
        ok = wia_template_set(T, row, B.cand_wp, B.cand_wr, B.cand_wv, BL, TL, set, acc, &role_free);
      if (__ballot(!ok)) break;  // the class is untemplated
    }
  }
  const bool all_ok = __ballot(!ok) == 0, all_free = __ballot(!role_free) == 0;
  wave_sync();
  const uint32_t ww = TL.exact - TL.work;
  for (uint32_t w = lane; w < ww; w += 64)
    if (rec[TL.work + w]) atomicOr(rec + TL.mask + (w >> 5), 1u << (w & 31u));
  wave_sync();
  uint32_t* dst = out + (size_t)c * TL.stride;
  for (uint32_t w = lane; w < TL.stride; w += 64) {
    uint32_t v = all_ok ? rec[w] : 0u;
    if (w == TL.flags) v = all_ok ? (TPL_OK | (all_free ? TPL_ROLE_FREE : 0u)) : 0u;
    dst[w] = v;
  }
}

// A templated lane's work-rule bits over the row the wave already wrote from the template(s):
// as TplSink, each section's current 16-B chunk gathers bits in registers, but only a chunk that
// got some is rewritten (template chunk(s) | bits); the lane is its row's only writer by then.
// (Device atomics per bit measured slower: c4 1M K2 4.71 vs 4.05 ms, r05_n; a word at a time,
// without the template read, too: 3.16 vs 2.22 ms, 4M 9.78 vs 6.10, r06_s.)
struct SparseTplSink {
  uint4* row;
  const uint4* t1;
  const uint4* t2;
  uint32_t cur[3];
  uint4 buf[3];
  uint32_t wm[3] = {0u, 0u, 0u};  // the chunks written (bit q of chunk q; rows of at most 96 chunks)
  __device__ SparseTplSink(uint32_t* r, const BitsLayout& L, const uint32_t* a, const uint32_t* b)
      : row(reinterpret_cast<uint4*>(r)), t1(reinterpret_cast<const uint4*>(a)), t2(reinterpret_cast<const uint4*>(b)) {
    cur[0] = 0;
    cur[1] = L.wp >> 2;
    cur[2] = L.wr >> 2;
    for (int k = 0; k < 3; ++k) buf[k] = make_uint4(0u, 0u, 0u, 0u);
  }
  template <int S> __device__ void flush() {
    const uint4 b = buf[S];
    if (!(b.x | b.y | b.z | b.w)) return;
    uint4 v = t1[cur[S]];
    if (t2) {
      const uint4 u = t2[cur[S]];
      v.x |= u.x; v.y |= u.y; v.z |= u.z; v.w |= u.w;
    }
    v.x |= b.x; v.y |= b.y; v.z |= b.z; v.w |= b.w;
    row[cur[S]] = v;
    const uint32_t c = cur[S], bit = 1u << (c & 31u);
    wm[0] |= c < 32u ? bit : 0u;
    wm[1] |= c >= 32u && c < 64u ? bit : 0u;
    wm[2] |= c >= 64u && c < 96u ? bit : 0u;
    buf[S] = make_uint4(0u, 0u, 0u, 0u);
  }
  template <int S> __device__ void set(uint32_t w, uint32_t bit) {
    const uint32_t c = w >> 2, q = w & 3u;
    if (c != cur[S]) {
      flush<S>();
      cur[S] = c;
    }
    buf[S].x |= q == 0u ? bit : 0u;
    buf[S].y |= q == 1u ? bit : 0u;
    buf[S].z |= q == 2u ? bit : 0u;
    buf[S].w |= q == 3u ? bit : 0u;
  }
  __device__ void finish() {
    flush<0>();
    flush<1>();
    flush<2>();
  }
};
// K2's work rules with their rule lines staged in LDS (what_is_allowed_tpl's walk and results).
// A work rule's target match is a chain of dependent reads — the rule record, then its action
// pairs and resource attributes (inline in the record's 128-B line), then its policy and set —
// and a wave meets ~12 of them one after the other.  Here the wave first lists its work rules in
// walk order (the union over its lanes), then loads up to `cap` rule lines and their (policy, set)
// at once into its LDS region (the filter-row region, free until a full walk), all active lanes
// sharing the 16-B pieces, and evaluates the listed rules from LDS.  Region layout (u32 words):
// [cap lines of 32 | cap (policy, set) | cap rule ids]; needs device rule lines (rstride 2).
constexpr uint32_t STAGE_WORDS_PER_RULE = 32u + 2u + 1u;
// (The unstaged walk, what_is_allowed_tpl, serves images without rule lines and regions too small
// to stage a rule: c4 1M 2.722 vs 2.523 ms staged, r06_l.)
template <class RQ, class SINK>
__device__ bool what_is_allowed_tpl_staged(const RQ& R, const TplLayout& TL, const BitsLayout& BL, const uint32_t* t1,
                                           const uint32_t* t2, SINK& sink, OblLog& obl, uint32_t* lds, uint32_t cap) {
  const Tables& T = R.T;
  uint32_t* lines = lds;
  uint32_t* ps = lds + 32u * cap;
  uint32_t* ids = ps + 2u * cap;
  const uint64_t act = __ballot(1);
  const uint32_t nact = (uint32_t)__builtin_popcountll(act);
  const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0u));
  bool ok = true;
  uint32_t n = 0, have = 0;  // listed rules (wave-uniform); this lane's among them (bit e)
  auto flush = [&]() {
    wave_sync();  // the listed ids
    for (uint32_t q = rank; q < 8u * n; q += nact) {
      const uint32_t r = ids[q >> 3];
      reinterpret_cast<uint4*>(lines)[q] =
          reinterpret_cast<const uint4*>(T.rules + (size_t)r * T.rstride)[q & 7u];
    }
    for (uint32_t e = rank; e < n; e += nact) {
      const uint32_t p = T.parents[ids[e] + T.n_pols];
      ps[2u * e] = p;
      ps[2u * e + 1u] = T.parents[p];
    }
    ACS_SCAN(n * 136u);
    wave_sync();
    for (uint32_t e = 0; e < n; ++e) {
      if (!ok || !((have >> e) & 1u)) continue;
      ACS_OPC(OP_TPL_TM);
      const uint32_t* L = lines + 32u * e;
      const NodeRec Q = load_words(T, reinterpret_cast<const NodeRec*>(L));
      const uint32_t r = wave_uniform(ids[e]);
      // inline attributes (acs_compile's rule lines): offsets that point into the rule's own line
      const RuleResAttr* ra =
          Q.res_off == r * 8u + 4u ? reinterpret_cast<const RuleResAttr*>(L + 16) : T.rres + Q.res_off;
      const Pair* ap = Q.act_off == r * 16u + 14u ? reinterpret_cast<const Pair*>(L + 28) : T.pairs + Q.act_off;
      const tri m = target_match_retry_at(Q, T.pairs + Q.subj_off, ap, ra, R, Q.effect, true, &obl);
      if (m < 0) {
        ok = false;
        continue;
      }
      if (m) {
        ACS_OPC(OP_TPL_HIT);
        const uint32_t p = ps[2u * e], s = ps[2u * e + 1u];
        sink.template set<0>(s >> 5, 1u << (s & 31u));
        sink.template set<1>(BL.wp + (p >> 5), 1u << (p & 31u));
        sink.template set<2>(BL.wr + (r >> 5), 1u << (r & 31u));
      }
    }
    wave_sync();  // the next batch overwrites the lines
    n = 0;
    have = 0;
  };
  const uint32_t MW = (TL.flags - TL.mask);
  ACS_OPC(OP_TPL_REQ);
  for (uint32_t k = 0; k < MW; ++k) {
    uint32_t u = wave_or(t1[TL.mask + k] | (t2 ? t2[TL.mask + k] : 0u));
    while (u) {
      const uint32_t w = wave_uniform(32u * k + (uint32_t)__builtin_ctz(u));
      u &= u - 1u;
      ACS_OPC(OP_TPL_WORD);
      uint32_t mine = t1[TL.work + w] & ~(t2 ? t2[BL.wr + w] : 0u);
      if (t2) mine |= t2[TL.work + w] & ~t1[BL.wr + w];
      uint32_t rest = wave_or(mine);
      while (rest) {
        const uint32_t b = (uint32_t)__builtin_ctz(rest);
        rest &= rest - 1u;
        ACS_OPC(OP_TPL_RULE);
        if (n == cap) flush();
        ids[n] = 32u * w + b;  // every active lane writes the same id
        have |= ((mine >> b) & 1u) << n;
        ++n;
      }
    }
  }
  if (n) flush();
  if (!ok) return false;
  sink.finish();
  return true;
}

// Order of one wave's stores to the same row chunk (the wave's template copy, then a lane's own
// rewrite of that chunk): the earlier stores complete before the later issue.  Workgroup scope is
// a wait for the wave's outstanding stores.  (Rejected, r06_k: agent scope, the round-5 form, also
// writes the XCD's L2 back to memory at every wave — c4 1M K2 3.445 vs 2.705 ms.)
__device__ inline void k2_store_order() { __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup"); }
// Timing probes (K2 results differ): no template copy / no work rules
#ifndef ACS_AB_PROBE_K2_NOCOPY
#define ACS_AB_PROBE_K2_NOCOPY 0
#endif
#ifndef ACS_AB_PROBE_K2_NOWORK
#define ACS_AB_PROBE_K2_NOWORK 0
#endif
// K2's LDS attribute slots: the line's 4, then the first extension attribute (c4: a quarter of the
// requests carry 5 resource attributes; every work rule's match reads all of them)
#ifndef ACS_K2_SLOTS
#define ACS_K2_SLOTS 5
#endif
#ifndef ACS_K2_WORK_FIRST
#define ACS_K2_WORK_FIRST 1  // 0: the copy first, then the rewrites (A/B)
#endif
constexpr int K2_SLOTS = ACS_K2_SLOTS;
// K2: whatIsAllowed inclusion bitset + maskedProperty log, one request per lane (perm
// order k).  Lane k writes request perm[k]'s BitsLayout row of the [n][words] output itself,
// once, 16 B per store (ChunkSink): no scratch buffer, no zeroing pass, no transpose.
// K2 occupancy A/B (5/6/8 waves per SIMD: 96/80/64 VGPRs with spills) measured no gain on c4
// (6.92-6.95 ms vs 6.62, r03_g; 3.97 / 4.00 vs 4.03, r05_final): the compiler's own 4 waves/SIMD stay.
template <class FL, bool CB>
__global__ __launch_bounds__(BLOCK) void what_is_allowed_kernel(Tables T, Batch B, const uint32_t* __restrict__ perm,
                                                                uint32_t lanes, BitsLayout BL,
                                                                uint32_t* __restrict__ bits,
                                                                uint32_t* __restrict__ obl,
                                                                uint32_t* __restrict__ obl_n,
                                                                Decision* __restrict__ out,
                                                                const uint32_t* __restrict__ tpl, TplLayout TL) {
  __shared__ ReqRes stage[K2_SLOTS * BLOCK];
  const uint32_t k = blockIdx.x * BLOCK + threadIdx.x;
  const uint32_t pk = k < lanes ? (perm ? perm[k] : k) : 0xFFFFFFFFu;  // padded perm: holes
  const bool in = pk < B.n;
  const uint32_t i = in ? pk : 0u;
  const ReqLine* ln = lane_line<CB>(B, in, i);
  ReqHdr h{};
  if (in) h = ln ? ln->h : B.hdr[i];
  const bool host = (h.flags & RQ_HOST) != 0;
#if defined(ACS_WAVE_TIMES)
  const uint32_t wt = k >> 6;
  if (wt < WT_MAX) {
    atomicMin(&acs_wt0[wt], (unsigned long long)wall_clock64());
    if (in) {
      atomicAdd(&acs_wt_lanes[wt], 1u);
      atomicMin(&acs_wt_cls[wt], request_pcol(h));
    }
  }
#endif
  // Every lane stays to the end: the wave filter (the full walk's) is built, with all lanes
  // present, only when some lane still needs the full walk after the template phase.
  const uint32_t o = i;
  Decision d{};
  bool done = !in;
  if (in && host) {
    ChunkSink sink(bits + (size_t)o * BL.words, BL);
    d.flags = OF_HOST_REQ;
    sink.finish();
    obl_n[o] = 0u;
    done = true;
  }
  ReqRes* scol = stage + threadIdx.x;
  if (!done) stage_attrs<K2_SLOTS, CB>(scol, B, ln, i, h.nres);
  if (tpl) {  // the class template(s) plus the work rules (acs_eval.h what_is_allowed_tpl)
    const uint32_t c1 = request_pcol(h), c2 = lane_cls2(ln, in);
    const uint32_t* t1 = !done && c1 < B.cand_rows ? tpl + (size_t)c1 * TL.stride : nullptr;
    const uint32_t* t2 = t1 && c2 && c2 - 1u < B.cand_rows ? tpl + (size_t)(c2 - 1u) * TL.stride : nullptr;
    const uint32_t* r1 = t1 ? B.cand + (size_t)c1 * B.cand_words : nullptr;
    const uint32_t* r2 = t2 ? B.cand + (size_t)(c2 - 1u) * B.cand_words : nullptr;
    const bool usable = t1 && !(c2 && !t2) && tpl_usable(TL, t1, t2, r1, r2, T.n_sets, h.flags);
    // The wave writes its templated lanes' rows one after the other, 16 B per lane per store
    // (1 KB contiguous per store instead of 64 lanes' 16-B pieces of 64 rows), then each lane
    // rewrites the chunks of its own row that its work rules add bits to.  (Rejected A/B, r06_g:
    // the template chunks held in registers and re-read only when the (class, second class) pair
    // changes — c4 1M K2 3.975 vs 4.007 ms, 131,072 1.751 vs 1.727: within the noise; the wave's rows
    // as one flat run of chunks, four steps' loads in flight — 2.290 vs 2.298 ms, 4M 6.27 vs 6.37,
    // r06_u: the copy is bound by its 1.4 GB of writes, not by the loads' latency.)
    const uint32_t q4 = BL.words >> 2, lane = threadIdx.x & 63u;
    // Rows of at most 96 chunks (c4: 89): the lanes' work rules first, each writing the chunks its
    // bits fall in (template | bits) and noting them, then the wave copies the template into the
    // other chunks only — every chunk written once, no store ordering between lanes.  Longer rows:
    // the copy first, then the rewrites after a store-order fence.
    const bool work_first = ACS_K2_WORK_FIRST && q4 <= 96u;
    uint32_t wm0 = 0, wm1 = 0, wm2 = 0;
    bool tpl_ok = false;
    for (uint64_t m = ACS_AB_PROBE_K2_NOCOPY || work_first ? 0u : __ballot(usable); m; m &= m - 1u) {
      const int j = __builtin_ctzll(m);
      const uint32_t oj = (uint32_t)__shfl((int)o, j), c1j = (uint32_t)__shfl((int)c1, j),
                     c2j = (uint32_t)__shfl((int)(t2 ? c2 : 0u), j);
      uint4* dst = reinterpret_cast<uint4*>(bits + (size_t)oj * BL.words);
      const uint4* s1 = reinterpret_cast<const uint4*>(tpl + (size_t)c1j * TL.stride);
      const uint4* s2 = c2j ? reinterpret_cast<const uint4*>(tpl + (size_t)(c2j - 1u) * TL.stride) : nullptr;
      ACS_SCAN(16u * q4 * (s2 ? 2u : 1u));  // the template row(s); the row write is B_out
      for (uint32_t q = lane; q < q4; q += 64u) {
        uint4 v = s1[q];
        if (s2) {
          const uint4 u = s2[q];
          v.x |= u.x; v.y |= u.y; v.z |= u.z; v.w |= u.w;
        }
        dst[q] = v;
      }
    }
    if (!work_first) k2_store_order();  // the copy's stores land before the lanes' own
    if (usable && ACS_AB_PROBE_K2_NOWORK) {  // timing probe: no work rules (rows lack their bits)
      obl_n[o] = 0u;
      done = tpl_ok = true;
    } else if (usable) {
      SparseTplSink sink(bits + (size_t)o * BL.words, BL, t1, t2);
      OblLog log{obl + (size_t)o * 2 * OBL_MAX, 0, false};
      const ReqLds<K2_SLOTS> R(T, B, i, h, scol, BLOCK, ln, !CB);
      const uint32_t cap = T.rstride == 2u ? min(32u, lds_wave_words(B) / STAGE_WORDS_PER_RULE) : 0u;
      if (cap ? what_is_allowed_tpl_staged(R, TL, BL, t1, t2, sink, log, wave_lds_row(B), cap)
              : what_is_allowed_tpl(R, TL, BL, t1, t2, sink, log)) {
        if (log.overflow) d.flags |= OF_OBL_OVERFLOW;
        obl_n[o] = log.n;
        done = tpl_ok = true;
        wm0 = sink.wm[0];
        wm1 = sink.wm[1];
        wm2 = sink.wm[2];
      }
    }
    // work first: the template into the chunks of each templated row that its lane did not write (a
    // lane whose template walk failed takes the full walk, which writes its whole row)
    for (uint64_t m = work_first && !ACS_AB_PROBE_K2_NOCOPY ? __ballot(tpl_ok) : 0u; m; m &= m - 1u) {
      const int j = __builtin_ctzll(m);
      const uint32_t oj = (uint32_t)__shfl((int)o, j), c1j = (uint32_t)__shfl((int)c1, j),
                     c2j = (uint32_t)__shfl((int)(t2 ? c2 : 0u), j);
      const uint32_t k0 = __builtin_amdgcn_readlane(wm0, j), k1 = __builtin_amdgcn_readlane(wm1, j),
                     k2 = __builtin_amdgcn_readlane(wm2, j);
      uint4* dst = reinterpret_cast<uint4*>(bits + (size_t)oj * BL.words);
      const uint4* s1 = reinterpret_cast<const uint4*>(tpl + (size_t)c1j * TL.stride);
      const uint4* s2 = c2j ? reinterpret_cast<const uint4*>(tpl + (size_t)(c2j - 1u) * TL.stride) : nullptr;
      ACS_SCAN(16u * q4 * (s2 ? 2u : 1u));
      for (uint32_t q = lane; q < q4; q += 64u) {
        const uint32_t km = q < 32u ? k0 : q < 64u ? k1 : k2;
        if ((km >> (q & 31u)) & 1u) continue;
        uint4 v = s1[q];
        if (s2) {
          const uint4 u = s2[q];
          v.x |= u.x; v.y |= u.y; v.z |= u.z; v.w |= u.w;
        }
        dst[q] = v;
      }
    }
  }
  if (__ballot(!done)) {  // the full walk (rewrites a failed template lane's whole row)
    if (tpl) k2_store_order();  // a failed lane's chunks land first
    const FL F = FilterMaker<FL>::make(B, !done, request_pcol(h), B.role_key && in ? B.role_key[i] : 0xFFFFu,
                                       lane_cls2(ln, in && !done), wave_lds_row(B));
    if (!done) {
      ChunkSink sink(bits + (size_t)o * BL.words, BL);
      OblLog log{obl + (size_t)o * 2 * OBL_MAX, 0, false};
      d = what_is_allowed_t(ReqLds<K2_SLOTS>(T, B, i, h, scol, BLOCK, ln, !CB), F, BL, sink, log);
      sink.finish();
      obl_n[o] = (d.flags & OF_ERR) ? 0u : log.n;
    }
  }
  if (!in) return;
  out[o] = d;
#if defined(ACS_WAVE_TIMES)
  if (wt < WT_MAX) atomicMax(&acs_wt1[wt], (unsigned long long)wall_clock64());
#endif
}

// Global set index g as an index of an image holding sets [base, base + n), clipped to [0, n].
__device__ inline uint32_t obl_range_local(uint32_t g, uint32_t base, uint32_t n) {
  return g <= base ? 0u : (g - base < n ? g - base : n);
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
template <class FL, bool CB>
__global__ __launch_bounds__(BLOCK) void what_is_allowed_obl_kernel(Tables T, Batch B, const uint32_t* __restrict__ idx,
                                                                    uint32_t m, uint32_t chunks, uint32_t cap,
                                                                    uint32_t* __restrict__ obl,
                                                                    uint32_t* __restrict__ obl_n, uint32_t g_sets,
                                                                    uint32_t set_base) {
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
  const ReqLine* ln = lane_line<CB>(B, in, i);
  ReqHdr h{};
  if (in) h = ln ? ln->h : B.hdr[i];
  const bool host = (h.flags & RQ_HOST) != 0;
  const FL F = FilterMaker<FL>::make(B, in && !host, request_pcol(h), B.role_key && in ? B.role_key[i] : 0xFFFFu,
                                     lane_cls2(ln, in), wave_lds_row(B));
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
    for (uint32_t q = 0; q < nq; ++q) scol[q * BLOCK] = ln ? ln->res[q] : B.res[(size_t)q * B.n + i];
    // range c of the whole store's sets (g_sets; a rule-sharded handle's image holds the sets
    // [set_base, + n_sets) of it), clipped to this image's sets
    const uint32_t s0 = obl_range_local((uint32_t)((uint64_t)g_sets * c / chunks), set_base, T.n_sets);
    const uint32_t s1 = obl_range_local((uint32_t)((uint64_t)g_sets * (c + 1) / chunks), set_base, T.n_sets);
    NullSink none;
    const Decision d = what_is_allowed_t(ReqLds<>(T, B, i, h, scol, BLOCK, ln, !CB), F, BitsLayout{}, none, log, s0, s1);
    total = (d.flags & OF_ERR) ? 0u : log.total;
  }
  obl_n[k] = total;
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

// Rule-sharded handles: the batch's class rows cut to this shard's nodes (acs_eval.h
// RowSlice), one thread per output word.
__global__ __launch_bounds__(BLOCK) void slice_rows_kernel(const uint32_t* __restrict__ src, uint32_t src_words,
                                                           uint32_t rows, RowSlice L, uint32_t* __restrict__ dst) {
  const size_t k = (size_t)blockIdx.x * BLOCK + threadIdx.x;
  if (k >= (size_t)rows * L.words) return;
  const uint32_t r = (uint32_t)(k / L.words), w = (uint32_t)(k % L.words);
  dst[k] = slice_word(src + (size_t)r * src_words, src_words, L, w);
}

// keys[i] = max(keys[i], other[i]): the MAX reduction of the shards' decision keys.
__global__ __launch_bounds__(BLOCK) void max_keys_kernel(uint64_t* __restrict__ keys, const uint64_t* __restrict__ other,
                                                         uint32_t n) {
  const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
  if (i < n && other[i] > keys[i]) keys[i] = other[i];
}

// ---------------------------------------------------------------- dense obligation logs
// The host-buffer whatIsAllowed downloads each request's maskedProperty log only up to its
// length (obl_n entries of 8 B) instead of the whole OBL_MAX-entry slot: the logs are packed on
// the device, request by request in index order, and the host places them into the caller's
// [n][OBL_MAX][2] slots (c4: 16.4 entries per request on average against 128).
// blk_tot[b] = entries of requests [b * BLOCK, (b + 1) * BLOCK)
__global__ __launch_bounds__(BLOCK) void obl_block_sums_kernel(const uint32_t* __restrict__ obl_n, uint32_t n,
                                                               uint32_t* __restrict__ blk_tot) {
  __shared__ uint32_t ws[BLOCK / 64];
  const uint32_t i = blockIdx.x * BLOCK + threadIdx.x;
  uint32_t c = i < n ? min(obl_n[i], (uint32_t)OBL_MAX) : 0u;
  for (int o = 32; o > 0; o >>= 1) c += (uint32_t)__shfl_xor((int)c, o);
  if ((threadIdx.x & 63u) == 0) ws[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int w = 0; w < BLOCK / 64; ++w) t += ws[w];
    blk_tot[blockIdx.x] = t;
  }
}

// In place: blk[b] = entries before block b (exclusive scan, one block, 64-bit safe total in
// blk[nb] as two words: low, high)
__global__ __launch_bounds__(BLOCK) void obl_scan_blocks_kernel(uint32_t* __restrict__ blk, uint32_t nb) {
  __shared__ uint32_t ws[BLOCK / 64];
  __shared__ unsigned long long carry;
  if (threadIdx.x == 0) carry = 0ull;
  __syncthreads();
  for (uint32_t base = 0; base < nb; base += BLOCK) {
    const uint32_t b = base + threadIdx.x;
    const uint32_t v = b < nb ? blk[b] : 0u;
    uint32_t x = v;  // inclusive scan within the wave
    const uint32_t lane = threadIdx.x & 63u;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = (uint32_t)__shfl_up((int)x, o);
      if (lane >= (uint32_t)o) x += y;
    }
    if (lane == 63u) ws[threadIdx.x >> 6] = x;
    __syncthreads();
    uint32_t before = 0;
    for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) before += ws[w];
    const unsigned long long c0 = carry;
    if (b < nb) blk[b] = (uint32_t)(c0 + before + x - v);
    __syncthreads();
    if (threadIdx.x == BLOCK - 1) carry = c0 + before + x;
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    blk[nb] = (uint32_t)carry;
    blk[nb + 1] = (uint32_t)(carry >> 32);
  }
}

// dense[blk[b] + ...] = the logs of block b's requests in index order; each thread copies every
// BLOCK-th entry of the block's concatenated log (a binary search over the block's prefix in LDS
// finds its request), so the stores are contiguous
__global__ __launch_bounds__(BLOCK) void obl_pack_kernel(const uint2* __restrict__ obl, const uint32_t* __restrict__ obl_n,
                                                         uint32_t n, const uint32_t* __restrict__ blk,
                                                         uint2* __restrict__ dense) {
  __shared__ uint32_t pre[BLOCK + 1];
  __shared__ uint32_t ws[BLOCK / 64];
  const uint32_t i = blockIdx.x * BLOCK + threadIdx.x, lane = threadIdx.x & 63u;
  const uint32_t c = i < n ? min(obl_n[i], (uint32_t)OBL_MAX) : 0u;
  uint32_t x = c;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, o);
    if (lane >= (uint32_t)o) x += y;
  }
  if (lane == 63u) ws[threadIdx.x >> 6] = x;
  __syncthreads();
  uint32_t before = 0;
  for (uint32_t w = 0; w < (threadIdx.x >> 6); ++w) before += ws[w];
  pre[threadIdx.x + 1] = before + x;
  if (threadIdx.x == 0) pre[0] = 0u;
  __syncthreads();
  const uint32_t total = pre[BLOCK];
  const size_t base = blk[blockIdx.x];
  for (uint32_t e = threadIdx.x; e < total; e += BLOCK) {
    uint32_t lo = 0, hi = BLOCK;  // the request r with pre[r] <= e < pre[r + 1]
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (pre[mid] <= e) lo = mid; else hi = mid;
    }
    const size_t r = (size_t)blockIdx.x * BLOCK + lo;
    dense[base + e] = obl[r * OBL_MAX + (e - pre[lo])];
  }
}

// ---------------------------------------------------------------- stable selection
// The overflowed-log bookkeeping of the device path: the indices i < n a predicate selects,
// in index order (count per 2048-item tile -> one-block exclusive scan -> per-tile write,
// ranked with wave ballots: deterministic, no atomics), plus the largest value of the
// selected items.
struct FlaggedRecords {  // decision records carrying `mask`
  const Decision* d;
  uint32_t mask;
  __device__ bool sel(uint32_t i) const { return (d[i].flags & mask) != 0; }
  __device__ uint32_t val(uint32_t) const { return 0; }
};

struct PermEntries {  // the requests of a coherence order, holes (indices >= n) left out
  const uint32_t* perm;
  uint32_t n;
  __device__ bool sel(uint32_t k) const { return perm[k] < n; }
  __device__ uint32_t val(uint32_t) const { return 0; }
};

struct TruncatedLogs {  // a pass's obl_n [chunks][m]: some range pushed more than cap
  const uint32_t* obl_n;
  uint32_t m, chunks, cap;
  __device__ uint32_t val(uint32_t j) const {
    uint32_t v = 0;
    for (uint32_t c = 0; c < chunks; ++c) {
      const uint32_t x = obl_n[(size_t)c * m + j];
      v = x != 0xFFFFFFFFu && x > v ? x : v;  // 0xFFFFFFFF: an index outside the batch
    }
    return v;
  }
  __device__ bool sel(uint32_t j) const { return val(j) > cap; }
};

template <class P>
__global__ __launch_bounds__(BLOCK) void select_count_kernel(P p, uint32_t n, uint32_t* __restrict__ tile_cnt,
                                                             uint32_t* __restrict__ tile_max) {
  __shared__ uint32_t sc[BLOCK / 64], sm[BLOCK / 64];
  uint32_t c = 0, mx = 0;
  const uint32_t t0 = blockIdx.x * SORT_TILE;
  for (uint32_t r = 0; r < SORT_ITEMS; ++r) {
    const uint32_t i = t0 + r * BLOCK + threadIdx.x;
    if (i < n && p.sel(i)) {
      ++c;
      const uint32_t v = p.val(i);
      mx = v > mx ? v : mx;
    }
  }
  for (int off = 32; off > 0; off >>= 1) {
    c += __shfl_xor(c, off);
    const uint32_t o = __shfl_xor(mx, off);
    mx = o > mx ? o : mx;
  }
  if ((threadIdx.x & 63u) == 0) {
    sc[threadIdx.x >> 6] = c;
    sm[threadIdx.x >> 6] = mx;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tc = 0, tm = 0;
    for (uint32_t w = 0; w < BLOCK / 64; ++w) {
      tc += sc[w];
      tm = sm[w] > tm ? sm[w] : tm;
    }
    tile_cnt[blockIdx.x] = tc;
    tile_max[blockIdx.x] = tm;
  }
}

// one block: tile_cnt -> exclusive offsets (in place); total[0] = selected, total[1] = max
__global__ __launch_bounds__(BLOCK) void select_scan_kernel(uint32_t* __restrict__ tile_cnt,
                                                            const uint32_t* __restrict__ tile_max, uint32_t nt,
                                                            uint32_t* __restrict__ total) {
  __shared__ uint32_t sv[BLOCK];
  uint32_t carry = 0, mx = 0;
  for (uint32_t b0 = 0; b0 < nt; b0 += BLOCK) {
    const uint32_t k = b0 + threadIdx.x;
    const uint32_t v = k < nt ? tile_cnt[k] : 0u;
    if (k < nt) mx = tile_max[k] > mx ? tile_max[k] : mx;
    sv[threadIdx.x] = v;
    __syncthreads();
    for (uint32_t off = 1; off < BLOCK; off <<= 1) {
      const uint32_t x = threadIdx.x >= off ? sv[threadIdx.x - off] : 0u;
      __syncthreads();
      sv[threadIdx.x] += x;
      __syncthreads();
    }
    if (k < nt) tile_cnt[k] = carry + sv[threadIdx.x] - v;
    carry += sv[BLOCK - 1];
    __syncthreads();
  }
  sv[threadIdx.x] = mx;
  __syncthreads();
  for (uint32_t off = BLOCK / 2; off > 0; off >>= 1) {
    if (threadIdx.x < off && sv[threadIdx.x + off] > sv[threadIdx.x]) sv[threadIdx.x] = sv[threadIdx.x + off];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    total[0] = carry;
    total[1] = sv[0];
  }
}

// out[offset + rank] = map ? map[i] : i for the selected i, in index order
template <class P>
__global__ __launch_bounds__(BLOCK) void select_write_kernel(P p, uint32_t n, const uint32_t* __restrict__ tile_off,
                                                             const uint32_t* __restrict__ map,
                                                             uint32_t* __restrict__ out) {
  __shared__ uint32_t wc[BLOCK / 64];
  const uint32_t lane = threadIdx.x & 63u, wave = threadIdx.x >> 6;
  uint32_t base = tile_off[blockIdx.x];
  const uint32_t t0 = blockIdx.x * SORT_TILE;
  for (uint32_t r = 0; r < SORT_ITEMS; ++r) {
    if (t0 + r * BLOCK >= n) break;  // block-uniform
    const uint32_t i = t0 + r * BLOCK + threadIdx.x;
    const bool s = i < n && p.sel(i);
    const uint64_t bal = __ballot(s);
    if (lane == 0) wc[wave] = (uint32_t)__popcll(bal);
    __syncthreads();
    uint32_t pos = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull)), tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < BLOCK / 64; ++w) {
      pos += w < wave ? wc[w] : 0u;
      tot += wc[w];
    }
    if (s) out[pos] = map ? map[i] : i;
    base += tot;
    __syncthreads();  // wc is rewritten by the next round
  }
}

// keys of the selected requests for the coherence order (sort_key), values = their indices
__global__ __launch_bounds__(BLOCK) void gather_sort_keys_kernel(Batch B, const uint32_t* __restrict__ idx, uint32_t m,
                                                                 uint32_t lowbits, uint32_t cbits,
                                                                 uint32_t* __restrict__ keys,
                                                                 uint32_t* __restrict__ vals) {
  const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
  if (j >= m) return;
  const uint32_t i = idx[j];
  keys[j] = sort_key(B, i, lowbits, cbits);
  vals[j] = i;
}

size_t align16(size_t x) { return (x + 15) & ~size_t(15); }

size_t filter_lds_bytes(const Batch& B) {
  if (!B.cand) return 0;
  return (size_t)(BLOCK / 64) * lds_wave_words(B) * 4;
}

// Which filter form a batch's kernels are instantiated with.
enum class FilterForm { All, Lds, General };
FilterForm filter_form(const Batch& B) {
  if (!B.cand) return FilterForm::All;
  return B.cand_words <= LDS_FILTER_WORDS && B.cand_wv ? FilterForm::Lds : FilterForm::General;
}

// one instantiation per filter form and batch form (compact: no SoA rows); X: further template
// arguments (ACS_TARGS_NONE, or K1's ACS_TARGS_ACL_NONE / ACS_TARGS_ACL_PLAIN)
#define ACS_TARGS_NONE
#define ACS_TARGS_ACL_NONE , true
#define ACS_TARGS_ACL_PLAIN , false
#define ACS_TARGS_ACL_PLAIN_SK , false, true
#define ACS_LAUNCH_FILTERED(kernel, ...) ACS_LAUNCH_FILTERED_X(kernel, ACS_TARGS_NONE, __VA_ARGS__)
#define ACS_LAUNCH_FILTERED_X(kernel, X, grid, lds, stream, form, compact, ...)                           \
  do {                                                                                                  \
    if (compact) {                                                                                      \
      switch (form) {                                                                                   \
        case FilterForm::All: hipLaunchKernelGGL((kernel<FilterAll, true X>), grid, dim3(BLOCK), lds, stream, __VA_ARGS__); break; \
        case FilterForm::Lds: hipLaunchKernelGGL((kernel<FilterLds, true X>), grid, dim3(BLOCK), lds, stream, __VA_ARGS__); break; \
        default: hipLaunchKernelGGL((kernel<Filter, true X>), grid, dim3(BLOCK), lds, stream, __VA_ARGS__); break;                \
      }                                                                                                 \
    } else {                                                                                            \
      switch (form) {                                                                                   \
        case FilterForm::All: hipLaunchKernelGGL((kernel<FilterAll, false X>), grid, dim3(BLOCK), lds, stream, __VA_ARGS__); break; \
        case FilterForm::Lds: hipLaunchKernelGGL((kernel<FilterLds, false X>), grid, dim3(BLOCK), lds, stream, __VA_ARGS__); break; \
        default: hipLaunchKernelGGL((kernel<Filter, false X>), grid, dim3(BLOCK), lds, stream, __VA_ARGS__); break;                \
      }                                                                                                 \
    }                                                                                                   \
  } while (0)

}  // namespace

namespace {
// Grow-only device allocation: a steady state of equal-sized batches allocates nothing.
struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
  int reserve(size_t n) {
    if (n <= bytes) return 0;
    if (p) HIP_OK(hipFree(p));
    p = nullptr;
    bytes = 0;
    const size_t want = n + n / 8;  // headroom: batches of slightly varying size reuse it
    HIP_OK(hipMalloc(&p, want));
    bytes = want;
    return 0;
  }
  void release() {
    if (p) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
};
// The device memory one evaluation needs beyond the tables: the coherence sort's keys /
// permutation, the uploaded request image and the outputs.
struct Workspace {
  DevBuf sort, img, out;
  DevBuf slice, keys;  // rule-sharded handles: the shard's class rows, decision keys
  DevBuf tpl;          // whatIsAllowed templates of the batch's class rows
  DevBuf spread;       // a small batch's order spread over more waves (spread_waves)
  DevBuf nopad;        // whatIsAllowed: the encoder's order with its holes left out (drop_holes)
  void release() {
    tpl.release();
    spread.release();
    nopad.release();
    sort.release();
    img.release();
    out.release();
    slice.release();
    keys.release();
  }
};
}  // namespace

struct acs_tables {
  int device = 0;
  void* dev = nullptr;  // one allocation holding every section
  Tables view{};
  hipStream_t stream = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  float last_ms = -1.f;
  int sort = 1;         // coherence sort of each batch (ACS_OPT_SORT)
  size_t chunk = 262144;  // host-buffer calls: requests per overlapped chunk (ACS_OPT_CHUNK; 0: off)
  uint32_t simds = 0;   // the device's SIMDs (spread_waves; 0 until first asked)
  // the device image as uploaded (acs_compile_update diffs against it): uninitialised storage,
  // 2-MB pages for a large store (every byte is written by compile_image)
  struct HostImage {
    struct Free {
      void operator()(char* q) const { free(q); }
    };
    std::unique_ptr<char, Free> p;
    size_t n = 0;
    bool alloc(size_t k) {
      const size_t huge = size_t(2) << 20;
      void* q = nullptr;
      if (k >= huge) {
        q = aligned_alloc(huge, (k + huge - 1) / huge * huge);
        if (q) madvise(q, (k + huge - 1) / huge * huge, MADV_HUGEPAGE);
      }
      if (!q) q = malloc(k ? k : 1);
      p.reset((char*)q);
      n = q ? k : 0;
      return q != nullptr;
    }
    char* data() { return p.get(); }
    const char* data() const { return p.get(); }
    size_t size() const { return n; }
  } host_img;
  size_t upload_bytes = 0;     // bytes the compile uploaded (acs_compile_update: the differing blocks)
  // acs_compile_update: the 64-KB blocks that differ from prev's image (delta_ok: the image is a
  // copy of prev's with those blocks replaced; else uploaded whole) — replicas apply the same delta
  static constexpr size_t DELTA_BLOCK = 64 * 1024;
  bool delta_ok = false;
  std::vector<uint32_t> delta_blocks;
  // ACS_OPT_TIMING: HIP events recorded on the launch stream around every eval kernel
  static constexpr int RING = 256;
  int timing = 0;
  hipEvent_t tev[2 * RING] = {};
  uint64_t launches = 0;
  // *_device entry points: the coherence sort's workspace (one stream at a time)
  Workspace dws;
  // host-buffer entry points (internal stream, events, their own workspace) may be called
  // from several host threads at once (e.g. the N-API addon's libuv pool): one at a time
  Workspace hws;
  Workspace ows;  // acs_overflow_*_device: selection scratch (.out) and the sort (.sort)
  // host-buffer calls cut into chunks (chunk_run): a workspace and a stream per pipeline slot
  static constexpr int CHUNK_SLOTS = 2;
  Workspace cws[CHUNK_SLOTS];
  hipStream_t cstream[CHUNK_SLOTS] = {};
  // page-locked host staging of the packed obligation logs, and of the chunks' coherence orders
  // (chunk_run), both grow-only
  void* hstage = nullptr;
  size_t hstage_bytes = 0;
  uint32_t* hperm = nullptr;
  size_t hperm_n = 0;
  std::mutex mu;
  uint32_t rx_rows_min = 0;  // regex-matrix rows the rule resource attributes read
  // acs_compile_multi: replicas of the same image on further devices (C0); the host-buffer
  // entry points split a compact batch across this handle and its replicas
  std::vector<acs_tables*> peers;
  size_t image_bytes = 0;
  // acs_compile_sharded: this image holds policy sets [base.set_base, + view.n_sets) of a store
  // of g_* sets / policies / rules; the peers hold the following runs (rule sharding, C1)
  int sharded = 0;
  ShardBase base{};
  uint32_t g_sets = 0, g_pols = 0, g_rules = 0;
};

// The entry points a rule-sharded handle does not serve (records need the cross-shard reduction)
static int refuse_sharded(const acs_tables* t, const char* fn) {
  if (!t || !t->sharded) return 0;
  g_err = std::string(fn) + ": a rule-sharded handle (acs_compile_sharded) serves the host-buffer entry points only "
          "(acs_is_allowed, acs_what_is_allowed, acs_what_is_allowed_obl)";
  return -1;
}

// csrc/acs_validate.cpp
extern "C" int acs_internal_check_blob(const void* blob, size_t n_bytes, uint32_t* rx_rows_min);
extern "C" int acs_internal_check_batch(const acs_req_batch* b, uint32_t n_sets, uint32_t n_pols, uint32_t n_rules,
                                        uint32_t rx_rows_min);
extern "C" void acs_internal_shard_plan(const acs_req_batch* b, size_t lo, size_t hi, const uint32_t* arena_end,
                                        size_t plan[4]);
extern "C" int acs_internal_check_batch2(const acs_req_batch* b, uint32_t n_sets, uint32_t n_pols, uint32_t n_rules,
                                         uint32_t rx_rows_min, uint32_t* arena_end);
extern "C" int acs_internal_check_acl_none(const acs_req_batch* b, uint32_t id_user);

static int check_batch(const acs_tables* t, const acs_req_batch* b) {
  return acs_internal_check_batch(b, t->view.n_sets, t->view.n_pols, t->view.n_rules, t->rx_rows_min) ||
         acs_internal_check_acl_none(b, t->view.id_user);
}

extern "C" {

const char* acs_last_error(void) { return g_err.c_str(); }

// The codec (acs_codec.cpp) reports through the same thread-local message.
void acs_internal_set_error(const char* msg) { g_err = msg ? msg : ""; }

#if defined(ACS_OP_COUNT)
// Operation-counting build only (tools/op_count.py): read and reset the per-operation wave and
// lane counts (acs_eval.h OpCount); out[0..n) waves, out[n..2n) lanes.
int acs_op_read(unsigned long long* out, int n) {
  if (n > (int)OP_N) n = OP_N;
  std::vector<unsigned long long> z(OP_N, 0);
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpyFromSymbol(out, HIP_SYMBOL(acs_op_wave), n * sizeof *out));
  HIP_OK(hipMemcpyFromSymbol(out + n, HIP_SYMBOL(acs_op_lane), n * sizeof *out));
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(acs_op_wave), z.data(), OP_N * sizeof z[0]));
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(acs_op_lane), z.data(), OP_N * sizeof z[0]));
  return 0;
}
#endif

#if defined(ACS_SCAN_COUNT)
// Counting build only: read and reset the table bytes the waves read (bench.py B_scan).
int acs_scan_read(unsigned long long* out) {
  unsigned long long z = 0;
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpyFromSymbol(out, HIP_SYMBOL(acs_scan_bytes), sizeof *out));
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(acs_scan_bytes), &z, sizeof z));
  return 0;
}
#endif

#if defined(ACS_WAVE_TIMES)
// Diagnostic build only: copy out the per-wave K2 records of the last launch(es) (ticks of the
// 100 MHz wall clock) and reset them; returns the capacity.
int acs_wave_times_read(unsigned long long* t0, unsigned long long* t1, unsigned int* cls, unsigned int* lanes,
                        int n) {
  static std::vector<unsigned long long> a(WT_MAX), b(WT_MAX);
  static std::vector<unsigned int> c(WT_MAX), l(WT_MAX);
  HIP_OK(hipDeviceSynchronize());
  HIP_OK(hipMemcpyFromSymbol(a.data(), HIP_SYMBOL(acs_wt0), WT_MAX * 8));
  HIP_OK(hipMemcpyFromSymbol(b.data(), HIP_SYMBOL(acs_wt1), WT_MAX * 8));
  HIP_OK(hipMemcpyFromSymbol(c.data(), HIP_SYMBOL(acs_wt_cls), WT_MAX * 4));
  HIP_OK(hipMemcpyFromSymbol(l.data(), HIP_SYMBOL(acs_wt_lanes), WT_MAX * 4));
  for (int k = 0; k < n && k < (int)WT_MAX; ++k) {
    t0[k] = a[k]; t1[k] = b[k]; cls[k] = c[k]; lanes[k] = l[k];
  }
  std::vector<unsigned long long> hi(WT_MAX, ~0ull), lo(WT_MAX, 0ull);
  std::vector<unsigned int> hc(WT_MAX, ~0u), lz(WT_MAX, 0u);
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(acs_wt0), hi.data(), WT_MAX * 8));
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(acs_wt1), lo.data(), WT_MAX * 8));
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(acs_wt_cls), hc.data(), WT_MAX * 4));
  HIP_OK(hipMemcpyToSymbol(HIP_SYMBOL(acs_wt_lanes), lz.data(), WT_MAX * 4));
  return (int)WT_MAX;
}
#endif

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

// Host memory for the codec's batch arrays (acs_codec.cpp HostPool): page-locked and portable
// (every device can DMA from it) when a device is present, so acs_is_allowed's per-section
// copies run at full PCIe speed; plain malloc on a machine without one.
void* acs_internal_host_alloc(size_t bytes, int* pinned) {
  static const bool have = [] {
    int n = 0;
    return hipGetDeviceCount(&n) == hipSuccess && n > 0;
  }();
  void* p = nullptr;
  if (have && hipHostMalloc(&p, bytes, hipHostMallocPortable) == hipSuccess) {
    *pinned = 1;
    return p;
  }
  *pinned = 0;
  return malloc(bytes);
}

void acs_internal_host_free(void* p, int pinned) {
  if (!p) return;
  if (pinned) (void)hipHostFree(p);
  else free(p);
}

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

}  // extern "C"
static acs_tables* compile_image(const void* blob, size_t n_bytes, int device, const acs_tables* prev);
static acs_tables* make_replica(const acs_tables* t, int device, const acs_tables* prev);
static acs_tables* compile_sharded(const void* blob, size_t n_bytes, const int* devices, int n_devices,
                                   const acs_tables* prev);
extern "C" {

acs_tables* acs_compile(const void* blob, size_t n_bytes, int device) {
  return compile_image(blob, n_bytes, device, nullptr);
}

// A new handle for a changed store (the delta upload): the image is laid out
// as acs_compile lays it out; when it has the previous handle's size (same node and pool counts:
// an updateRule / updatePolicy that keeps the shape), the new device image is a device-side copy
// of the previous one with only the 64-KB blocks that differ uploaded.  The previous handle stays
// valid (in-flight batches keep it).
acs_tables* acs_compile_update(const acs_tables* prev, const void* blob, size_t n_bytes) {
  if (!prev) {
    fail("acs_compile_update: null previous handle");
    return nullptr;
  }
  if (prev->sharded) {  // every shard against its previous image (the store's new cut)
    std::vector<int> dev{prev->device};
    for (const acs_tables* p : prev->peers) dev.push_back(p->device);
    return compile_sharded(blob, n_bytes, dev.data(), (int)dev.size(), prev);
  }
  acs_tables* t = compile_image(blob, n_bytes, prev->device, prev);
  if (!t) return nullptr;
  t->sort = prev->sort;
  t->chunk = prev->chunk;
  for (const acs_tables* p : prev->peers) {  // replicas: each its previous image + the primary's delta
    acs_tables* r = make_replica(t, p->device, p);
    if (!r) {
      acs_free(t);
      return nullptr;
    }
    t->peers.push_back(r);
  }
  (void)hipSetDevice(t->device);
  return t;
}

// host-to-device bytes of the compile (every shard of a rule-sharded handle; replicas copy
// device to device)
size_t acs_image_upload_bytes(const acs_tables* t) {
  if (!t) return 0;
  size_t b = t->upload_bytes;
  if (t->sharded)
    for (const acs_tables* p : t->peers) b += p->upload_bytes;
  return b;
}

}  // extern "C"

static acs_tables* compile_image(const void* blob, size_t n_bytes, int device, const acs_tables* prev) {
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
  uint32_t rx_rows_min = 0;
  if (acs_internal_check_blob(blob, n_bytes, &rx_rows_min)) return nullptr;
  // Device image: the blob's sections, except that each rule becomes a 128-B line (its 64-B
  // record, then up to 3 resource attributes and 2 action pairs inline), so a rule visit's
  // record, action and resource reads hit one cache line instead of three (large stores miss
  // L2 on each).  The rres and pair pools follow the lines, and one base (the first line)
  // addresses both: every node's res_off / act_off / subj_off is rebased, inline attributes
  // point into their line (pools too large for rebased u32 offsets keep the blob layout).
  const char* bsrc = (const char*)blob + src;
  size_t doff[6];
  uint32_t rstride = 1;
  size_t up_bytes = total;
  const size_t lines = (size_t)h.n_rules * 128;
  const size_t l0 = (align16(sz[0]) + align16(sz[1]) + 127) & ~size_t(127);
  const size_t p_rel = lines + align16(sz[3]);  // pair pool, bytes past the first line
  if (h.n_rules && (p_rel / 8 + h.n_pairs) < 0xFFFFFFFFull && (lines / 16 + h.n_rres) < 0xFFFFFFFFull) {
    rstride = 2;
    doff[0] = 0;
    doff[1] = align16(sz[0]);
    doff[2] = l0;
    doff[3] = l0 + lines;
    doff[4] = l0 + p_rel;
    doff[5] = doff[4] + align16(sz[4]);
    up_bytes = doff[5] + align16(sz[5]);
  } else {
    for (int k = 0; k < 6; ++k) doff[k] = off[k];
  }
  // the event index (acs_eval.h build_event_index) after the image, from the blob's records
  // and the parent index (acs_eval.h build_parents: whatIsAllowed templates) after it
  const size_t ev_words = event_index_words(h.n_sets, h.n_pols, h.n_rules);
  const size_t ex_words = ev_words + parent_index_words(h.n_pols, h.n_rules);
  const size_t ev_off = align16(up_bytes);
  const size_t img_total = ev_off + ex_words * sizeof(uint32_t);
  auto* t = new acs_tables();
  t->device = device;
  t->rx_rows_min = rx_rows_min;
  // The host image (kept: acs_compile_update diffs the next image against it), written in
  // place over the host threads — c5 (1M rules, 130 MB): one pass instead of a zero-fill, a
  // staging copy and a second copy.
  if (!t->host_img.alloc(img_total)) {
    fail("acs_compile: host image allocation failed");
    delete t;
    return nullptr;
  }
  char* d = t->host_img.data();
  const size_t T = std::max<size_t>(1, std::min<size_t>(16, std::thread::hardware_concurrency()));
  // copy [from, from + len) of the blob to d + to in pieces over the pool
  struct Piece {
    const char* from;
    char* to;
    size_t len;
  };
  std::vector<Piece> pieces;
  auto add_copy = [&](const char* from, char* to, size_t len) {
    constexpr size_t PIECE = size_t(4) << 20;
    for (size_t o = 0; o < len; o += PIECE) pieces.push_back({from + o, to + o, std::min(PIECE, len - o)});
  };
  auto run_pieces = [&] {
    std::atomic<size_t> next{0};
    acs_pool::run((int)std::min(T, std::max<size_t>(pieces.size(), 1)), [&](int) {
      for (size_t x; (x = next.fetch_add(1)) < pieces.size();) std::memcpy(pieces[x].to, pieces[x].from, pieces[x].len);
    });
    pieces.clear();
  };
  if (rstride == 2) {
    // sections 0, 1, 3, 4, 5 as in the blob; the padding after each zeroed
    const int secs[5] = {0, 1, 3, 4, 5};
    const size_t ends[6] = {doff[1], l0, 0, doff[4], doff[5], up_bytes};
    for (int k : secs) {
      add_copy(bsrc + off[k], d + doff[k], sz[k]);
      std::memset(d + doff[k] + sz[k], 0, ends[k] - doff[k] - sz[k]);
    }
    run_pieces();
    const uint32_t R0 = (uint32_t)(lines / 16), P0 = (uint32_t)(p_rel / 8);
    auto rebase = [&](NodeRec& N) {
      N.res_off += R0;
      N.act_off += P0;
      N.subj_off += P0;
    };
    for (uint32_t k = 0; k < h.n_sets + h.n_pols; ++k) {
      NodeRec* N = (NodeRec*)(d + (k < h.n_sets ? doff[0] + (size_t)k * 64 : doff[1] + (size_t)(k - h.n_sets) * 64));
      rebase(*N);
    }
    const RuleResAttr* rres = (const RuleResAttr*)(bsrc + off[3]);
    const Pair* pairs = (const Pair*)(bsrc + off[4]);
    const size_t nr = h.n_rules, chunk = 8192;
    std::atomic<size_t> next{0};
    acs_pool::run((int)std::min(T, (nr + chunk - 1) / chunk), [&](int) {
      for (size_t c; (c = next.fetch_add(1)) * chunk < nr;)
        for (uint32_t r = (uint32_t)(c * chunk); r < std::min(nr, (c + 1) * chunk); ++r) {
          NodeRec N;
          std::memcpy(&N, bsrc + off[2] + (size_t)r * 64, 64);
          char* line = d + l0 + (size_t)r * 128;
          std::memset(line + 64, 0, 64);
          const uint32_t res_off = N.res_off, act_off = N.act_off;
          rebase(N);
          if (N.res_n <= 3) {  // validated: [res_off, res_off + res_n) lies in the pool
            std::memcpy(line + 64, rres + res_off, (size_t)N.res_n * sizeof(RuleResAttr));
            N.res_off = r * 8 + 4;
          }
          if (N.act_n <= 2) {
            std::memcpy(line + 112, pairs + act_off, (size_t)N.act_n * sizeof(Pair));
            N.act_off = r * 16 + 14;
          }
          std::memcpy(line, &N, 64);
        }
    });
  } else {
    add_copy(bsrc, d, total);
    run_pieces();
  }
  std::memset(d + up_bytes, 0, ev_off - up_bytes);
  uint32_t* evx = (uint32_t*)(d + ev_off);
  std::memset(evx, 0, ex_words * sizeof(uint32_t));  // (the builders OR bits into it)
  if (ex_words) {
    build_event_index((const NodeRec*)(bsrc + off[0]), h.n_sets, (const NodeRec*)(bsrc + off[1]), h.n_pols,
                      (const NodeRec*)(bsrc + off[2]), h.n_rules, evx);
    build_parents((const NodeRec*)(bsrc + off[0]), h.n_sets, (const NodeRec*)(bsrc + off[1]), h.n_pols,
                  (const NodeRec*)(bsrc + off[2]), h.n_rules, evx + ev_words);
  }
  const char* hi = t->host_img.data();
  bool copied = hipSetDevice(device) == hipSuccess && hipMalloc(&t->dev, img_total + 128) == hipSuccess;
  if (copied && prev && prev->device == device && prev->host_img.size() == img_total && prev->view.rstride == rstride) {
    // delta: the previous image copied on the device, the differing 64-KB blocks uploaded
    constexpr size_t BLK = acs_tables::DELTA_BLOCK;
    copied = hipMemcpy(t->dev, prev->dev, img_total, hipMemcpyDeviceToDevice) == hipSuccess;
    t->delta_ok = true;
    const size_t nblk = (img_total + BLK - 1) / BLK;
    std::vector<uint8_t> differs(nblk, 0);  // blocks compared over the pool, uploaded in order
    std::atomic<size_t> next{0};
    acs_pool::run((int)std::min(T, std::max<size_t>(nblk / 16, 1)), [&](int) {
      for (size_t b; (b = next.fetch_add(1)) < nblk;) {
        const size_t o = b * BLK, len = std::min(BLK, img_total - o);
        differs[b] = std::memcmp(hi + o, prev->host_img.data() + o, len) != 0;
      }
    });
    for (size_t b = 0; copied && b < nblk; ++b) {
      if (!differs[b]) continue;
      const size_t o = b * BLK, len = std::min(BLK, img_total - o);
      copied = hipMemcpy((char*)t->dev + o, hi + o, len, hipMemcpyHostToDevice) == hipSuccess;
      t->upload_bytes += len;
      t->delta_blocks.push_back((uint32_t)b);
    }
  } else if (copied) {
    copied = hipMemcpy(t->dev, hi, img_total, hipMemcpyHostToDevice) == hipSuccess;
    t->upload_bytes = img_total;
  }
  if (!copied ||
      hipStreamCreateWithFlags(&t->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&t->ev0) != hipSuccess || hipEventCreate(&t->ev1) != hipSuccess) {
    fail("acs_compile: device allocation / upload failed");
    acs_free(t);
    return nullptr;
  }
  char* base = (char*)t->dev;
  t->view.sets = (const NodeRec*)(base + doff[0]);
  t->view.pols = (const NodeRec*)(base + doff[1]);
  t->view.rules = (const NodeRec*)(base + doff[2]);
  // rule lines: one base for both attribute pools (offsets rebased above)
  t->view.rres = (const RuleResAttr*)(base + (rstride == 2 ? doff[2] : doff[3]));
  t->view.pairs = (const Pair*)(base + (rstride == 2 ? doff[2] : doff[4]));
  t->view.u32pool = (const uint32_t*)(base + doff[5]);
  t->view.n_sets = h.n_sets;
  t->view.n_pols = h.n_pols;
  t->view.n_rules = h.n_rules;
  t->view.id_user = h.id_user;
  t->view.rstride = rstride;
  // the index packs a set's rule end in 30 bits (flags in bits 30 / 31): a store of 2^30 rules or
  // more runs without it (no set is skipped for it; the decisions are the same)
  t->view.ev_index = h.n_rules < (1u << 30) ? (const uint32_t*)(base + ev_off) : nullptr;
  t->view.parents = (const uint32_t*)(base + ev_off) + ev_words;
  t->image_bytes = img_total;
  return t;
}

extern "C" {

void acs_free(acs_tables* t) {
  if (!t) return;
  for (acs_tables* p : t->peers) acs_free(p);
  t->peers.clear();
  (void)hipSetDevice(t->device);
  if (t->dev) (void)hipFree(t->dev);
  if (t->ev0) (void)hipEventDestroy(t->ev0);
  if (t->ev1) (void)hipEventDestroy(t->ev1);
  if (t->stream) (void)hipStreamDestroy(t->stream);
  t->dws.release();
  t->hws.release();
  t->ows.release();
  for (int k = 0; k < acs_tables::CHUNK_SLOTS; ++k) {
    t->cws[k].release();
    if (t->cstream[k]) (void)hipStreamDestroy(t->cstream[k]);
  }
  if (t->hstage) (void)hipHostFree(t->hstage);
  if (t->hperm) (void)hipHostFree(t->hperm);
  for (hipEvent_t e : t->tev)
    if (e) (void)hipEventDestroy(e);
  delete t;
}

// A replica of primary t's image on `device` (C0: copied over the device interconnect, not again
// from the host).  prev (optional): this device's replica of the image t was updated from
// (acs_compile_update) — then the replica is prev's image copied on the device with only t's
// delta blocks copied from t.
static acs_tables* make_replica(const acs_tables* t, int device, const acs_tables* prev) {
  auto* r = new acs_tables();
  r->device = device;
  r->rx_rows_min = t->rx_rows_min;
  r->view = t->view;
  r->image_bytes = t->image_bytes;
  bool ok = hipSetDevice(r->device) == hipSuccess && hipMalloc(&r->dev, t->image_bytes + 128) == hipSuccess;
  if (ok && prev && t->delta_ok && prev->device == device && prev->image_bytes == t->image_bytes) {
    ok = hipMemcpy(r->dev, prev->dev, t->image_bytes, hipMemcpyDeviceToDevice) == hipSuccess;
    for (size_t k = 0; ok && k < t->delta_blocks.size(); ++k) {
      const size_t o = (size_t)t->delta_blocks[k] * acs_tables::DELTA_BLOCK;
      const size_t len = std::min(acs_tables::DELTA_BLOCK, t->image_bytes - o);
      ok = hipMemcpyPeer((char*)r->dev + o, r->device, (const char*)t->dev + o, t->device, len) == hipSuccess;
    }
  } else if (ok) {
    ok = hipMemcpyPeer(r->dev, r->device, t->dev, t->device, t->image_bytes) == hipSuccess;
  }
  if (!ok || hipStreamCreateWithFlags(&r->stream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&r->ev0) != hipSuccess || hipEventCreate(&r->ev1) != hipSuccess) {
    fail("acs_compile_multi: replica allocation / peer copy failed");
    acs_free(r);
    return nullptr;
  }
  // rebase the view's pointers from the primary's image onto the replica's
  auto rebase = [&](const void* p) -> const void* { return (const char*)r->dev + ((const char*)p - (const char*)t->dev); };
  r->view.sets = (const NodeRec*)rebase(t->view.sets);
  r->view.pols = (const NodeRec*)rebase(t->view.pols);
  r->view.rules = (const NodeRec*)rebase(t->view.rules);
  r->view.rres = (const RuleResAttr*)rebase(t->view.rres);
  r->view.pairs = (const Pair*)rebase(t->view.pairs);
  r->view.u32pool = (const uint32_t*)rebase(t->view.u32pool);
  r->view.ev_index = t->view.ev_index ? (const uint32_t*)rebase(t->view.ev_index) : nullptr;
  r->view.parents = (const uint32_t*)rebase(t->view.parents);
  r->sort = t->sort;
  r->chunk = t->chunk;
  return r;
}

acs_tables* acs_compile_multi(const void* blob, size_t n_bytes, const int* devices, int n_devices) {
  if (!devices || n_devices < 1) {
    fail("acs_compile_multi: no devices");
    return nullptr;
  }
  acs_tables* t = acs_compile(blob, n_bytes, devices[0]);
  if (!t) return nullptr;
  for (int k = 1; k < n_devices; ++k) {
    acs_tables* r = make_replica(t, devices[k], nullptr);
    if (!r) {
      acs_free(t);
      return nullptr;
    }
    t->peers.push_back(r);
  }
  (void)hipSetDevice(t->device);
  return t;
}

// ---------------------------------------------------------------- rule-sharded handles (C1)
// The sub-image of policy sets [s0, s1) of a validated blob: those sets' node records, their
// policies' and rules' child ranges rebased to the slice and NF_CLEAN_BELOW recomputed from the
// slice's first set (the other shards find the events below it), the pools whole (pool offsets
// unchanged), no codec section.  *b: the slice's first global set / policy / rule.
static std::vector<char> slice_blob(const void* blob, uint32_t s0, uint32_t s1, ShardBase* b) {
  acs_blob_header h;
  std::memcpy(&h, blob, sizeof h);
  const char* p = (const char*)blob + align16(sizeof h);
  const NodeRec* sets = (const NodeRec*)p;
  p += align16((size_t)h.n_sets * sizeof(NodeRec));
  const NodeRec* pols = (const NodeRec*)p;
  p += align16((size_t)h.n_pols * sizeof(NodeRec));
  const NodeRec* rules = (const NodeRec*)p;
  p += align16((size_t)h.n_rules * sizeof(NodeRec));
  const size_t pool_bytes = align16((size_t)h.n_rres * sizeof(RuleResAttr)) + align16((size_t)h.n_pairs * sizeof(Pair)) +
                            align16((size_t)h.n_u32pool * sizeof(uint32_t));
  const uint32_t p0 = s0 < s1 ? sets[s0].child_begin : 0u, p1 = s0 < s1 ? sets[s1 - 1].child_end : 0u;
  const uint32_t r0 = p0 < p1 ? pols[p0].child_begin : 0u, r1 = p0 < p1 ? pols[p1 - 1].child_end : r0;
  *b = ShardBase{s0, p0, r0};
  acs_blob_header o = h;
  o.n_sets = s1 - s0;
  o.n_pols = p1 - p0;
  o.n_rules = r1 - r0;
  for (uint32_t& x : o.reserved) x = 0;
  const size_t total = align16(sizeof o) + align16((size_t)o.n_sets * sizeof(NodeRec)) +
                       align16((size_t)o.n_pols * sizeof(NodeRec)) + align16((size_t)o.n_rules * sizeof(NodeRec)) +
                       pool_bytes;
  std::vector<char> out(total, 0);
  char* q = out.data();
  std::memcpy(q, &o, sizeof o);
  q += align16(sizeof o);
  NodeRec* S = (NodeRec*)q;
  bool clean_so_far = true;
  for (uint32_t k = 0; k < o.n_sets; ++k) {
    NodeRec n = sets[s0 + k];
    n.child_begin -= p0;
    n.child_end -= p0;
    n.nflags &= (uint8_t)~NF_CLEAN_BELOW;
    if (clean_so_far) n.nflags |= NF_CLEAN_BELOW;
    clean_so_far = clean_so_far && (n.nflags & NF_CLEAN);
    S[k] = n;
  }
  q += align16((size_t)o.n_sets * sizeof(NodeRec));
  NodeRec* P = (NodeRec*)q;
  for (uint32_t k = 0; k < o.n_pols; ++k) {
    NodeRec n = pols[p0 + k];
    n.child_begin -= r0;
    n.child_end -= r0;
    n.fe -= r0;
    P[k] = n;
  }
  q += align16((size_t)o.n_pols * sizeof(NodeRec));
  if (o.n_rules) std::memcpy(q, rules + r0, (size_t)o.n_rules * sizeof(NodeRec));
  q += align16((size_t)o.n_rules * sizeof(NodeRec));
  std::memcpy(q, p, pool_bytes);
  return out;
}

// Contiguous set runs [cut[k], cut[k + 1]), balanced by sets + policies + rules
// (acs_mi355x/shard.partition).
static std::vector<uint32_t> shard_cuts(const void* blob, int parts) {
  acs_blob_header h;
  std::memcpy(&h, blob, sizeof h);
  const NodeRec* sets = (const NodeRec*)((const char*)blob + align16(sizeof h));
  const NodeRec* pols = (const NodeRec*)((const char*)sets + align16((size_t)h.n_sets * sizeof(NodeRec)));
  std::vector<double> cum(h.n_sets + 1, 0.0);
  for (uint32_t s = 0; s < h.n_sets; ++s) {
    double w = 1.0 + (sets[s].child_end - sets[s].child_begin);
    for (uint32_t q = sets[s].child_begin; q < sets[s].child_end && q < h.n_pols; ++q)
      w += pols[q].child_end - pols[q].child_begin;
    cum[s + 1] = cum[s] + w;
  }
  std::vector<uint32_t> cut{0};
  for (int r = 1; r < parts; ++r) {
    const double want = cum[h.n_sets] * r / parts;
    uint32_t c = (uint32_t)(std::lower_bound(cum.begin(), cum.end(), want) - cum.begin());
    cut.push_back(std::min(std::max(c, cut.back()), h.n_sets));
  }
  cut.push_back(h.n_sets);
  return cut;
}

// Test hook (tests/test_rule_shard_lib.py): shard k of `parts` as acs_compile_sharded cuts it.
void* acs_internal_blob_alloc(size_t n);  // acs_compiler.cpp
int acs_internal_shard_blob(const void* blob, size_t n_bytes, int parts, int k, void** out, size_t* out_len,
                            acs_shard* base) {
  if (!blob || n_bytes < sizeof(acs_blob_header) || parts < 1 || k < 0 || k >= parts || !out || !out_len || !base)
    return fail("acs_internal_shard_blob: bad argument");
  uint32_t rows = 0;
  if (acs_internal_check_blob(blob, n_bytes, &rows)) return -1;
  const std::vector<uint32_t> cut = shard_cuts(blob, parts);
  ShardBase b{};
  std::vector<char> img = slice_blob(blob, cut[k], cut[k + 1], &b);
  void* mem = acs_internal_blob_alloc(img.size());  // freed by acs_blob_free
  if (!mem) return fail("acs_internal_shard_blob: out of memory");
  std::memcpy(mem, img.data(), img.size());
  *out = mem;
  *out_len = img.size();
  base->set_base = b.set_base;
  base->pol_base = b.pol_base;
  base->rule_base = b.rule_base;
  return 0;
}

// Test hook: a batch's class rows (and role rows) cut to a shard's nodes on the host, with
// the slice_rows_kernel's code (acs_eval.h RowSlice / slice_word).  layout[6] <- the shard's
// row words, cand_wp, cand_wr, cand_wsu, cand_wpu, cand_wv; dst_rows NULL: layout only.
int acs_internal_slice_rows(const acs_req_batch* b, uint32_t g_pols, const acs_shard* base, uint32_t ns,
                            uint32_t np, uint32_t nr, uint32_t* dst_rows, uint32_t* dst_role_rows, uint32_t* layout) {
  if (!b || !base || !layout || !b->cand) return fail("acs_internal_slice_rows: bad argument");
  const ShardBase sb{base->set_base, base->pol_base, base->rule_base};
  const RowSlice L = make_row_slice(g_pols, b->cand_wp, b->cand_wr, b->cand_wsu, b->cand_wpu, b->cand_wv, sb, ns, np, nr);
  const uint32_t lay[6] = {L.words, L.wp, L.wr, L.wsu, L.wpu, L.wv};
  std::memcpy(layout, lay, sizeof lay);
  if (!dst_rows) return 0;
  for (uint32_t r = 0; r < b->cand_rows; ++r)
    for (uint32_t w = 0; w < L.words; ++w)
      dst_rows[(size_t)r * L.words + w] = slice_word(b->cand + (size_t)r * b->cand_words, b->cand_words, L, w);
  if (b->role_key && dst_role_rows)
    for (uint32_t r = 0; r < b->role_rows; ++r)
      for (uint32_t w = 0; w < L.words; ++w)
        dst_role_rows[(size_t)r * L.words + w] =
            slice_word(b->role_rows_bits + (size_t)r * b->cand_words, b->cand_words, L, w);
  return 0;
}

// prev (optional, acs_compile_update): the sharded handle this store replaces — shard k compiled
// against prev's shard k (a delta when its slice keeps the shape)
static acs_tables* compile_sharded(const void* blob, size_t n_bytes, const int* devices, int n_devices,
                                   const acs_tables* prev) {
  if (!blob || n_bytes < sizeof(acs_blob_header) || !devices || n_devices < 1) {
    fail("acs_compile_sharded: bad argument");
    return nullptr;
  }
  acs_blob_header h;
  std::memcpy(&h, blob, sizeof h);
  if (h.magic != ACS_BLOB_MAGIC || h.version != ACS_ABI_VERSION) {
    fail("acs_compile_sharded: bad blob magic/version");
    return nullptr;
  }
  const size_t need = align16(sizeof h) + align16((size_t)h.n_sets * sizeof(NodeRec)) +
                      align16((size_t)h.n_pols * sizeof(NodeRec)) + align16((size_t)h.n_rules * sizeof(NodeRec)) +
                      align16((size_t)h.n_rres * sizeof(RuleResAttr)) + align16((size_t)h.n_pairs * sizeof(Pair)) +
                      align16((size_t)h.n_u32pool * sizeof(uint32_t));
  uint32_t rows = 0;
  if (need > n_bytes) {
    fail("acs_compile_sharded: blob shorter than its header declares");
    return nullptr;
  }
  if (acs_internal_check_blob(blob, n_bytes, &rows)) return nullptr;
  const std::vector<uint32_t> cut = shard_cuts(blob, n_devices);
  acs_tables* t = nullptr;
  for (int k = 0; k < n_devices; ++k) {
    ShardBase b{};
    const std::vector<char> img = slice_blob(blob, cut[k], cut[k + 1], &b);
    const acs_tables* p = prev ? (k == 0 ? prev : prev->peers[(size_t)k - 1]) : nullptr;
    acs_tables* s = compile_image(img.data(), img.size(), devices[k], p && p->device == devices[k] ? p : nullptr);
    if (!s) {
      acs_free(t);
      return nullptr;
    }
    s->sharded = 1;
    s->base = b;
    s->g_sets = h.n_sets;
    s->g_pols = h.n_pols;
    s->g_rules = h.n_rules;
    s->rx_rows_min = rows;
    if (prev) {
      s->sort = prev->sort;
      s->chunk = prev->chunk;
    }
    if (!t) t = s;
    else t->peers.push_back(s);
  }
  (void)hipSetDevice(t->device);
  return t;
}

acs_tables* acs_compile_sharded(const void* blob, size_t n_bytes, const int* devices, int n_devices) {
  return compile_sharded(blob, n_bytes, devices, n_devices, nullptr);
}

int acs_device_list(const acs_tables* t, int* devices, int n) {
  if (!t) return fail("acs_device_list: null tables");
  const int m = 1 + (int)t->peers.size();
  for (int k = 0; k < n && k < m; ++k) devices[k] = k == 0 ? t->device : t->peers[k - 1]->device;
  return m;
}

uint32_t acs_wia_words_per_request(const acs_tables* t) {
  if (t->sharded) return bits_layout(t->g_sets, t->g_pols, t->g_rules).words;  // the joined rows
  return bits_layout(t->view.n_sets, t->view.n_pols, t->view.n_rules).words;
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
  B.cand_wsu = b->cand_wsu;
  B.cand_wpu = b->cand_wpu;
  B.cand_wv = b->cand_wv;
  B.no_verdicts = ACS_AB_NO_VERDICTS ? 1u : 0u;
  if (ACS_AB_NO_USEFUL) B.cand_wsu = B.cand_wpu = 0;
  B.no_cut = ACS_AB_NO_CUT ? 1u : 0u;
  // long rows: the LDS union covers the set and policy sections (rule words: the lanes' rows)
  B.lds_pref = b->cand_wr < LDS_FILTER_WORDS ? b->cand_wr : LDS_FILTER_WORDS;
  B.role_major = b->role_key ? 1u : 0u;  // role-major keys (c5 A/B: 269 ms class-major, 244 ms role-major, r02_h)
  B.cand_rows = b->cand ? b->cand_rows : 0u;
  B.role_key = b->cand ? b->role_key : nullptr;
  B.role_bits = b->role_rows_bits;
  B.role_rows = b->role_key ? b->role_rows : 0u;
  // compact batches (no SoA rows) always read their lines; SoA batches may skip them (A/B)
  B.lines = (const ReqLine*)b->lines;  // (composed class rows are read from the lines)
  B.ext = b->ext;
  return B;
}

int acs_set_option(acs_tables* t, int option, int value) {
  if (!t) return fail("acs_set_option: null tables");
  std::lock_guard<std::mutex> lock(t->mu);  // the host-buffer entry points read these under it
  if (option == ACS_OPT_SORT) {
    t->sort = value ? 1 : 0;
    return 0;
  }
  if (option == ACS_OPT_CHUNK) {
    if (value < 0) return fail("acs_set_option: ACS_OPT_CHUNK must be >= 0");
    t->chunk = (size_t)value;
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

// Sort-key geometry of a batch: low field bits and the key's end bit.
static void sort_bits(const Batch& B, uint32_t* lowbits_out, uint32_t* end_bit_out) {
  // Low field: the dense role key with a role factor; otherwise none — a class row already
  // folds in the action filter (measured: 0 low bits time the same as 4 or 8, r01_sort).
  uint32_t lowbits = 0;
  if (B.role_key) {
    lowbits = 1;
    while (lowbits < 16 && (B.role_rows - 1) >> lowbits) ++lowbits;
  }
  uint32_t end_bit = lowbits;  // keys < (cand_rows + 1) << lowbits
  while (end_bit < 32 && (uint64_t(B.cand_rows) >> (end_bit - lowbits)) != 0) ++end_bit;
  *lowbits_out = lowbits;
  *end_bit_out = end_bit;
}

static size_t radix_scratch_bytes(size_t n) {
  const size_t nt = (n + SORT_TILE - 1) / SORT_TILE, ng = (nt + SCAN_GROUP - 1) / SCAN_GROUP;
  return 4 * n * sizeof(uint32_t) + (size_t)RADIX * (nt + ng) * sizeof(uint32_t);
}

// LSD passes over (k0, v0) of n pairs in the scratch `base` (radix_scratch_bytes(n)): pass 0's
// histogram already written by the caller when hist0; returns the sorted values.
static int radix_passes(uint32_t* base, size_t n, uint32_t end_bit, bool hist0, hipStream_t s, const uint32_t** vals) {
  const uint32_t passes = end_bit ? (end_bit + 7) / 8 : 1;
  const uint32_t nt = (uint32_t)((n + SORT_TILE - 1) / SORT_TILE);
  const uint32_t ng = (nt + SCAN_GROUP - 1) / SCAN_GROUP;
  uint32_t* k0 = base;
  uint32_t* k1 = k0 + n;
  uint32_t* v0 = k1 + n;
  uint32_t* v1 = v0 + n;
  uint32_t* counts = v1 + n;
  uint32_t* gsum = counts + (size_t)RADIX * nt;
  for (uint32_t p = 0; p < passes; ++p) {
    if (p > 0 || !hist0) {
      hipLaunchKernelGGL(radix_histogram_kernel, dim3(nt), dim3(BLOCK), 0, s, (const uint32_t*)k0, (uint32_t)n,
                         8 * p, counts);
      HIP_OK(hipGetLastError());
    }
    hipLaunchKernelGGL(radix_tile_scan_kernel, dim3(ng), dim3(RADIX), 0, s, counts, nt, gsum);
    HIP_OK(hipGetLastError());
    hipLaunchKernelGGL(radix_group_scan_kernel, dim3(1), dim3(RADIX), 0, s, gsum, ng);
    HIP_OK(hipGetLastError());
    hipLaunchKernelGGL(radix_scatter_kernel, dim3(nt), dim3(BLOCK), 0, s, (const uint32_t*)k0, (const uint32_t*)v0,
                       k1, v1, (const uint32_t*)counts, (const uint32_t*)gsum, (uint32_t)n, 8 * p,
                       (uint32_t)(p + 1 < passes));
    HIP_OK(hipGetLastError());
    std::swap(k0, k1);
    std::swap(v0, v1);
  }
  *vals = v0;
  return 0;
}

// Coherence sort: permutation of request indices ordered by (class, low field).
// pad (counting path only): each class's run starts a wave; *lanes = the launch width (holes and
// the tail past the padded runs hold 0xFFFFFFFF).  Without padding *lanes = n.
static int coherence_perm(acs_tables* t, Workspace& W, const Batch& B, hipStream_t s, const uint32_t** perm,
                          bool pad = false, size_t* lanes = nullptr) {
  *perm = nullptr;
  if (lanes) *lanes = B.n;
  if (!t->sort || B.n < 2 * BLOCK) return 0;
  const size_t n = B.n;
  uint32_t lowbits, end_bit;
  sort_bits(B, &lowbits, &end_bit);
  // key space: class-major keys are < (cand_rows + 1) << lowbits, role-major ones < 2^end_bit
  const uint64_t K = B.role_major ? (1ull << end_bit) : ((uint64_t)B.cand_rows + 1u) << lowbits;
  if (K <= CS_BINS) {  // one counting pass (class_count_kernel)
    uint32_t nb = (uint32_t)((n + 1023) / 1024);
    if (nb > 256) nb = 256;  // one block per CU
    uint32_t chunk = (uint32_t)((n + nb - 1) / nb);
    if (chunk > CS_MAX_CHUNK) {
      chunk = CS_MAX_CHUNK;
      nb = (uint32_t)((n + chunk - 1) / chunk);
    }
    pad = pad && lanes;
    const size_t width = pad ? n + 63 * std::min<size_t>(n, K) : n;  // padded runs fit in it
    const size_t words = n + width + (size_t)nb * K + K;
    if (W.sort.reserve(words * sizeof(uint32_t))) return -1;
    uint32_t* keys = (uint32_t*)W.sort.p;
    uint32_t* out = keys + n;
    uint32_t* counts = out + width;
    if (pad) {
      HIP_OK(hipMemsetAsync(out, 0xFF, width * sizeof(uint32_t), s));
      *lanes = width;
    }
    uint32_t* tot = counts + (size_t)nb * K;
    hipLaunchKernelGGL(class_count_kernel, dim3(nb), dim3(CS_THREADS), 0, s, B, lowbits, end_bit - lowbits, chunk,
                       (uint32_t)K, keys, counts);
    HIP_OK(hipGetLastError());
    hipLaunchKernelGGL(class_columns_kernel, dim3((unsigned)((K + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, counts, nb,
                       (uint32_t)K, tot);
    HIP_OK(hipGetLastError());
    hipLaunchKernelGGL(class_bases_kernel, dim3(1), dim3(CS_THREADS), 0, s, tot, (uint32_t)K, (uint32_t)pad);
    HIP_OK(hipGetLastError());
    hipLaunchKernelGGL(class_scatter_kernel, dim3(nb), dim3(CS_THREADS), 0, s, (const uint32_t*)keys, (uint32_t)n,
                       chunk, (uint32_t)K, (const uint32_t*)counts, (const uint32_t*)tot, out);
    HIP_OK(hipGetLastError());
    *perm = out;
    return 0;
  }
  const uint32_t nt = (uint32_t)((n + SORT_TILE - 1) / SORT_TILE);
  if (W.sort.reserve(radix_scratch_bytes(n))) return -1;
  uint32_t* k0 = (uint32_t*)W.sort.p;
  uint32_t* v0 = k0 + 2 * n;
  uint32_t* counts = k0 + 4 * n;
  hipLaunchKernelGGL(sort_keys_kernel, dim3(nt), dim3(BLOCK), 0, s, B, lowbits, end_bit - lowbits, k0, v0, counts);
  HIP_OK(hipGetLastError());
  return radix_passes(k0, n, end_bit, true, s, perm);
}

// The order the evaluation kernels run a batch in: the encoder's coherence order when the batch
// carries one (it knows every request's class: no device sort on the step), else the device
// coherence sort (pad: wave-aligned class runs of the counting sort), or input order with
// ACS_OPT_SORT off.  *lanes = the launch width.
static int batch_order(acs_tables* t, Workspace& W, const acs_req_batch* b, const Batch& B, hipStream_t s,
                       const uint32_t** perm, bool pad, size_t* lanes) {
  *perm = nullptr;
  *lanes = b->n;
  if (b->perm && !ACS_AB_DEVICE_SORT) {
    if (b->perm_lanes < b->n || b->perm_lanes > 0xFFFFFFFFull) return fail("batch: perm_lanes outside [n, 2^32)");
    if (!t->sort) return 0;
    *perm = b->perm;
    *lanes = b->perm_lanes;
    return 0;
  }
  return coherence_perm(t, W, B, s, perm, pad, lanes);
}

// Small batches: a batch of fewer waves than the device holds runs as long as its longest wave,
// and short class runs make every wave mix several classes (it walks the union of their
// candidates).  Such a batch is spread over more waves, L requests each (the rest holes), L the
// smallest of 64 / 32 / ... / ACS_SPREAD_MIN_L that keeps the waves within ACS_SPREAD_PER_SIMD per
// SIMD of the device:
// each wave then holds fewer classes (profiles/r05_a: at 131,072 c3 requests every wave lasts
// about as long as the launch).
#ifndef ACS_SPREAD_MIN_L
// fewest requests per spread wave: c3 K1 at 131,072 / 32,768 / 4,096 requests 0.432 / 0.348 /
// 0.353 ms at 16, 0.390 / 0.276 / 0.236 at 8, 0.390 / 0.283 / 0.168 at 4 (r05_final/ab_c3_*)
#define ACS_SPREAD_MIN_L 4
#endif
#ifndef ACS_K2_SPREAD_MIN_L
#define ACS_K2_SPREAD_MIN_L 16  // K2 (c4 131,072: 1.683 ms at 16, 1.875 at 8; r05_o, r05_u)
#endif
#ifndef ACS_SPREAD_PER_SIMD
// 0: off.  c3 131,072 requests: K1 0.814 ms unspread, 0.670 at 4, 0.543 at 8 (r05_e), 0.446 at 16
// with the skips; 524,288: 0.905 at 8 (unspread), 0.658 at 16 (r05_g, r05_i)
#define ACS_SPREAD_PER_SIMD 16
#endif
__global__ __launch_bounds__(BLOCK) void spread_perm_kernel(const uint32_t* __restrict__ in, uint32_t lanes, uint32_t L,
                                                            uint32_t out_lanes, uint32_t* __restrict__ out) {
  const uint32_t j = blockIdx.x * BLOCK + threadIdx.x;
  if (j >= out_lanes) return;
  const uint32_t q = j & 63u, k = (j >> 6) * L + q;
  out[j] = q < L && k < lanes ? (in ? in[k] : k) : 0xFFFFFFFFu;
}

// *spread: set when the batch was spread (its waves hold fewer than 64 requests)
static int spread_waves(acs_tables* t, Workspace& W, hipStream_t s, const uint32_t** perm, size_t* lanes,
                        uint32_t min_l, bool* spread = nullptr) {
  if (spread) *spread = false;
  if (!ACS_SPREAD_PER_SIMD || !t->sort) return 0;
  if (!t->simds) {
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, t->device) != hipSuccess || cus <= 0) cus = 256;
    t->simds = 4 * (uint32_t)cus;
  }
  const size_t cap = (size_t)t->simds * ACS_SPREAD_PER_SIMD;
  uint32_t L = 64;
  while (L > min_l && (*lanes + L / 2 - 1) / (L / 2) <= cap) L /= 2;
  if (L == 64) return 0;
  const size_t out_lanes = (*lanes + L - 1) / L * 64;
  if (W.spread.reserve(out_lanes * sizeof(uint32_t))) return -1;
  hipLaunchKernelGGL(spread_perm_kernel, dim3((unsigned)((out_lanes + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, *perm,
                     (uint32_t)*lanes, L, (uint32_t)out_lanes, (uint32_t*)W.spread.p);
  HIP_OK(hipGetLastError());
  *perm = (const uint32_t*)W.spread.p;
  *lanes = out_lanes;
  if (spread) *spread = true;
  return 0;
}

// whatIsAllowed runs without wave-aligned class runs: an encoder order that carries holes (0xFFFFFFFF
// lanes padding each class run to a wave) is compacted on the device, stably, into its n requests
// (select_* kernels, no host sync: every request appears exactly once).  K2's waves then mix the
// ~36-request classes of a 1M batch, but there are 2.3x fewer of them: c4 1M K2 4.03 -> 3.43 ms
// (r06_h), while K1 keeps the holes (c3r1 1M 0.41 padded vs 0.75, c3 0.76 vs 0.84) except in a
// batch with ACL_NONE requests whose lanes are mostly holes (is_allowed_launch).

static int drop_holes(Workspace& W, const uint32_t** perm, size_t* lanes, uint32_t n, hipStream_t s) {
  if (!*perm || *lanes <= n) return 0;
  const uint32_t nt = (uint32_t)((*lanes + SORT_TILE - 1) / SORT_TILE);
  // room for every lane of the order (a malformed order of the device entry points, which do not
  // validate it, can select more than n: still written inside the buffer)
  if (W.nopad.reserve((*lanes + 2 * (size_t)nt + 4) * sizeof(uint32_t))) return -1;
  uint32_t* out = (uint32_t*)W.nopad.p;
  uint32_t* cnt = out + *lanes;
  uint32_t* mx = cnt + nt;
  uint32_t* total = mx + nt;
  const PermEntries p{*perm, n};
  hipLaunchKernelGGL(select_count_kernel<PermEntries>, dim3(nt), dim3(BLOCK), 0, s, p, (uint32_t)*lanes, cnt, mx);
  hipLaunchKernelGGL(select_scan_kernel, dim3(1), dim3(BLOCK), 0, s, cnt, (const uint32_t*)mx, nt, total);
  hipLaunchKernelGGL(select_write_kernel<PermEntries>, dim3(nt), dim3(BLOCK), 0, s, p, (uint32_t)*lanes,
                     (const uint32_t*)cnt, *perm, out);
  HIP_OK(hipGetLastError());
  *perm = out;
  *lanes = n;
  return 0;
}

static int is_allowed_launch(acs_tables* t, Workspace& W, const acs_req_batch* b, acs_decision* out, hipStream_t s) {
  Batch B = to_batch(b);
  const uint32_t* perm = nullptr;
  // wave-aligned class runs when the classes are short (most waves would mix two or three
  // classes and walk the union of their candidates): 32 to 256 requests per class on average
  // (shorter classes would multiply the launch width)
  const bool pad = !ACS_AB_NO_PAD && B.cand && (uint64_t)B.n >= 32ull * B.cand_rows &&
                   (uint64_t)B.n < 256ull * B.cand_rows;
  size_t lanes = b->n;
  bool spread = false;
  if (batch_order(t, W, b, B, s, &perm, pad, &lanes)) return -1;
  // a batch with ACL_NONE requests whose wave-aligned class runs are mostly holes (more than 40 %
  // of the lanes) runs without them: its waves are as long as their ACL lanes' walks whichever
  // classes they mix (c3adv 1M, 57 % holes: 1.669 → 1.638 ms, r06_h)
  if ((b->hints & ACS_HINT_ACL_NONE) && perm && (lanes - b->n) * 5 > lanes * 2 &&
      drop_holes(W, &perm, &lanes, B.n, s))
    return -1;
  const bool padded = lanes > b->n;  // wave-aligned class runs (holes): one class per wave
  if (spread_waves(t, W, s, &perm, &lanes, ACS_SPREAD_MIN_L, &spread)) return -1;
  // waves that mix classes: spread, or unpadded with short class runs (< 256 requests per class
  // row on average), or long rows (the general Filter form: a wave ORs its lanes' rule words)
  const FilterForm form = filter_form(B);
  const bool mixed = spread || (!padded && form != FilterForm::All &&
                                (form == FilterForm::General || (uint64_t)b->n < 256ull * B.cand_rows));
  dim3 grid((unsigned)((lanes + BLOCK - 1) / BLOCK));
  const int slot = (int)(t->launches % acs_tables::RING);
  if (t->timing) HIP_OK(hipEventRecord(t->tev[2 * slot], s));
  // (Rejected A/Bs: the own-row skips in the ACL_NONE instantiation, c3adv 1M 1.773 vs 1.782 ms,
  // r05_u; the skipping instantiation for every plain batch, c3 10M 3.10 vs 3.02 ms, r05_j.)
  if (b->hints & ACS_HINT_ACL_NONE)
    ACS_LAUNCH_FILTERED_X(is_allowed_kernel, ACS_TARGS_ACL_NONE, grid, filter_lds_bytes(B), s, filter_form(B),
                          B.hdr == nullptr, t->view, B, perm, (uint32_t)lanes, (Decision*)out);
  else if (mixed)
    ACS_LAUNCH_FILTERED_X(is_allowed_kernel, ACS_TARGS_ACL_PLAIN_SK, grid, filter_lds_bytes(B), s, filter_form(B),
                          B.hdr == nullptr, t->view, B, perm, (uint32_t)lanes, (Decision*)out);
  else
    ACS_LAUNCH_FILTERED_X(is_allowed_kernel, ACS_TARGS_ACL_PLAIN, grid, filter_lds_bytes(B), s, filter_form(B),
                          B.hdr == nullptr, t->view, B, perm, (uint32_t)lanes, (Decision*)out);
  HIP_OK(hipGetLastError());
  if (t->timing) {
    HIP_OK(hipEventRecord(t->tev[2 * slot + 1], s));
    t->launches++;
  }
  return 0;
}

int acs_is_allowed_device(acs_tables* t, const acs_req_batch* b, acs_decision* out, void* stream) {
  if (refuse_sharded(t, "acs_is_allowed_device")) return -1;
  if (!t || !b) return fail("acs_is_allowed_device: null argument");
  if (b->n == 0) return 0;
  return is_allowed_launch(t, t->dws, b, out, (hipStream_t)stream);
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

static int what_is_allowed_launch(acs_tables* t, Workspace& W, const acs_req_batch* b, uint32_t* bits, uint32_t* obl,
                                  uint32_t* obl_n, acs_decision* out, hipStream_t s) {
  Batch B = to_batch(b);
  const uint32_t* perm = nullptr;
  size_t lanes = b->n;
  if (((uintptr_t)bits & 15u) != 0) return fail("acs_what_is_allowed_device: bits must be 16-byte aligned");
  if (batch_order(t, W, b, B, s, &perm, false, &lanes)) return -1;
  const int slot = (int)(t->launches % acs_tables::RING);
  // the timed K2 includes the order's compaction and the template pass
  if (t->timing) HIP_OK(hipEventRecord(t->tev[2 * slot], s));
  if (drop_holes(W, &perm, &lanes, B.n, s) || spread_waves(t, W, s, &perm, &lanes, ACS_K2_SPREAD_MIN_L)) return -1;
  dim3 grid((unsigned)((lanes + BLOCK - 1) / BLOCK));
  const BitsLayout BL = bits_layout(t->view.n_sets, t->view.n_pols, t->view.n_rules);
  const TplLayout TL = tpl_layout(t->view.n_sets, t->view.n_pols, t->view.n_rules);
  // templates: batches whose class rows carry verdicts in the LDS form, without a role factor
  const bool use_tpl = filter_form(B) == FilterForm::Lds && !B.role_key && B.cand_rows &&
                       t->view.parents && (size_t)(BLOCK / 64) * TL.stride * 4 <= 64 * 1024;
  const uint32_t* tpl = nullptr;
  if (use_tpl) {
    if (W.tpl.reserve((size_t)B.cand_rows * TL.stride * sizeof(uint32_t))) return -1;
    tpl = (const uint32_t*)W.tpl.p;
    hipLaunchKernelGGL(wia_template_kernel, dim3((B.cand_rows + BLOCK / 64 - 1) / (BLOCK / 64)), dim3(BLOCK),
                       (size_t)(BLOCK / 64) * TL.stride * 4, s, t->view, B, TL, BL, (uint32_t*)W.tpl.p);
  }
  ACS_LAUNCH_FILTERED(what_is_allowed_kernel, grid, filter_lds_bytes(B), s, filter_form(B), B.hdr == nullptr, t->view, B, perm, (uint32_t)lanes, BL, bits,
                      obl, obl_n, (Decision*)out, tpl, TL);
  HIP_OK(hipGetLastError());
  if (t->timing) {
    HIP_OK(hipEventRecord(t->tev[2 * slot + 1], s));
    t->launches++;
  }
  return 0;
}

int acs_what_is_allowed_device(acs_tables* t, const acs_req_batch* b, uint32_t* bits, uint32_t* obl,
                               uint32_t* obl_n, acs_decision* out, void* stream) {
  if (refuse_sharded(t, "acs_what_is_allowed_device")) return -1;
  if (!t || !b) return fail("acs_what_is_allowed_device: null argument");
  if (b->n == 0) return 0;
  return what_is_allowed_launch(t, t->dws, b, bits, obl, obl_n, out, (hipStream_t)stream);
}

constexpr uint32_t OBL_CAP_LIMIT = 1u << 20;

}  // extern "C"

// The obligation-only pass on one image; the ranges cut the sets of the whole store (g_sets, this
// image holding [set_base, + its n_sets): a shard of a rule-sharded handle).
static int obl_launch(acs_tables* t, const acs_req_batch* b, const uint32_t* idx, size_t m, uint32_t chunks,
                      uint32_t cap, uint32_t* obl, uint32_t* obl_n, hipStream_t stream, uint32_t g_sets,
                      uint32_t set_base) {
  if (m == 0 || b->n == 0) return 0;
  Batch B = to_batch(b);
  const size_t lanes = ((m + 63) & ~(size_t)63) * chunks;  // each range padded to whole waves
  ACS_LAUNCH_FILTERED(what_is_allowed_obl_kernel, dim3((unsigned)((lanes + BLOCK - 1) / BLOCK)), filter_lds_bytes(B),
                      stream, filter_form(B), B.hdr == nullptr, t->view, B, idx, (uint32_t)m, chunks, cap, obl,
                      obl_n, g_sets, set_base);
  HIP_OK(hipGetLastError());
  return 0;
}

extern "C" {

int acs_what_is_allowed_obl_device(acs_tables* t, const acs_req_batch* b, const uint32_t* idx, size_t m,
                                   uint32_t chunks, uint32_t cap, uint32_t* obl, uint32_t* obl_n, void* stream) {
  if (refuse_sharded(t, "acs_what_is_allowed_obl_device")) return -1;
  if (!t || !b || (m && (!idx || !obl || !obl_n))) return fail("acs_what_is_allowed_obl_device: null argument");
  if (cap == 0 || cap > OBL_CAP_LIMIT) return fail("acs_what_is_allowed_obl_device: cap must be in [1, 2^20]");
  if (chunks == 0 || chunks > 64) return fail("acs_what_is_allowed_obl_device: chunks must be in [1, 64]");
  if (m > 0xFFFFFFFFull || m * chunks > 0xFFFFFFFFull) return fail("acs_what_is_allowed_obl_device: too many requests");
  return obl_launch(t, b, idx, m, chunks, cap, obl, obl_n, (hipStream_t)stream, t->view.n_sets, 0);
}

}  // extern "C"

// idx[0..*m) <- the items of p (n of them) selected, in index order (map[i] when map); syncs s.
// *vmax <- the largest value of a selected item.
template <class P>
static int select_device(Workspace& W, const P& p, size_t n, const uint32_t* map, uint32_t* idx, size_t* m,
                         uint32_t* vmax, hipStream_t s) {
  const uint32_t nt = (uint32_t)((n + SORT_TILE - 1) / SORT_TILE);
  if (W.out.reserve((2 * (size_t)nt + 4) * sizeof(uint32_t))) return -1;
  uint32_t* cnt = (uint32_t*)W.out.p;
  uint32_t* mx = cnt + nt;
  uint32_t* total = mx + nt;
  hipLaunchKernelGGL(select_count_kernel<P>, dim3(nt), dim3(BLOCK), 0, s, p, (uint32_t)n, cnt, mx);
  HIP_OK(hipGetLastError());
  hipLaunchKernelGGL(select_scan_kernel, dim3(1), dim3(BLOCK), 0, s, cnt, (const uint32_t*)mx, nt, total);
  HIP_OK(hipGetLastError());
  hipLaunchKernelGGL(select_write_kernel<P>, dim3(nt), dim3(BLOCK), 0, s, p, (uint32_t)n, (const uint32_t*)cnt, map,
                     idx);
  HIP_OK(hipGetLastError());
  uint32_t h[2] = {0, 0};
  HIP_OK(hipMemcpyAsync(h, total, sizeof h, hipMemcpyDeviceToHost, s));
  HIP_OK(hipStreamSynchronize(s));
  *m = h[0];
  if (vmax) *vmax = h[1];
  return 0;
}

extern "C" {

int acs_overflow_index_device(acs_tables* t, const acs_req_batch* b, const acs_decision* out, uint32_t* idx, size_t* m,
                              void* stream) {
  if (!t || !b || !m || (b->n && (!out || !idx))) return fail("acs_overflow_index_device: null argument");
  *m = 0;
  if (b->n == 0) return 0;
  const hipStream_t s = (hipStream_t)stream;
  const Batch B = to_batch(b);
  const FlaggedRecords p{(const Decision*)out, OF_OBL_OVERFLOW};
  if (select_device(t->ows, p, B.n, nullptr, idx, m, nullptr, s)) return -1;
  // the coherence order of K2 (class, low field; stable: request order within a key), so
  // that a wave of the obligation pass shares its candidate rows
  if (!t->sort || *m < 2 || !B.cand) return 0;
  uint32_t lowbits, end_bit;
  sort_bits(B, &lowbits, &end_bit);
  if (t->ows.sort.reserve(radix_scratch_bytes(*m))) return -1;
  uint32_t* k0 = (uint32_t*)t->ows.sort.p;
  hipLaunchKernelGGL(gather_sort_keys_kernel, dim3((unsigned)((*m + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s, B,
                     (const uint32_t*)idx, (uint32_t)*m, lowbits, end_bit - lowbits, k0, k0 + 2 * *m);
  HIP_OK(hipGetLastError());
  const uint32_t* sorted = nullptr;
  if (radix_passes(k0, *m, end_bit, false, s, &sorted)) return -1;
  HIP_OK(hipMemcpyAsync(idx, sorted, *m * sizeof(uint32_t), hipMemcpyDeviceToDevice, s));
  return 0;
}

int acs_overflow_repass_device(acs_tables* t, const uint32_t* obl_n, const uint32_t* idx, size_t m, uint32_t chunks,
                               uint32_t cap, uint32_t* idx_out, size_t* m_out, uint32_t* cap_out, void* stream) {
  if (!t || !m_out || !cap_out || (m && (!obl_n || !idx || !idx_out)))
    return fail("acs_overflow_repass_device: null argument");
  if (chunks == 0 || chunks > 64) return fail("acs_overflow_repass_device: chunks must be in [1, 64]");
  if (m > 0xFFFFFFFFull) return fail("acs_overflow_repass_device: too many requests");
  *m_out = 0;
  *cap_out = 0;
  if (m == 0) return 0;
  const TruncatedLogs p{obl_n, (uint32_t)m, chunks, cap};
  return select_device(t->ows, p, m, idx, idx_out, m_out, cap_out, (hipStream_t)stream);
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

constexpr size_t IMG_ALIGN = 256;

// The device image of a host batch: every section the kernels read, copied into one
// grow-only device buffer (no per-call allocation) with one async copy per section — from
// pinned memory (the native codec's buffers) these run at full PCIe speed.  A compact batch
// ships request lines + extension records + arena + regex matrix + class rows (~220 B per
// request at c3); an SoA batch its rows as well.
struct Image {
  acs_req_batch d{};
  struct Sec {
    const void* src;
    size_t bytes;
    const void** dst;
  };
  std::vector<Sec> secs;
  size_t total = 0;
  void add(const void* src, size_t bytes, const void** dst) {
    if (!src) {
      *dst = nullptr;
      return;
    }
    secs.push_back({src, bytes, dst});
    total += (bytes + IMG_ALIGN - 1) & ~(IMG_ALIGN - 1);
  }
};

int upload_batch(Workspace& W, const acs_req_batch* b, acs_req_batch* dev, hipStream_t s) {
  Image I;
  I.d = *b;
  const size_t n = b->n;
  if (b->hdr) {
    I.add(b->hdr, n * sizeof(ReqHdr), &I.d.hdr);
    I.add(b->res, n * QMAX * sizeof(ReqRes), &I.d.res);
    I.add(b->subj, n * SMAX * sizeof(Pair), &I.d.subj);
    I.add(b->act, n * AMAX * sizeof(Pair), &I.d.act);
    I.add(b->roles, n * RMAX * sizeof(uint32_t), (const void**)&I.d.roles);
  }
  I.add(b->lines, n * sizeof(ReqLine), &I.d.lines);
  I.add(b->ext, b->ext_words * sizeof(uint32_t), (const void**)&I.d.ext);
  I.add(b->arena, b->arena_words * sizeof(uint32_t), (const void**)&I.d.arena);
  I.add(b->rx, (size_t)b->rx_cols * b->rx_rows, (const void**)&I.d.rx);
  if (b->cand) I.add(b->cand, (size_t)b->cand_rows * b->cand_words * sizeof(uint32_t), (const void**)&I.d.cand);
  if (b->role_key) {
    I.add(b->role_key, n * sizeof(uint32_t), (const void**)&I.d.role_key);
    I.add(b->role_rows_bits, (size_t)b->role_rows * b->cand_words * sizeof(uint32_t),
          (const void**)&I.d.role_rows_bits);
  }
  if (b->perm) I.add(b->perm, b->perm_lanes * sizeof(uint32_t), (const void**)&I.d.perm);
  if (W.img.reserve(I.total ? I.total : IMG_ALIGN)) return -1;
  char* base = (char*)W.img.p;
  size_t off = 0;
  for (const Image::Sec& x : I.secs) {
    if (x.bytes) HIP_OK(hipMemcpyAsync(base + off, x.src, x.bytes, hipMemcpyHostToDevice, s));
    *x.dst = base + off;
    off += (x.bytes + IMG_ALIGN - 1) & ~(IMG_ALIGN - 1);
  }
  *dev = I.d;
  return 0;
}

// Requests [lo, hi) of a compact batch on one device: their lines, extension records and
// arena words only (the shard's slices, uploaded so that the batch's absolute offsets still
// index them: the device pointers are based one slice-start below the copy), plus the whole
// regex matrix and class rows.  arena_end: per request, one past its last arena word.
// sperm: the shard's coherence order (shard-relative indices, the batch's order restricted to
// the shard) or empty.
// shared (optional): device copies of the batch-wide sections (regex matrix, class rows, role
// rows) already uploaded once for every chunk of a call (chunk_run); they are not copied again.
int upload_shard(Workspace& W, const acs_req_batch* b, size_t lo, size_t hi, const uint32_t* arena_end,
                 const uint32_t* sperm, size_t sperm_n, acs_req_batch* dev, hipStream_t s,
                 const acs_req_batch* shared = nullptr) {
  size_t plan[4];
  acs_internal_shard_plan(b, lo, hi, arena_end, plan);
  const size_t a0 = plan[0], a1 = plan[1], e0 = plan[2], e1 = plan[3];
  const size_t m = hi - lo;
  Image I;
  I.d = *b;
  I.d.n = (uint32_t)m;
  I.add((const ReqLine*)b->lines + lo, m * sizeof(ReqLine), &I.d.lines);
  const void* ext_dst = nullptr;
  const void* arena_dst = nullptr;
  I.add(b->ext ? b->ext + e0 : (const uint32_t*)b->lines, (e1 - e0) * 4, &ext_dst);
  I.add(b->arena + a0, (a1 - a0) * 4, &arena_dst);
  if (shared) {
    I.d.rx = shared->rx;
    I.d.cand = shared->cand;
    I.d.role_rows_bits = shared->role_rows_bits;
  } else {
    I.add(b->rx, (size_t)b->rx_cols * b->rx_rows, (const void**)&I.d.rx);
    if (b->cand) I.add(b->cand, (size_t)b->cand_rows * b->cand_words * sizeof(uint32_t), (const void**)&I.d.cand);
    if (b->role_key)
      I.add(b->role_rows_bits, (size_t)b->role_rows * b->cand_words * sizeof(uint32_t),
            (const void**)&I.d.role_rows_bits);
  }
  if (b->role_key) I.add(b->role_key + lo, m * sizeof(uint32_t), (const void**)&I.d.role_key);
  I.d.perm = nullptr;
  I.d.perm_lanes = 0;
  if (sperm && sperm_n) {
    I.add(sperm, sperm_n * sizeof(uint32_t), (const void**)&I.d.perm);
    I.d.perm_lanes = sperm_n;
  }
  if (W.img.reserve(I.total ? I.total : IMG_ALIGN)) return -1;
  char* base = (char*)W.img.p;
  size_t off = 0;
  for (const Image::Sec& x : I.secs) {
    if (x.bytes) HIP_OK(hipMemcpyAsync(base + off, x.src, x.bytes, hipMemcpyHostToDevice, s));
    *x.dst = base + off;
    off += (x.bytes + IMG_ALIGN - 1) & ~(IMG_ALIGN - 1);
  }
  // absolute offsets: the device pointers sit one slice-start below the copies (only
  // [start, end) is ever dereferenced)
  I.d.arena = (const uint32_t*)arena_dst - a0;
  I.d.ext = b->ext ? (const uint32_t*)ext_dst - e0 : nullptr;
  *dev = I.d;
  return 0;
}

// Output regions of one call in the workspace's `out` buffer (256-B aligned).
struct OutLayout {
  size_t off[4] = {};
  size_t total = 0;
  size_t put(size_t bytes) {
    const size_t o = total;
    total += (bytes + IMG_ALIGN - 1) & ~(IMG_ALIGN - 1);
    return o;
  }
};

}  // namespace

// Each of D contiguous shards' coherence order (shard-relative indices): the batch's order
// restricted to the shard, holes dropped (empty vectors when the batch carries none).
static std::vector<std::vector<uint32_t>> shard_perms(const acs_req_batch* b, size_t D) {
  const size_t n = b->n;
  auto lo_of = [&](size_t k) { return n * k / D; };
  std::vector<std::vector<uint32_t>> sperm(D);
  if (!b->perm) return sperm;
  for (size_t k = 0; k < D; ++k) sperm[k].reserve(lo_of(k + 1) - lo_of(k));
  for (size_t x = 0; x < b->perm_lanes; ++x) {
    const uint32_t i = b->perm[x];
    if (i >= n) continue;
    size_t k = std::min(D - 1, (size_t)i * D / n);
    while (k > 0 && i < lo_of(k)) --k;
    while (k + 1 < D && i >= lo_of(k + 1)) ++k;
    sperm[k].push_back((uint32_t)(i - lo_of(k)));
  }
  return sperm;
}

// One device, overlapped (host buffers): a large compact batch is cut into K contiguous chunks,
// each validated, uploaded as a shard (its lines, extension and arena slices, its coherence order)
// and evaluated on the pipeline slots' streams in turn, so chunk k + 1 is validated and uploaded
// while chunk k is evaluated and chunk k - 1's results come back (validate, H2D, kernel and D2H
// of one call were serial before: 17 GB/s effective at c3's 10M requests, BENCH_r05).  Before a
// slot is reused its stream is drained (its workspace may grow for the next chunk).  On an error
// the chunks already queued are drained and the outputs of the call are unspecified.
static constexpr size_t CHUNK_MAX_K = 16;  // chunks per call, at most (t->chunk: requests per chunk, at least)
// A batch is cut only into 8 chunks or more: a K1 launch on a small chunk lasts about as long as
// its longest wave, so a few chunks each pay that (c3adv 1M in 4 chunks: 61 M/s against 74 M/s in
// one launch, r06_final; c3 10M in 16 chunks: 155 M/s against 116 M/s)
static constexpr size_t CHUNK_MIN_K = 8;
static bool chunk_host_batch(const acs_tables* t, const acs_req_batch* b) {
  return t->chunk && t->peers.empty() && !t->sharded && !b->hdr && b->lines && b->n >= CHUNK_MIN_K * t->chunk;
}

// The chunks' coherence orders into the page-locked t->hperm: chunk k's order (the batch's
// perm restricted to [lo_k, hi_k), chunk-relative, holes dropped) at [lo_k, hi_k), built over the
// pool in two passes (count per part and chunk, then place), and checked as acs_internal_check_batch2
// checks a perm: every index < n or a hole, every request exactly once.
static int chunk_perms(acs_tables* t, const acs_req_batch* b, size_t K) {
  const size_t n = b->n, L = b->perm_lanes;
  if (L < n || L > 0xFFFFFFFFull) return fail("batch: perm_lanes");
  if (t->hperm_n < n) {
    if (t->hperm) HIP_OK(hipHostFree(t->hperm));
    t->hperm = nullptr;
    t->hperm_n = 0;
    HIP_OK(hipHostMalloc((void**)&t->hperm, (n + n / 8) * sizeof(uint32_t), 0));
    t->hperm_n = n + n / 8;
  }
  auto lo_of = [&](size_t k) { return n * k / K; };
  auto chunk_of = [&](uint32_t i) {
    size_t k = std::min(K - 1, (size_t)i * K / n);
    while (k > 0 && i < lo_of(k)) --k;
    while (k + 1 < K && i >= lo_of(k + 1)) ++k;
    return k;
  };
  const size_t T = std::max<size_t>(1, std::min<size_t>({16, std::thread::hardware_concurrency(), L / 65536 + 1}));
  std::vector<size_t> cnt(T * K, 0);
  std::atomic<size_t> bad{L};
  acs_pool::run((int)T, [&](int p) {
    size_t* c = cnt.data() + (size_t)p * K;
    for (size_t x = L * p / T; x < L * (p + 1) / T; ++x) {
      const uint32_t i = b->perm[x];
      if (i == 0xFFFFFFFFu) continue;
      if (i >= n) {
        size_t cur = bad.load();
        while (x < cur && !bad.compare_exchange_weak(cur, x)) {}
        return;
      }
      ++c[chunk_of(i)];
    }
  });
  if (bad.load() < L) return fail("batch: perm (an index outside the batch, or twice)");
  for (size_t k = 0; k < K; ++k) {  // per chunk: its parts' positions, and its count
    size_t at = lo_of(k);
    for (size_t p = 0; p < T; ++p) {
      const size_t c = cnt[p * K + k];
      cnt[p * K + k] = at;
      at += c;
    }
    if (at != lo_of(k + 1)) return fail("batch: perm misses requests (or holds one twice)");
  }
  acs_pool::run((int)T, [&](int p) {
    size_t* pos = cnt.data() + (size_t)p * K;
    for (size_t x = L * p / T; x < L * (p + 1) / T; ++x) {
      const uint32_t i = b->perm[x];
      if (i == 0xFFFFFFFFu) continue;
      const size_t k = chunk_of(i);
      t->hperm[pos[k]++] = (uint32_t)(i - lo_of(k));
    }
  });
  // with every chunk's count right, an index twice means another one missing: a bitmap per chunk
  std::atomic<int> dup{0};
  acs_pool::run((int)std::min(T, K), [&](int p) {
    for (size_t k = p; k < K; k += std::min(T, K)) {
      const size_t lo = lo_of(k), m = lo_of(k + 1) - lo;
      std::vector<uint64_t> seen((m + 63) / 64, 0);
      for (size_t x = 0; x < m; ++x) {
        const uint32_t r = t->hperm[lo + x];
        if (seen[r >> 6] >> (r & 63) & 1u) {
          dup = 1;
          return;
        }
        seen[r >> 6] |= 1ull << (r & 63);
      }
    }
  });
  if (dup) return fail("batch: perm (an index outside the batch, or twice)");
  return 0;
}

extern "C++" {
template <class F>
static int chunk_run(acs_tables* t, const acs_req_batch* b, const char* what, F chunk) {
  const size_t n = b->n, K = std::min(CHUNK_MAX_K, n / t->chunk);
  std::lock_guard<std::mutex> lock(t->mu);
  HIP_OK(hipSetDevice(t->device));
  if (b->perm && chunk_perms(t, b, K)) return -1;
  for (int q = 0; q < acs_tables::CHUNK_SLOTS; ++q)
    if (!t->cstream[q]) HIP_OK(hipStreamCreateWithFlags(&t->cstream[q], hipStreamNonBlocking));
  auto drain = [&] {
    const std::string err = g_err;
    for (int q = 0; q < acs_tables::CHUNK_SLOTS; ++q) (void)hipStreamSynchronize(t->cstream[q]);
    g_err = err;
    return -1;
  };
  const std::string sync_msg = std::string(what) + ": device synchronisation failed";
  // the batch-wide sections (regex matrix, class rows, role rows: c3 10M ~90 MB of class rows),
  // once per call into the handle's host-path workspace; the other slots wait for them
  acs_req_batch shared{};
  {
    Image I;
    I.add(b->rx, (size_t)b->rx_cols * b->rx_rows, (const void**)&shared.rx);
    if (b->cand) I.add(b->cand, (size_t)b->cand_rows * b->cand_words * sizeof(uint32_t), (const void**)&shared.cand);
    if (b->role_key && b->role_rows_bits)
      I.add(b->role_rows_bits, (size_t)b->role_rows * b->cand_words * sizeof(uint32_t),
            (const void**)&shared.role_rows_bits);
    if (t->hws.img.reserve(I.total ? I.total : IMG_ALIGN)) return -1;
    char* base = (char*)t->hws.img.p;
    size_t off = 0;
    for (const Image::Sec& x : I.secs) {
      if (x.bytes && hipMemcpyAsync(base + off, x.src, x.bytes, hipMemcpyHostToDevice, t->cstream[0]) != hipSuccess)
        return fail(sync_msg.c_str()), drain();
      *x.dst = base + off;
      off += (x.bytes + IMG_ALIGN - 1) & ~(IMG_ALIGN - 1);
    }
    if (hipEventRecord(t->ev0, t->cstream[0]) != hipSuccess) return fail(sync_msg.c_str()), drain();
    for (int q = 1; q < acs_tables::CHUNK_SLOTS; ++q)
      if (hipStreamWaitEvent(t->cstream[q], t->ev0, 0) != hipSuccess) return fail(sync_msg.c_str()), drain();
  }
  std::vector<uint32_t> arena_end(n / K + 1);
  for (size_t k = 0; k < K; ++k) {
    const int q = (int)(k % acs_tables::CHUNK_SLOTS);
    hipStream_t s = t->cstream[q];
    const size_t lo = n * k / K, hi = n * (k + 1) / K;
    // chunk k's requests validated (on the host threads, while the device works on chunk k - 1)
    acs_req_batch v = *b;
    v.n = hi - lo;
    v.lines = (const ReqLine*)b->lines + lo;
    if (b->role_key) v.role_key = b->role_key + lo;
    v.perm = nullptr;
    v.perm_lanes = 0;
    if (acs_internal_check_batch2(&v, t->view.n_sets, t->view.n_pols, t->view.n_rules, t->rx_rows_min,
                                  arena_end.data()) ||
        acs_internal_check_acl_none(&v, t->view.id_user))
      return drain();
    if (k >= (size_t)acs_tables::CHUNK_SLOTS && hipStreamSynchronize(s) != hipSuccess)
      return fail(sync_msg.c_str()), drain();
    acs_req_batch d;
    if (upload_shard(t->cws[q], &v, 0, hi - lo, arena_end.data(), b->perm ? t->hperm + lo : nullptr, hi - lo, &d, s,
                     &shared))
      return drain();
    if (chunk(t->cws[q], s, &d, lo, hi)) return drain();
  }
  for (int q = 0; q < acs_tables::CHUNK_SLOTS; ++q)
    if (hipStreamSynchronize(t->cstream[q]) != hipSuccess) return fail(sync_msg.c_str()), drain();
  return 0;
}
}  // extern "C++"

// A compact batch split over the handle and its replicas (acs_compile_multi): contiguous
// request shards, one per device, each uploaded (its slices only), sorted, decided and
// downloaded on that device's stream; all devices run concurrently.
static constexpr size_t MULTI_MIN_PER_DEVICE = 4096;

static bool split_across_devices(const acs_tables* t, const acs_req_batch* b) {
  return !t->peers.empty() && !b->hdr && b->lines && b->n >= 2 * MULTI_MIN_PER_DEVICE;
}

// Run `shard(T, d, lo, hi)` for each device's contiguous shard [lo, hi) of a compact batch: d is
// the shard uploaded to T (its slices, its coherence order), shard queues T's kernels and its
// copies into the caller's buffers on T->stream (returning nonzero on failure); then every
// device is synchronised.  On a failure every shard already queued is drained first (the caller
// may free its buffers, and the next call reuses the workspaces).
extern "C++" {
template <class F>
static int multi_run(acs_tables* t, const acs_req_batch* b, const uint32_t* arena_end, const char* what, F shard) {
  std::vector<acs_tables*> dev{t};
  dev.insert(dev.end(), t->peers.begin(), t->peers.end());
  size_t D = dev.size();
  if (b->n / D < MULTI_MIN_PER_DEVICE) D = b->n / MULTI_MIN_PER_DEVICE;
  const size_t n = b->n;
  auto lo_of = [&](size_t k) { return n * k / D; };
  // each shard's coherence order: the batch's order restricted to the shard (holes dropped)
  const std::vector<std::vector<uint32_t>> sperm = shard_perms(b, D);
  std::vector<std::unique_lock<std::mutex>> locks;
  for (size_t k = 0; k < D; ++k) locks.emplace_back(dev[k]->mu);
  size_t launched = 0;  // devices with work queued into the caller's buffers
  auto drain = [&] {
    const std::string err = g_err;
    for (size_t k = 0; k < launched; ++k) {
      (void)hipSetDevice(dev[k]->device);
      (void)hipStreamSynchronize(dev[k]->stream);
    }
    (void)hipSetDevice(t->device);
    g_err = err;
    return -1;
  };
  const std::string sync_msg = std::string(what) + ": device synchronisation failed";
  for (size_t k = 0; k < D; ++k) {
    acs_tables* T = dev[k];
    const size_t lo = lo_of(k), hi = lo_of(k + 1);
    if (hipSetDevice(T->device) != hipSuccess) return fail(sync_msg.c_str()), drain();
    launched = k + 1;  // the copies below are queued on T's stream from here on
    acs_req_batch d;
    if (upload_shard(T->hws, b, lo, hi, arena_end, sperm[k].data(), sperm[k].size(), &d, T->stream)) return drain();
    if (shard(T, &d, lo, hi)) return drain();
  }
  for (size_t k = 0; k < D; ++k) {
    if (hipSetDevice(dev[k]->device) != hipSuccess || hipStreamSynchronize(dev[k]->stream) != hipSuccess)
      return fail(sync_msg.c_str()), drain();
  }
  HIP_OK(hipSetDevice(t->device));
  return 0;
}
}  // extern "C++"

static int multi_is_allowed(acs_tables* t, const acs_req_batch* b, acs_decision* out, const uint32_t* arena_end) {
  return multi_run(t, b, arena_end, "acs_is_allowed", [&](acs_tables* T, const acs_req_batch* d, size_t lo, size_t hi) {
    if (T->hws.out.reserve((hi - lo) * sizeof(Decision))) return -1;
    if (is_allowed_launch(T, T->hws, d, (acs_decision*)T->hws.out.p, T->stream)) return -1;
    if (hipMemcpyAsync(out + lo, T->hws.out.p, (hi - lo) * sizeof(Decision), hipMemcpyDeviceToHost, T->stream) !=
        hipSuccess)
      return fail("acs_is_allowed: result copy failed");
    return 0;
  });
}

// whatIsAllowed over the replicas: each device decides its shard and writes its rows of the
// caller's bitset / logs / records (the same bytes as one device: K2 is per request).
static int multi_what_is_allowed(acs_tables* t, const acs_req_batch* b, uint32_t* bits, uint32_t* obl,
                                 uint32_t* obl_n, acs_decision* out, const uint32_t* arena_end) {
  const size_t words = acs_wia_words_per_request(t);
  return multi_run(t, b, arena_end, "acs_what_is_allowed",
                   [&](acs_tables* T, const acs_req_batch* d, size_t lo, size_t hi) {
    const size_t m = hi - lo;
    OutLayout O;
    const size_t o_bits = O.put(m * words * sizeof(uint32_t)), o_obl = O.put(m * 2 * OBL_MAX * sizeof(uint32_t));
    const size_t o_n = O.put(m * sizeof(uint32_t)), o_out = O.put(m * sizeof(Decision));
    if (T->hws.out.reserve(O.total)) return -1;
    char* ob = (char*)T->hws.out.p;
    if (what_is_allowed_launch(T, T->hws, d, (uint32_t*)(ob + o_bits), (uint32_t*)(ob + o_obl),
                               (uint32_t*)(ob + o_n), (acs_decision*)(ob + o_out), T->stream))
      return -1;
    if (hipMemcpyAsync(bits + lo * words, ob + o_bits, m * words * sizeof(uint32_t), hipMemcpyDeviceToHost,
                       T->stream) != hipSuccess ||
        hipMemcpyAsync(obl + lo * 2 * OBL_MAX, ob + o_obl, m * 2 * OBL_MAX * sizeof(uint32_t), hipMemcpyDeviceToHost,
                       T->stream) != hipSuccess ||
        hipMemcpyAsync(obl_n + lo, ob + o_n, m * sizeof(uint32_t), hipMemcpyDeviceToHost, T->stream) != hipSuccess ||
        hipMemcpyAsync(out + lo, ob + o_out, m * sizeof(Decision), hipMemcpyDeviceToHost, T->stream) != hipSuccess)
      return fail("acs_what_is_allowed: result copy failed");
    return 0;
  });
}

// Shard T of rule-sharded handle t: the whole batch uploaded to T, its class rows (and role rows)
// cut to T's nodes on the device (slice_rows_kernel, acs_eval.h RowSlice); *d: the device batch.
static int upload_shard_batch(acs_tables* t, acs_tables* T, const acs_req_batch* b, acs_req_batch* d) {
  if (upload_batch(T->hws, b, d, T->stream)) return -1;
  if (!b->cand) return 0;
  const RowSlice L = make_row_slice(t->g_pols, b->cand_wp, b->cand_wr, b->cand_wsu, b->cand_wpu, b->cand_wv, T->base,
                                    T->view.n_sets, T->view.n_pols, T->view.n_rules);
  const size_t rows_w = (size_t)b->cand_rows * L.words, role_w = b->role_key ? (size_t)b->role_rows * L.words : 0;
  if (T->hws.slice.reserve((rows_w + role_w + 1) * sizeof(uint32_t))) return -1;
  uint32_t* dst = (uint32_t*)T->hws.slice.p;
  if (rows_w)
    hipLaunchKernelGGL(slice_rows_kernel, dim3((unsigned)((rows_w + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, T->stream,
                       d->cand, b->cand_words, b->cand_rows, L, dst);
  if (role_w)
    hipLaunchKernelGGL(slice_rows_kernel, dim3((unsigned)((role_w + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, T->stream,
                       d->role_rows_bits, b->cand_words, b->role_rows, L, dst + rows_w);
  if (hipGetLastError() != hipSuccess) return fail("rule-sharded handle: row slice launch failed");
  d->cand = dst;
  d->cand_words = L.words;
  d->cand_wp = L.wp;
  d->cand_wr = L.wr;
  d->cand_wsu = L.wsu;
  d->cand_wpu = L.wpu;
  d->cand_wv = L.wv;
  d->role_rows_bits = role_w ? dst + rows_w : nullptr;
  return 0;
}

// ---- whatIsAllowed on a rule-sharded handle ("set-sharded bitsets concatenate
// (gather, no reduction); obligations merged on the host in set order").  whatIsAllowed keeps no
// state across policy sets but the push log and the first throw (accessController.ts:343-419), so
// each shard's run of sets is evaluated alone and the results are joined on the host:
//  * bitset rows: each section of a shard's row (its local sets / policies / rules) ORed into the
//    whole store's row at the shard's first global index (disjoint ranges);
//  * the first shard whose record carries an error decides the request (the walk stops at the
//    first set that throws): its record, aux made global, bits up to and including that shard;
//  * maskedProperty logs: the shards' logs concatenated in shard (= set) order, cut at
//    ACS_OBL_MAX entries; OF_OBL_OVERFLOW when a shard's log overflowed or the joined one did.
// The CPU test (tests/test_rule_shard_lib.py) runs the same join over the host core's shards.
namespace {
// OR bits [0, nbits) of src into dst from bit d0 (only words that receive a set bit are written)
void or_bits_at(uint32_t* dst, uint32_t d0, const uint32_t* src, uint32_t nbits) {
  const uint32_t words = (nbits + 31) / 32, sh = d0 & 31u;
  uint32_t* d = dst + (d0 >> 5);
  for (uint32_t w = 0; w < words; ++w) {
    uint32_t x = src[w];
    const uint32_t left = nbits - 32 * w;
    if (left < 32) x &= (1u << left) - 1u;
    if (!x) continue;
    d[w] |= x << sh;
    if (sh && (x >> (32u - sh))) d[w + 1] |= x >> (32u - sh);
  }
}
}  // namespace

extern "C" {
// One shard's whatIsAllowed outputs for the join (csrc: acs_what_is_allowed on a sharded handle;
// tests: the host core on the shard's sub-image).
typedef struct {
  acs_shard base;                     /* the shard's first global set / policy / rule */
  uint32_t n_sets, n_pols, n_rules;   /* its image's node counts */
  const uint32_t* bits;               /* [n][its words_per_req] */
  const uint32_t* obl;                /* [n][ACS_OBL_MAX][2] */
  const uint32_t* obl_n;              /* [n] */
  const acs_decision* out;            /* [n] */
} acs_internal_wia_part;

// Requests [lo, hi) of the join; g_*: the whole store's node counts; bits / obl / obl_n / out: the
// caller's outputs in the unsharded layout (bits zeroed here).
void acs_internal_wia_join(uint32_t g_sets, uint32_t g_pols, uint32_t g_rules, int parts,
                           const acs_internal_wia_part* P, size_t lo, size_t hi, uint32_t* bits, uint32_t* obl,
                           uint32_t* obl_n, acs_decision* out) {
  const BitsLayout G = bits_layout(g_sets, g_pols, g_rules);
  std::vector<BitsLayout> LL(parts);
  for (int k = 0; k < parts; ++k) LL[k] = bits_layout(P[k].n_sets, P[k].n_pols, P[k].n_rules);
  for (size_t i = lo; i < hi; ++i) {
    uint32_t* row = bits + i * G.words;
    std::memset(row, 0, (size_t)G.words * sizeof(uint32_t));
    Decision d{};
    std::memcpy(&d, &P[0].out[i], sizeof d);
    if (d.flags & OF_HOST_REQ) {  // request level: the same record from every shard, no bits, no log
      std::memcpy(&out[i], &d, sizeof d);
      obl_n[i] = 0;
      continue;
    }
    int last = parts - 1;  // the shards whose bits count (up to the first that threw)
    bool err = false;
    for (int k = 0; k < parts && !err; ++k) {
      Decision e;
      std::memcpy(&e, &P[k].out[i], sizeof e);
      if (e.flags & OF_ERR) {
        err = true;
        last = k;
        d = e;
        if (d.aux) d.aux += P[k].base.set_base;
      }
    }
    for (int k = 0; k <= last; ++k) {
      const uint32_t* src = P[k].bits + i * LL[k].words;
      or_bits_at(row, P[k].base.set_base, src, P[k].n_sets);
      or_bits_at(row + G.wp, P[k].base.pol_base, src + LL[k].wp, P[k].n_pols);
      or_bits_at(row + G.wr, P[k].base.rule_base, src + LL[k].wr, P[k].n_rules);
    }
    if (err) {
      std::memcpy(&out[i], &d, sizeof d);
      obl_n[i] = 0;
      continue;
    }
    Decision o{};
    uint32_t n = 0;
    for (int k = 0; k < parts; ++k) {
      Decision e;
      std::memcpy(&e, &P[k].out[i], sizeof e);
      if (e.flags & OF_OBL_OVERFLOW) o.flags |= OF_OBL_OVERFLOW;
      const uint32_t kn = P[k].obl_n[i];
      const uint32_t take = kn < OBL_MAX - n ? kn : OBL_MAX - n;
      if (take < kn) o.flags |= OF_OBL_OVERFLOW;
      std::memcpy(obl + (i * OBL_MAX + n) * 2, P[k].obl + (i * OBL_MAX) * 2, (size_t)take * 2 * sizeof(uint32_t));
      n += take;
    }
    obl_n[i] = n;
    std::memcpy(&out[i], &o, sizeof o);
  }
}

// The obligation-only pass's join: range c of request j is the concatenation of the shards' parts
// of range c (each shard ran the same global ranges clipped to its sets); its total is their sum,
// and its log is written only when it fits `cap` (else the caller re-runs with cap = the total).
void acs_internal_wia_obl_join(int parts, const uint32_t* const* part_obl, const uint32_t* const* part_n, size_t m,
                               uint32_t chunks, uint32_t cap, uint32_t* obl, uint32_t* obl_n) {
  for (size_t x = 0; x < (size_t)chunks * m; ++x) {
    uint64_t total = 0;
    bool outside = false;
    for (int k = 0; k < parts; ++k) {
      if (part_n[k][x] == 0xFFFFFFFFu) outside = true;
      total += part_n[k][x];
    }
    if (outside) {
      obl_n[x] = 0xFFFFFFFFu;
      continue;
    }
    obl_n[x] = total > 0xFFFFFFFEull ? 0xFFFFFFFEu : (uint32_t)total;
    if (total > cap) continue;
    uint32_t at = 0;
    for (int k = 0; k < parts; ++k) {
      std::memcpy(obl + (x * cap + at) * 2, part_obl[k] + x * cap * 2, (size_t)part_n[k][x] * 2 * sizeof(uint32_t));
      at += part_n[k][x];
    }
  }
}
}  // extern "C"

// The join over host threads (a few rows each).
static void wia_join_threaded(const acs_tables* t, const std::vector<acs_internal_wia_part>& P, size_t n,
                              uint32_t* bits, uint32_t* obl, uint32_t* obl_n, acs_decision* out) {
  const size_t T = std::max<size_t>(1, std::min<size_t>(16, std::min<size_t>(std::thread::hardware_concurrency(),
                                                                             n / 4096 + 1)));
  std::vector<std::thread> th;
  for (size_t k = 0; k < T; ++k)
    th.emplace_back([&, k] {
      acs_internal_wia_join(t->g_sets, t->g_pols, t->g_rules, (int)P.size(), P.data(), n * k / T, n * (k + 1) / T,
                            bits, obl, obl_n, out);
    });
  for (auto& x : th) x.join();
}

// Every shard evaluates the whole batch against its sets (K2 on its image, class rows cut to its
// nodes), the outputs come back to host staging, and the join writes the caller's buffers.
static int sharded_what_is_allowed(acs_tables* t, const acs_req_batch* b, uint32_t* bits, uint32_t* obl,
                                   uint32_t* obl_n, acs_decision* out) {
  if (acs_internal_check_batch(b, t->g_sets, t->g_pols, t->g_rules, t->rx_rows_min) ||
      acs_internal_check_acl_none(b, t->view.id_user))
    return -1;
  if (b->n > 0xFFFFFFFFull) return fail("acs_what_is_allowed: batch too large");
  std::vector<acs_tables*> dev{t};
  dev.insert(dev.end(), t->peers.begin(), t->peers.end());
  const size_t D = dev.size(), n = b->n;
  std::vector<std::unique_lock<std::mutex>> locks;
  for (size_t k = 0; k < D; ++k) locks.emplace_back(dev[k]->mu);
  struct Stage {
    std::vector<uint32_t> bits, obl, obl_n;
    std::vector<acs_decision> out;
  };
  std::vector<Stage> st(D);
  size_t launched = 0;
  auto drain = [&] {
    const std::string err = g_err;
    for (size_t k = 0; k < launched; ++k) {
      (void)hipSetDevice(dev[k]->device);
      (void)hipStreamSynchronize(dev[k]->stream);
    }
    (void)hipSetDevice(t->device);
    g_err = err;
    return -1;
  };
  for (size_t k = 0; k < D; ++k) {
    acs_tables* T = dev[k];
    const size_t words = bits_layout(T->view.n_sets, T->view.n_pols, T->view.n_rules).words;  // its own rows
    Stage& S = st[k];
    S.bits.resize(n * words);
    S.obl.resize(n * 2 * OBL_MAX);
    S.obl_n.resize(n);
    S.out.resize(n);
    if (hipSetDevice(T->device) != hipSuccess) return fail("acs_what_is_allowed: hipSetDevice failed"), drain();
    launched = k + 1;
    acs_req_batch d;
    if (upload_shard_batch(t, T, b, &d)) return drain();
    OutLayout O;
    const size_t o_bits = O.put(n * words * sizeof(uint32_t)), o_obl = O.put(n * 2 * OBL_MAX * sizeof(uint32_t));
    const size_t o_n = O.put(n * sizeof(uint32_t)), o_out = O.put(n * sizeof(Decision));
    if (T->hws.out.reserve(O.total)) return drain();
    char* ob = (char*)T->hws.out.p;
    if (what_is_allowed_launch(T, T->hws, &d, (uint32_t*)(ob + o_bits), (uint32_t*)(ob + o_obl), (uint32_t*)(ob + o_n),
                               (acs_decision*)(ob + o_out), T->stream))
      return drain();
    if (hipMemcpyAsync(S.bits.data(), ob + o_bits, n * words * sizeof(uint32_t), hipMemcpyDeviceToHost, T->stream) !=
            hipSuccess ||
        hipMemcpyAsync(S.obl.data(), ob + o_obl, n * 2 * OBL_MAX * sizeof(uint32_t), hipMemcpyDeviceToHost,
                       T->stream) != hipSuccess ||
        hipMemcpyAsync(S.obl_n.data(), ob + o_n, n * sizeof(uint32_t), hipMemcpyDeviceToHost, T->stream) !=
            hipSuccess ||
        hipMemcpyAsync(S.out.data(), ob + o_out, n * sizeof(Decision), hipMemcpyDeviceToHost, T->stream) != hipSuccess)
      return fail("acs_what_is_allowed: result copy failed"), drain();
  }
  for (size_t k = 0; k < D; ++k)
    if (hipSetDevice(dev[k]->device) != hipSuccess || hipStreamSynchronize(dev[k]->stream) != hipSuccess)
      return fail("acs_what_is_allowed: device synchronisation failed"), drain();
  HIP_OK(hipSetDevice(t->device));
  std::vector<acs_internal_wia_part> P(D);
  for (size_t k = 0; k < D; ++k) {
    const acs_tables* T = dev[k];
    P[k].base = acs_shard{T->base.set_base, T->base.pol_base, T->base.rule_base};
    P[k].n_sets = T->view.n_sets;
    P[k].n_pols = T->view.n_pols;
    P[k].n_rules = T->view.n_rules;
    P[k].bits = st[k].bits.data();
    P[k].obl = st[k].obl.data();
    P[k].obl_n = st[k].obl_n.data();
    P[k].out = st[k].out.data();
  }
  wia_join_threaded(t, P, n, bits, obl, obl_n, out);
  return 0;
}

// The obligation-only pass on a rule-sharded handle: every shard runs the same global set ranges
// clipped to its sets; the parts are joined per (range, request) in shard order.
static int sharded_what_is_allowed_obl(acs_tables* t, const acs_req_batch* b, const uint32_t* idx, size_t m,
                                       uint32_t chunks, uint32_t cap, uint32_t* obl, uint32_t* obl_n) {
  if (acs_internal_check_batch(b, t->g_sets, t->g_pols, t->g_rules, t->rx_rows_min) ||
      acs_internal_check_acl_none(b, t->view.id_user))
    return -1;
  std::vector<acs_tables*> dev{t};
  dev.insert(dev.end(), t->peers.begin(), t->peers.end());
  const size_t D = dev.size(), lanes = m * chunks;
  std::vector<std::unique_lock<std::mutex>> locks;
  for (size_t k = 0; k < D; ++k) locks.emplace_back(dev[k]->mu);
  std::vector<std::vector<uint32_t>> pobl(D), pn(D);
  size_t launched = 0;
  auto drain = [&] {
    const std::string err = g_err;
    for (size_t k = 0; k < launched; ++k) {
      (void)hipSetDevice(dev[k]->device);
      (void)hipStreamSynchronize(dev[k]->stream);
    }
    (void)hipSetDevice(t->device);
    g_err = err;
    return -1;
  };
  for (size_t k = 0; k < D; ++k) {
    acs_tables* T = dev[k];
    pobl[k].resize(lanes * 2 * (size_t)cap);
    pn[k].resize(lanes);
    if (hipSetDevice(T->device) != hipSuccess) return fail("acs_what_is_allowed_obl: hipSetDevice failed"), drain();
    launched = k + 1;
    acs_req_batch d;
    if (upload_shard_batch(t, T, b, &d)) return drain();
    OutLayout O;
    const size_t o_idx = O.put(m * sizeof(uint32_t)), o_obl = O.put(lanes * 2 * (size_t)cap * sizeof(uint32_t));
    const size_t o_n = O.put(lanes * sizeof(uint32_t));
    if (T->hws.out.reserve(O.total)) return drain();
    char* ob = (char*)T->hws.out.p;
    if (hipMemcpyAsync(ob + o_idx, idx, m * sizeof(uint32_t), hipMemcpyHostToDevice, T->stream) != hipSuccess)
      return fail("acs_what_is_allowed_obl: index upload failed"), drain();
    if (obl_launch(T, &d, (const uint32_t*)(ob + o_idx), m, chunks, cap, (uint32_t*)(ob + o_obl), (uint32_t*)(ob + o_n),
                   T->stream, t->g_sets, T->base.set_base))
      return drain();
    if (hipMemcpyAsync(pobl[k].data(), ob + o_obl, lanes * 2 * (size_t)cap * sizeof(uint32_t), hipMemcpyDeviceToHost,
                       T->stream) != hipSuccess ||
        hipMemcpyAsync(pn[k].data(), ob + o_n, lanes * sizeof(uint32_t), hipMemcpyDeviceToHost, T->stream) != hipSuccess)
      return fail("acs_what_is_allowed_obl: result copy failed"), drain();
  }
  for (size_t k = 0; k < D; ++k)
    if (hipSetDevice(dev[k]->device) != hipSuccess || hipStreamSynchronize(dev[k]->stream) != hipSuccess)
      return fail("acs_what_is_allowed_obl: device synchronisation failed"), drain();
  HIP_OK(hipSetDevice(t->device));
  std::vector<const uint32_t*> po(D), pc(D);
  for (size_t k = 0; k < D; ++k) {
    po[k] = pobl[k].data();
    pc[k] = pn[k].data();
  }
  acs_internal_wia_obl_join((int)D, po.data(), pc.data(), m, chunks, cap, obl, obl_n);
  return 0;
}

// A rule-sharded handle (acs_compile_sharded): every device evaluates the whole batch against
// its run of policy sets — the batch uploaded to each, its class rows cut to the device's nodes
// (slice_rows_kernel), K1, then the records turned into 64-bit keys (shard_key) — and the
// primary MAX-reduces the keys (peer copies over xGMI, max_keys_kernel) and decodes them into
// the records an unsharded evaluation writes.
static int sharded_is_allowed(acs_tables* t, const acs_req_batch* b, acs_decision* out) {
  if (acs_internal_check_batch(b, t->g_sets, t->g_pols, t->g_rules, t->rx_rows_min) ||
      acs_internal_check_acl_none(b, t->view.id_user))
    return -1;
  if (b->n > 0xFFFFFFFFull) return fail("acs_is_allowed: batch too large");
  std::vector<acs_tables*> dev{t};
  dev.insert(dev.end(), t->peers.begin(), t->peers.end());
  const size_t D = dev.size(), n = b->n;
  std::vector<std::unique_lock<std::mutex>> locks;
  for (size_t k = 0; k < D; ++k) locks.emplace_back(dev[k]->mu);
  size_t launched = 0;
  auto drain = [&] {
    const std::string err = g_err;
    for (size_t k = 0; k < launched; ++k) {
      (void)hipSetDevice(dev[k]->device);
      (void)hipStreamSynchronize(dev[k]->stream);
    }
    (void)hipSetDevice(t->device);
    g_err = err;
    return -1;
  };
  const dim3 grid_n((unsigned)((n + BLOCK - 1) / BLOCK));
  for (size_t k = 0; k < D; ++k) {
    acs_tables* T = dev[k];
    if (hipSetDevice(T->device) != hipSuccess) return fail("acs_is_allowed: hipSetDevice failed"), drain();
    launched = k + 1;
    acs_req_batch d;
    if (upload_shard_batch(t, T, b, &d)) return drain();
    if (T->hws.out.reserve(n * sizeof(Decision)) || T->hws.keys.reserve(n * sizeof(uint64_t) * (k == 0 ? 2 : 1)))
      return drain();
    if (is_allowed_launch(T, T->hws, &d, (acs_decision*)T->hws.out.p, T->stream)) return drain();
    hipLaunchKernelGGL(shard_key_kernel, grid_n, dim3(BLOCK), 0, T->stream, T->view, (const Decision*)T->hws.out.p,
                       (uint32_t)n, T->base, (uint64_t*)T->hws.keys.p);
    if (hipGetLastError() != hipSuccess || (k > 0 && hipEventRecord(T->ev1, T->stream) != hipSuccess))
      return fail("acs_is_allowed: shard key launch failed"), drain();
  }
  if (hipSetDevice(t->device) != hipSuccess) return fail("acs_is_allowed: hipSetDevice failed"), drain();
  uint64_t* keys = (uint64_t*)t->hws.keys.p;
  for (size_t k = 1; k < D; ++k) {
    if (hipStreamWaitEvent(t->stream, dev[k]->ev1, 0) != hipSuccess ||
        hipMemcpyPeerAsync(keys + n, t->device, dev[k]->hws.keys.p, dev[k]->device, n * sizeof(uint64_t),
                           t->stream) != hipSuccess)
      return fail("acs_is_allowed: key gather failed"), drain();
    hipLaunchKernelGGL(max_keys_kernel, grid_n, dim3(BLOCK), 0, t->stream, keys, (const uint64_t*)(keys + n),
                       (uint32_t)n);
  }
  hipLaunchKernelGGL(shard_decode_kernel, grid_n, dim3(BLOCK), 0, t->stream, (const uint64_t*)keys, (uint32_t)n,
                     (Decision*)t->hws.out.p);
  if (hipGetLastError() != hipSuccess ||
      hipMemcpyAsync(out, t->hws.out.p, n * sizeof(Decision), hipMemcpyDeviceToHost, t->stream) != hipSuccess)
    return fail("acs_is_allowed: decode / result copy failed"), drain();
  for (size_t k = 0; k < D; ++k)
    if (hipSetDevice(dev[k]->device) != hipSuccess || hipStreamSynchronize(dev[k]->stream) != hipSuccess)
      return fail("acs_is_allowed: device synchronisation failed"), drain();
  HIP_OK(hipSetDevice(t->device));
  return 0;
}

int acs_is_allowed(acs_tables* t, const acs_req_batch* b, acs_decision* out) {
  if (!t || !b || (b && b->n && !out)) return fail("acs_is_allowed: null argument");
  if (b->n == 0) return 0;
  if (t->sharded) return sharded_is_allowed(t, b, out);
  if (split_across_devices(t, b)) {
    std::vector<uint32_t> arena_end(b->n);
    if (acs_internal_check_batch2(b, t->view.n_sets, t->view.n_pols, t->view.n_rules, t->rx_rows_min,
                                  arena_end.data()) ||
        acs_internal_check_acl_none(b, t->view.id_user))
      return -1;
    return multi_is_allowed(t, b, out, arena_end.data());
  }
  if (chunk_host_batch(t, b)) {
    if (!b->lines) return fail("batch: compact batch without request lines");
    return chunk_run(t, b, "acs_is_allowed",
                     [&](Workspace& W, hipStream_t s, const acs_req_batch* d, size_t lo, size_t hi) {
      if (W.out.reserve((hi - lo) * sizeof(Decision))) return -1;
      if (is_allowed_launch(t, W, d, (acs_decision*)W.out.p, s)) return -1;
      if (hipMemcpyAsync(out + lo, W.out.p, (hi - lo) * sizeof(Decision), hipMemcpyDeviceToHost, s) != hipSuccess)
        return fail("acs_is_allowed: result copy failed");
      return 0;
    });
  }
  if (check_batch(t, b)) return -1;
  std::lock_guard<std::mutex> lock(t->mu);
  HIP_OK(hipSetDevice(t->device));
  acs_req_batch d;
  if (upload_batch(t->hws, b, &d, t->stream)) return -1;
  if (t->hws.out.reserve(b->n * sizeof(Decision))) return -1;
  void* dout = t->hws.out.p;
  HIP_OK(hipEventRecord(t->ev0, t->stream));
  if (is_allowed_launch(t, t->hws, &d, (acs_decision*)dout, t->stream)) return -1;
  HIP_OK(hipEventRecord(t->ev1, t->stream));
  HIP_OK(hipMemcpyAsync(out, dout, b->n * sizeof(Decision), hipMemcpyDeviceToHost, t->stream));
  HIP_OK(hipStreamSynchronize(t->stream));
  HIP_OK(hipEventElapsedTime(&t->last_ms, t->ev0, t->ev1));
  return 0;
}

int acs_what_is_allowed(acs_tables* t, const acs_req_batch* b, uint32_t* bits, uint32_t* obl, uint32_t* obl_n,
                        acs_decision* out) {
  if (!t || !b || (b->n && (!bits || !obl || !obl_n || !out))) return fail("acs_what_is_allowed: null argument");
  if (b->n == 0) return 0;
  if (t->sharded) return sharded_what_is_allowed(t, b, bits, obl, obl_n, out);
  if (split_across_devices(t, b)) {
    std::vector<uint32_t> arena_end(b->n);
    if (acs_internal_check_batch2(b, t->view.n_sets, t->view.n_pols, t->view.n_rules, t->rx_rows_min,
                                  arena_end.data()) ||
        acs_internal_check_acl_none(b, t->view.id_user))
      return -1;
    return multi_what_is_allowed(t, b, bits, obl, obl_n, out, arena_end.data());
  }
  if (check_batch(t, b)) return -1;
  std::lock_guard<std::mutex> lock(t->mu);
  HIP_OK(hipSetDevice(t->device));
  acs_req_batch d;
  if (upload_batch(t->hws, b, &d, t->stream)) return -1;
  const size_t n = b->n, words = acs_wia_words_per_request(t);
  // the logs come back packed (obl_n entries per request; see obl_pack_kernel) when the packed
  // offsets fit 32 bits
  const bool dense = n * (size_t)OBL_MAX < 0xFFFFFFFFull;
  const uint32_t nb = (uint32_t)((n + BLOCK - 1) / BLOCK);
  OutLayout O;
  const size_t o_bits = O.put(n * words * sizeof(uint32_t)), o_obl = O.put(n * 2 * OBL_MAX * sizeof(uint32_t));
  const size_t o_n = O.put(n * sizeof(uint32_t)), o_out = O.put(n * sizeof(Decision));
  const size_t o_blk = dense ? O.put(((size_t)nb + 2) * sizeof(uint32_t)) : 0;
  const size_t o_dense = dense ? O.put(n * 2 * OBL_MAX * sizeof(uint32_t)) : 0;
  if (t->hws.out.reserve(O.total)) return -1;
  char* ob = (char*)t->hws.out.p;
  HIP_OK(hipEventRecord(t->ev0, t->stream));
  if (what_is_allowed_launch(t, t->hws, &d, (uint32_t*)(ob + o_bits), (uint32_t*)(ob + o_obl), (uint32_t*)(ob + o_n),
                             (acs_decision*)(ob + o_out), t->stream))
    return -1;
  HIP_OK(hipEventRecord(t->ev1, t->stream));
  HIP_OK(hipMemcpyAsync(bits, ob + o_bits, n * words * sizeof(uint32_t), hipMemcpyDeviceToHost, t->stream));
  HIP_OK(hipMemcpyAsync(obl_n, ob + o_n, n * sizeof(uint32_t), hipMemcpyDeviceToHost, t->stream));
  HIP_OK(hipMemcpyAsync(out, ob + o_out, n * sizeof(Decision), hipMemcpyDeviceToHost, t->stream));
  if (!dense) {
    HIP_OK(hipMemcpyAsync(obl, ob + o_obl, n * 2 * OBL_MAX * sizeof(uint32_t), hipMemcpyDeviceToHost, t->stream));
    HIP_OK(hipStreamSynchronize(t->stream));
    HIP_OK(hipEventElapsedTime(&t->last_ms, t->ev0, t->ev1));
    return 0;
  }
  uint32_t* blk = (uint32_t*)(ob + o_blk);
  hipLaunchKernelGGL(obl_block_sums_kernel, dim3(nb), dim3(BLOCK), 0, t->stream, (const uint32_t*)(ob + o_n),
                     (uint32_t)n, blk);
  hipLaunchKernelGGL(obl_scan_blocks_kernel, dim3(1), dim3(BLOCK), 0, t->stream, blk, nb);
  hipLaunchKernelGGL(obl_pack_kernel, dim3(nb), dim3(BLOCK), 0, t->stream, (const uint2*)(ob + o_obl),
                     (const uint32_t*)(ob + o_n), (uint32_t)n, (const uint32_t*)blk, (uint2*)(ob + o_dense));
  HIP_OK(hipGetLastError());
  uint32_t tot[2] = {0, 0};
  HIP_OK(hipMemcpyAsync(tot, blk + nb, sizeof tot, hipMemcpyDeviceToHost, t->stream));
  HIP_OK(hipStreamSynchronize(t->stream));
  const size_t total = (size_t)tot[0] | ((size_t)tot[1] << 32);
  if (total > n * (size_t)OBL_MAX) return fail("acs_what_is_allowed: packed log size out of range");
  if (total * 8 > t->hstage_bytes) {
    if (t->hstage) HIP_OK(hipHostFree(t->hstage));
    t->hstage = nullptr;
    t->hstage_bytes = 0;
    const size_t want = total * 8 + total * 8 / 8 + 4096;
    HIP_OK(hipHostMalloc(&t->hstage, want, 0));
    t->hstage_bytes = want;
  }
  if (total) {
    HIP_OK(hipMemcpyAsync(t->hstage, ob + o_dense, total * 8, hipMemcpyDeviceToHost, t->stream));
    HIP_OK(hipStreamSynchronize(t->stream));
  }
  // each request's entries into its OBL_MAX-entry slot (its offset: the counts before it)
  const size_t T = std::max<size_t>(1, std::min<size_t>(16, std::thread::hardware_concurrency()));
  const size_t parts = std::min(T, (n + 65535) / 65536);
  std::vector<size_t> start(parts + 1, 0);
  for (size_t p = 0; p < parts; ++p) {  // entries before each part (one pass over obl_n per part)
    const size_t lo = n * p / parts, hi = n * (p + 1) / parts;
    size_t c = 0;
    for (size_t i = lo; i < hi; ++i) c += std::min<uint32_t>(obl_n[i], OBL_MAX);
    start[p + 1] = c;
  }
  for (size_t p = 0; p < parts; ++p) start[p + 1] += start[p];
  if (start[parts] != total) return fail("acs_what_is_allowed: packed log size mismatch");
  const uint64_t* src = (const uint64_t*)t->hstage;
  acs_pool::run((int)parts, [&](int p) {
    size_t at = start[p];
    for (size_t i = n * p / parts, hi = n * (p + 1) / parts; i < hi; ++i) {
      const uint32_t c = std::min<uint32_t>(obl_n[i], OBL_MAX);
      if (c) std::memcpy(obl + i * 2 * OBL_MAX, src + at, (size_t)c * 8);
      at += c;
    }
  });
  HIP_OK(hipEventElapsedTime(&t->last_ms, t->ev0, t->ev1));
  return 0;
}

int acs_what_is_allowed_obl(acs_tables* t, const acs_req_batch* b, const uint32_t* idx, size_t m, uint32_t chunks,
                            uint32_t cap, uint32_t* obl, uint32_t* obl_n) {
  if (!t || !b || (m && (!idx || !obl || !obl_n))) return fail("acs_what_is_allowed_obl: null argument");
  if (cap == 0 || cap > OBL_CAP_LIMIT) return fail("acs_what_is_allowed_obl: cap must be in [1, 2^20]");
  if (chunks == 0 || chunks > 64) return fail("acs_what_is_allowed_obl: chunks must be in [1, 64]");
  if (m == 0) return 0;
  if (m > 0xFFFFFFFFull || m * chunks > 0xFFFFFFFFull) return fail("acs_what_is_allowed_obl: too many requests");
  for (size_t k = 0; k < m; ++k)
    if (idx[k] >= b->n) return fail("acs_what_is_allowed_obl: request index outside the batch");
  if (t->sharded) return sharded_what_is_allowed_obl(t, b, idx, m, chunks, cap, obl, obl_n);
  if (check_batch(t, b)) return -1;
  std::lock_guard<std::mutex> lock(t->mu);
  HIP_OK(hipSetDevice(t->device));
  acs_req_batch d;
  if (upload_batch(t->hws, b, &d, t->stream)) return -1;
  const size_t lanes = m * chunks;
  OutLayout O;
  const size_t o_idx = O.put(m * sizeof(uint32_t)), o_obl = O.put(lanes * 2 * (size_t)cap * sizeof(uint32_t));
  const size_t o_n = O.put(lanes * sizeof(uint32_t));
  if (t->hws.out.reserve(O.total)) return -1;
  char* ob = (char*)t->hws.out.p;
  HIP_OK(hipMemcpyAsync(ob + o_idx, idx, m * sizeof(uint32_t), hipMemcpyHostToDevice, t->stream));
  if (acs_what_is_allowed_obl_device(t, &d, (const uint32_t*)(ob + o_idx), m, chunks, cap, (uint32_t*)(ob + o_obl),
                                     (uint32_t*)(ob + o_n), t->stream))
    return -1;
  HIP_OK(hipMemcpyAsync(obl, ob + o_obl, lanes * 2 * (size_t)cap * sizeof(uint32_t), hipMemcpyDeviceToHost,
                        t->stream));
  HIP_OK(hipMemcpyAsync(obl_n, ob + o_n, lanes * sizeof(uint32_t), hipMemcpyDeviceToHost, t->stream));
  HIP_OK(hipStreamSynchronize(t->stream));
  return 0;
}

// ---------------------------------------------------------------- decision pipeline
// JSON text -> decision records with encode and device work overlapped: the request array is
// delimited once, then cut into chunks; chunk k+1 is encoded on the host threads while chunk
// k's upload (from the codec's page-locked blocks), coherence sort, K1 and download run on
// one of two streams, each with its own device workspace and page-locked output staging.
struct acs_internal_items;
acs_internal_items* acs_internal_split(const char* json, size_t len, int threads, size_t* n);
void acs_internal_items_free(acs_internal_items* it);
acs_codec_batch* acs_internal_encode_range(acs_codec* c, const acs_internal_items* it, size_t lo, size_t hi,
                                           int threads);

}  // extern "C"

struct acs_pipeline {
  acs_tables* t = nullptr;
  acs_codec* c = nullptr;
  int threads = 1;
  uint32_t chunk = 131072;
  struct Slot {
    acs_tables* T = nullptr;  // the device this slot runs on (the handle or one of its replicas)
    hipStream_t stream = nullptr;
    hipEvent_t ev0 = nullptr, ev1 = nullptr, done = nullptr;
    Workspace ws;
    acs_decision* stage = nullptr;  // page-locked output staging
    size_t stage_n = 0;
    acs_codec_batch* batch = nullptr;  // in flight
    size_t lo = 0, n = 0;              // its requests
    bool busy = false;
  };
  std::vector<Slot> slot;  // two per device: chunk k -> device k % D, slot (k / D) % 2
  std::mutex mu;           // one run at a time per pipeline
  std::unordered_map<size_t, std::string> reasons;  // host-path requests of the last run
};

namespace {

double steady_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// Finish slot S: wait for its chunk, copy its records out, free its batch.
int pipeline_retire(acs_pipeline* p, acs_pipeline::Slot& S, acs_decision* out, acs_pipeline_stats* st) {
  if (!S.busy) return 0;
  const double w0 = steady_s();
  HIP_OK(hipEventSynchronize(S.done));
  const double w1 = steady_s();
  float ms = 0.f;
  HIP_OK(hipEventElapsedTime(&ms, S.ev0, S.ev1));
  std::memcpy(out + S.lo, S.stage, S.n * sizeof(acs_decision));
  for (size_t i = 0; i < S.n; ++i)
    if (S.stage[i].flags & ACS_OF_HOST_REQ) {
      const char* why = acs_codec_batch_reason(S.batch, (uint32_t)i);
      p->reasons[S.lo + i] = why ? why : "host path";
    }
  if (st) {
    st->wait_s += w1 - w0;
    st->gpu_ms += ms;
  }
  acs_codec_batch_free(S.batch);
  S.batch = nullptr;
  S.busy = false;
  return 0;
}

// Drop every slot's chunk without copying it anywhere: wait for its device work (its download
// writes the slot's own staging buffer, never the caller's), free its batch.  Run after a
// failed run — whose slots may still hold chunks in flight — and at the start of each run, so
// no later retire copies a stale chunk into a new caller's output.  Keeps the error message.
void pipeline_reset(acs_pipeline* p) {
  const std::string err = g_err;
  for (auto& S : p->slot) {
    if (S.busy) {
      (void)hipSetDevice(S.T->device);
      (void)hipEventSynchronize(S.done);
    }
    if (S.batch) acs_codec_batch_free(S.batch);
    S.batch = nullptr;
    S.busy = false;
    S.lo = S.n = 0;
  }
  (void)hipSetDevice(p->t->device);
  g_err = err;
}

}  // namespace

extern "C" {

acs_pipeline* acs_pipeline_create(acs_tables* t, acs_codec* c, int threads, uint32_t chunk) {
  if (!t || !c) {
    fail("acs_pipeline_create: null argument");
    return nullptr;
  }
  auto p = new acs_pipeline();
  p->t = t;
  p->c = c;
  p->threads = threads < 1 ? 1 : threads;
  p->chunk = chunk ? chunk : 131072;
  if (t->sharded) return p;  // a rule-sharded handle: each chunk through sharded_is_allowed (no slots)
  std::vector<acs_tables*> dev{t};
  dev.insert(dev.end(), t->peers.begin(), t->peers.end());
  p->slot.resize(2 * dev.size());
  for (size_t k = 0; k < p->slot.size(); ++k) {
    acs_pipeline::Slot& S = p->slot[k];
    S.T = dev[k / 2];
    if (hipSetDevice(S.T->device) != hipSuccess || hipStreamCreateWithFlags(&S.stream, hipStreamNonBlocking) != hipSuccess ||
        hipEventCreate(&S.ev0) != hipSuccess || hipEventCreate(&S.ev1) != hipSuccess ||
        hipEventCreateWithFlags(&S.done, hipEventDisableTiming) != hipSuccess) {
      fail("acs_pipeline_create: stream / event creation failed");
      acs_pipeline_free(p);
      return nullptr;
    }
  }
  (void)hipSetDevice(t->device);
  return p;
}

void acs_pipeline_free(acs_pipeline* p) {
  if (!p) return;
  for (auto& S : p->slot) {
    if (S.T) (void)hipSetDevice(S.T->device);
    if (S.busy) (void)hipEventSynchronize(S.done);
    if (S.batch) acs_codec_batch_free(S.batch);
    S.ws.release();
    if (S.stage) (void)hipHostFree(S.stage);
    if (S.ev0) (void)hipEventDestroy(S.ev0);
    if (S.ev1) (void)hipEventDestroy(S.ev1);
    if (S.done) (void)hipEventDestroy(S.done);
    if (S.stream) (void)hipStreamDestroy(S.stream);
  }
  if (!p->slot.empty()) (void)hipSetDevice(p->t->device);
  delete p;
}

}  // extern "C"

// The pipeline on a rule-sharded handle: chunk k is evaluated by sharded_is_allowed (every device
// its run of policy sets, the keys MAX-reduced on the primary) on a worker thread while the host
// encodes chunk k + 1; the records land straight in the caller's buffer.
static int pipeline_sharded(acs_pipeline* p, const acs_internal_items* items, size_t n, acs_decision* out,
                            acs_pipeline_stats* st) {
  struct Pending {
    std::thread th;
    acs_codec_batch* batch = nullptr;
    size_t lo = 0, n = 0;
    int rc = 0;
    std::string err;
    double ms = 0;
  } cur;
  auto finish = [&](Pending& P) -> int {
    if (!P.batch) return 0;
    const double w0 = steady_s();
    P.th.join();
    if (st) {
      st->wait_s += steady_s() - w0;
      st->gpu_ms += P.ms;
    }
    int rc = P.rc;
    if (rc) {
      g_err = P.err;
    } else {
      for (size_t i = 0; i < P.n; ++i)
        if (out[P.lo + i].flags & ACS_OF_HOST_REQ) {
          const char* why = acs_codec_batch_reason(P.batch, (uint32_t)i);
          p->reasons[P.lo + i] = why ? why : "host path";
        }
    }
    acs_codec_batch_free(P.batch);
    P.batch = nullptr;
    return rc;
  };
  for (size_t lo = 0; lo < n; lo += p->chunk) {
    const size_t hi = lo + p->chunk < n ? lo + p->chunk : n;
    const double e0 = steady_s();
    acs_codec_batch* b = acs_internal_encode_range(p->c, items, lo, hi, p->threads);
    if (!b) {
      const std::string err = g_err;
      finish(cur);
      g_err = err;
      return -1;
    }
    if (st) st->encode_s += steady_s() - e0;
    if (finish(cur)) {
      acs_codec_batch_free(b);
      return -1;
    }
    acs_req_batch view;
    if (acs_codec_batch_view(b, &view)) {
      acs_codec_batch_free(b);
      return -1;
    }
    cur.batch = b;
    cur.lo = lo;
    cur.n = hi - lo;
    cur.rc = 0;
    acs_tables* t = p->t;
    cur.th = std::thread([t, view, out, lo, &cur] {
      const double a = steady_s();
      cur.rc = sharded_is_allowed(t, &view, out + lo);
      cur.ms = (steady_s() - a) * 1e3;
      if (cur.rc) cur.err = g_err;
    });
    if (st) {
      st->chunks += 1;
      st->upload_bytes += (double)(cur.n * sizeof(ReqLine) + view.ext_words * 4 + view.arena_words * 4) *
                          (1 + t->peers.size());
    }
  }
  return finish(cur);
}

extern "C" {

int acs_pipeline_is_allowed(acs_pipeline* p, const char* json, size_t len, acs_decision* out, size_t out_cap,
                            size_t* n_out, acs_pipeline_stats* st) {
  if (!p || (!json && len) || !n_out) return fail("acs_pipeline_is_allowed: null argument");
  std::lock_guard<std::mutex> lock(p->mu);
  pipeline_reset(p);  // nothing of an earlier (failed) run may retire into this one's `out`
  if (st) *st = acs_pipeline_stats{};
  p->reasons.clear();
  const double t0 = steady_s();
  size_t n = 0;
  acs_internal_items* items = acs_internal_split(json, len, p->threads, &n);
  if (!items) return -1;
  if (st) st->split_s = steady_s() - t0;
  *n_out = n;
  struct Free {
    acs_internal_items* it;
    ~Free() { acs_internal_items_free(it); }
  } free_items{items};
  if (n > out_cap || (n && !out)) return fail("acs_pipeline_is_allowed: output holds fewer records than the requests");
  if (p->t->sharded) {
    if (pipeline_sharded(p, items, n, out, st)) return -1;
    if (st) {
      st->requests = n;
      st->host_requests = p->reasons.size();
      st->total_s = steady_s() - t0;
    }
    return 0;
  }
  // any failure once a chunk is in flight: drain every slot (pipeline_reset) before returning
  auto bail = [&] {
    pipeline_reset(p);
    return -1;
  };
#define PIPE_HIP(expr)                                                              \
  do {                                                                              \
    hipError_t e_ = (expr);                                                         \
    if (e_ != hipSuccess) return fail(std::string(#expr ": ") + hipGetErrorString(e_)), bail(); \
  } while (0)
  const size_t D = p->slot.size() / 2;
  size_t k = 0;
  for (size_t lo = 0; lo < n; lo += p->chunk, ++k) {
    const size_t hi = lo + p->chunk < n ? lo + p->chunk : n;
    const double e0 = steady_s();
    acs_codec_batch* b = acs_internal_encode_range(p->c, items, lo, hi, p->threads);
    if (!b) return bail();
    if (st) st->encode_s += steady_s() - e0;
    acs_pipeline::Slot& S = p->slot[2 * (k % D) + (k / D) % 2];
    if (pipeline_retire(p, S, out, st)) {  // this slot's previous chunk
      acs_codec_batch_free(b);
      return bail();
    }
    S.batch = b;  // owned by the slot from here on (pipeline_reset frees it on a failure)
    S.lo = lo;
    S.n = hi - lo;
    acs_tables* T = S.T;
    acs_req_batch view;
    const double c0 = steady_s();
    if (acs_codec_batch_view(b, &view) || check_batch(T, &view)) return bail();
    if (st) st->check_s += steady_s() - c0;
    PIPE_HIP(hipSetDevice(T->device));
    if (S.stage_n < S.n) {
      if (S.stage) PIPE_HIP(hipHostFree(S.stage));
      S.stage = nullptr;
      S.stage_n = 0;
      PIPE_HIP(hipHostMalloc((void**)&S.stage, S.n * sizeof(acs_decision), hipHostMallocPortable));
      S.stage_n = S.n;
    }
    {
      std::lock_guard<std::mutex> tl(T->mu);  // the device handle's launch bookkeeping
      acs_req_batch d;
      S.busy = true;  // work may be queued from here on: a failure waits for it
      PIPE_HIP(hipEventRecord(S.ev0, S.stream));
      if (upload_batch(S.ws, &view, &d, S.stream)) return bail();
      if (S.ws.out.reserve(S.n * sizeof(Decision))) return bail();
      if (is_allowed_launch(T, S.ws, &d, (acs_decision*)S.ws.out.p, S.stream)) return bail();
      PIPE_HIP(hipMemcpyAsync(S.stage, S.ws.out.p, S.n * sizeof(Decision), hipMemcpyDeviceToHost, S.stream));
      PIPE_HIP(hipEventRecord(S.ev1, S.stream));
      PIPE_HIP(hipEventRecord(S.done, S.stream));
    }
    if (st) {
      st->chunks += 1;
      st->upload_bytes += (double)(S.n * sizeof(ReqLine) + view.ext_words * 4 + view.arena_words * 4 +
                                   (size_t)view.rx_cols * view.rx_rows +
                                   (size_t)view.cand_rows * view.cand_words * 4 +
                                   (view.perm ? view.perm_lanes * 4 : 0));
    }
  }
  for (auto& S : p->slot)
    if (pipeline_retire(p, S, out, st)) return bail();
#undef PIPE_HIP
  HIP_OK(hipSetDevice(p->t->device));
  if (st) {
    st->requests = n;
    st->host_requests = p->reasons.size();
    st->total_s = steady_s() - t0;
  }
  return 0;
}

const char* acs_pipeline_host_reason(acs_pipeline* p, size_t i) {
  if (!p) return nullptr;
  auto it = p->reasons.find(i);
  return it == p->reasons.end() ? nullptr : it->second.c_str();
}

}  // extern "C"
