// acs_eval.h — per-request decision core of the MI355X access-control evaluator.
//
// One call evaluates one request against the whole compiled store in the
// reference's order (sets -> policies -> rules, Map order), so decisions,
// evaluation_cacheable, whatIsAllowed inclusion bits and the maskedProperty
// push log are bit-identical to the TypeScript PDP.  The GPU kernels
// (acs_kernels.hip) run it one request per lane over requests sorted so that a
// wave shares its entity/role/action: node records are read through
// wave-uniform addresses (scalar loads of one 64-B record per set/policy/rule),
// the request's resource attributes live in registers (RQ template).
//
// Reference semantics restated (paths in restorecommerce/access-control-srv):
//   isAllowed                 src/core/accessController.ts:88-324
//   whatIsAllowed             src/core/accessController.ts:326-427
//   checkMultipleEntities     src/core/accessController.ts:429-463
//   resourceAttributesMatch   src/core/accessController.ts:465-654
//   targetMatches             src/core/accessController.ts:661-672
//   attributesMatch           src/core/accessController.ts:681-699
//   checkSubjectMatches       src/core/accessController.ts:793-823
//   decide + CAs              src/core/accessController.ts:832-893
//   checkHierarchicalScope    src/core/hierarchicalScope.ts:10-259
//   verifyACLList             src/core/verifyACL.ts:11-251
#pragma once
#include <hip/hip_runtime.h>

#include "acs_layout.h"

namespace acs {

#define ACS_FN __host__ __device__ inline

// A composed lane reads its second class row's verdict only for targets that test role
// associations (same-call A/B, r05_c: c3 K1 3.29 -> 3.17 ms, c4 K2 8.27 -> 7.96 ms).
// ACS_OWN_SKIP (bits): the skips K1's SK instantiation takes for waves that mix classes — lanes
// leave the rules (1), loop-2b policies (2), sets (4) outside their own filter rows.  In the plain
// instantiation the same skips cut rule target matches per wave (c3: 2.52 -> 0.98, r05_b op counts)
// but were slower on long class runs (c3 3.17 -> 3.35 ms, c3r1 1.86 -> 2.09: the per-lane row loads
// and their registers, r05_c).  Rejected forms (removed): clean sets below the deciding
// set dropped from the event index's bits (c3 3.16 -> 3.29 ms, r05_c) or a word at a time once the
// whole wave is below it (c3adv 1.794 vs 1.756 ms, r05_n; a parity bug in its first form, r05_m),
// and K2 lanes skipping the rules outside their own rows.
#ifndef ACS_OWN_SKIP
#define ACS_OWN_SKIP 7
#endif

// Value every active lane of the wave holds identically (a table index or bitset word of
// the wave-shared candidate iteration): move it to an SGPR so the node records behind it
// are fetched with scalar loads.  Identity in the host build of the core.
ACS_FN uint32_t wave_uniform(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_readfirstlane(x);
#else
  return x;
#endif
}

// Phase profiling (tools/phase_prof.py; a separate -DACS_PHASE_PROF build only): per-lane
// cycle counters of the evaluation phases, summed per wave by the kernel.
enum ProfPhase { PH_TOTAL, PH_SET_TARGET, PH_POL_EXACT, PH_MULTI, PH_POL_TARGET, PH_RULE_TARGET, PH_RULE_HR,
                 PH_RULE_ACL, PH_N };
#if defined(ACS_PHASE_PROF)
#define PROF_T0(v) const uint64_t v = __builtin_readcyclecounter()
#define PROF_ADD(k, v) (R.prof[k] += __builtin_readcyclecounter() - (v))
#else
#define PROF_T0(v)
#define PROF_ADD(k, v)
#endif

// Operation counting (tools/op_count.py; a separate -DACS_OP_COUNT build only): how many times
// the waves execute each evaluation step (once per wave that runs it) and how many lanes are
// active when they do — the per-wave attribution of K1's instruction and load counts.
enum OpCount {
  OP_SET_ITER, OP_SET_SKIP, OP_SET_EVAL, OP_SET_EVENTS, OP_SET_TARGET, OP_P2A_ITER, OP_P2A_TM, OP_MULTI,
  OP_P2B_ITER, OP_P2B_TM, OP_P2B_HR, OP_RULE_LOOP, OP_RULE_ITER, OP_RULE_TM, OP_RULE_HR, OP_RULE_ACL,
  OP_WORD, OP_V_LDS, OP_V_OWN, OP_V_OWN2, OP_ROWS, OP_ROWS2, OP_LANE_DONE,
  OP_TPL_REQ, OP_TPL_WORD, OP_TPL_RULE, OP_TPL_TM, OP_TPL_HIT, OP_N
};
#if defined(ACS_OP_COUNT)
__device__ unsigned long long acs_op_wave[OP_N], acs_op_lane[OP_N];
#endif
#if defined(ACS_OP_COUNT) && defined(__HIP_DEVICE_COMPILE__)
__device__ inline void op_count(int k) {
  const uint64_t m = __ballot(1);
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if (lane == (uint32_t)__builtin_ctzll(m)) {
    atomicAdd(&acs_op_wave[k], 1ull);
    atomicAdd(&acs_op_lane[k], (unsigned long long)__builtin_popcountll(m));
  }
}
#define ACS_OPC(k) op_count(k)
#else
#define ACS_OPC(k)
#endif

// Cost probes (timing-only A/B builds, records unchanged): ACS_AB_PROBE_HR2 / ACS_AB_PROBE_TM2
// evaluate a rule's checkHierarchicalScope / target match a second time on an opaque copy of its
// record and keep the first result, so the difference to the product's time is one more check of
// that kind per call.  acs_opaque0(): a zero the compiler cannot see through.
#ifndef ACS_AB_PROBE_HR2
#define ACS_AB_PROBE_HR2 0
#endif
#ifndef ACS_AB_PROBE_TM2
#define ACS_AB_PROBE_TM2 0
#endif
#ifndef ACS_AB_PROBE_NR2
#define ACS_AB_PROBE_NR2 0
#endif
ACS_FN uint32_t acs_opaque0() {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t z;
  asm volatile("s_mov_b32 %0, 0" : "=s"(z));
  return z;
#else
  return 0u;
#endif
}

// regex matrix cell bits (rule entity value row x request entity value column)
enum RxBits : uint8_t { RX_HIT = 1, RX_RESET = 2, RX_THROW_TYPE = 4, RX_THROW_SYNTAX = 8, RX_HOST = 16 };

struct Tables {
  const NodeRec* sets;
  const NodeRec* pols;
  const NodeRec* rules;
  const RuleResAttr* rres;
  const Pair* pairs;
  const uint32_t* u32pool;
  uint32_t n_sets, n_pols, n_rules;
  uint32_t id_user;  // interned urns.user
  uint32_t rstride;  // NodeRec slots per rule record: 1 (blob layout), 2 (device rule lines, acs_compile)
  const uint32_t* ev_index;  // event index (build_event_index; nullptr: K1 never skips a set for it)
  const uint32_t* parents;   // [P] set of each policy, then [R] policy of each rule (build_parents;
                             // nullptr: no whatIsAllowed templates)
};

// The parent of every policy (its set) and rule (its policy), then two rule bitsets: non-null
// rules and rules with a target, then four policy bitsets: null, with a target, with a target
// testing role associations, truthy effect (the whatIsAllowed template pass decides a set's
// policies and a policy's rules a word at a time from them, without reading every record):
// parent_index_words(P, R) words.
inline size_t parent_index_words(uint32_t n_pols, uint32_t n_rules) {
  return (size_t)n_pols + n_rules + 2 * (((size_t)n_rules + 31) / 32) + 4 * (((size_t)n_pols + 31) / 32);
}
// rules: the blob's 64-B rule records
inline void build_parents(const NodeRec* sets, uint32_t n_sets, const NodeRec* pols, uint32_t n_pols,
                          const NodeRec* rules, uint32_t n_rules, uint32_t* out) {
  for (size_t k = 0; k < parent_index_words(n_pols, n_rules); ++k) out[k] = 0;
  for (uint32_t s = 0; s < n_sets; ++s)
    for (uint32_t p = sets[s].child_begin; p < sets[s].child_end && p < n_pols; ++p) out[p] = s;
  for (uint32_t p = 0; p < n_pols; ++p)
    for (uint32_t r = pols[p].child_begin; r < pols[p].child_end && r < n_rules; ++r) out[n_pols + r] = p;
  uint32_t* live = out + (size_t)n_pols + n_rules;
  uint32_t* tgt = live + (n_rules + 31) / 32;
  for (uint32_t r = 0; r < n_rules; ++r) {
    if (!(rules[r].nflags & NF_NULL)) live[r >> 5] |= 1u << (r & 31);
    if (rules[r].nflags & NF_HAS_TARGET) tgt[r >> 5] |= 1u << (r & 31);
  }
  const uint32_t PW = (n_pols + 31) / 32;
  uint32_t* pb = tgt + (n_rules + 31) / 32;
  for (uint32_t p = 0; p < n_pols; ++p) {
    const uint32_t bit = 1u << (p & 31), w = p >> 5;
    if (pols[p].nflags & NF_NULL) pb[w] |= bit;
    if (pols[p].nflags & NF_HAS_TARGET) pb[PW + w] |= bit;
    if ((pols[p].nflags & NF_HAS_TARGET) && (pols[p].tflags & TF_SUBJ_ROLE)) pb[2 * PW + w] |= bit;
    if (pols[p].nflags & NF_EFFECT_TRUTHY) pb[3 * PW + w] |= bit;
  }
}
ACS_FN const uint32_t* rule_live_bits(const Tables& T) { return T.parents + (size_t)T.n_pols + T.n_rules; }
ACS_FN const uint32_t* rule_target_bits(const Tables& T) { return rule_live_bits(T) + (T.n_rules + 31u) / 32u; }
// policy bitset k (0 null, 1 with a target, 2 role-testing target, 3 truthy effect)
ACS_FN const uint32_t* policy_bits(const Tables& T, uint32_t k) {
  return rule_target_bits(T) + (T.n_rules + 31u) / 32u + k * ((T.n_pols + 31u) / 32u);
}

// K1's event index (is_allowed_body's events-only skip): per set its rules' range [r0, r1) and,
// in bit 31 of the r1 word, whether it holds a null policy or a policy with an invalid combining
// algorithm (events that need no rule), in bit 30 whether every policy of it has rules and is
// ACL-gated (below); then one bit per rule carrying a condition; then one bit
// per policy whose every non-null rule has a target and does not skip ACLs (ACL-gated: for an
// ACL_NONE request none of its rules can push).
// Last, one bit per set that is clean (NF_CLEAN): below the deciding set the walk skips those
// without loading their records.
// event_index_words(n_sets, n_pols, n_rules) u32 words, built on the host from the blob's records.
inline size_t event_index_words(uint32_t n_sets, uint32_t n_pols, uint32_t n_rules) {
  return 2 * (size_t)n_sets + ((size_t)n_rules + 31) / 32 + ((size_t)n_pols + 31) / 32 + ((size_t)n_sets + 31) / 32;
}
ACS_FN size_t event_index_clean_off(uint32_t n_sets, uint32_t n_pols, uint32_t n_rules) {
  return 2 * (size_t)n_sets + ((size_t)n_rules + 31) / 32 + ((size_t)n_pols + 31) / 32;
}
inline void build_event_index(const NodeRec* sets, uint32_t n_sets, const NodeRec* pols, uint32_t n_pols,
                              const NodeRec* rules, uint32_t n_rules, uint32_t* out) {
  for (uint32_t s = 0; s < n_sets; ++s) {
    const NodeRec& S = sets[s];
    uint32_t r0 = 0xFFFFFFFFu, r1 = 0;
    bool bare = false;  // an event source without any rule
    for (uint32_t p = S.child_begin; p < S.child_end && p < n_pols; ++p) {
      const NodeRec& P = pols[p];
      if ((P.nflags & NF_NULL) || P.ca == CA_INVALID) bare = true;
      if (P.child_end > P.child_begin) {
        r0 = P.child_begin < r0 ? P.child_begin : r0;
        r1 = P.child_end > r1 ? P.child_end : r1;
      }
    }
    if (r0 >= r1) r0 = r1 = 0;
    out[2 * s] = r0;
    out[2 * s + 1] = (r1 & 0x3FFFFFFFu) | (bare ? 0x80000000u : 0u);
  }
  uint32_t* cb = out + 2 * (size_t)n_sets;
  for (uint32_t w = 0; w < (n_rules + 31) / 32; ++w) cb[w] = 0;
  for (uint32_t r = 0; r < n_rules; ++r)
    if (rules[r].nflags & NF_HAS_CONDITION) cb[r >> 5] |= 1u << (r & 31);
  uint32_t* gb = cb + (n_rules + 31) / 32;
  for (uint32_t w = 0; w < (n_pols + 31) / 32; ++w) gb[w] = 0;
  for (uint32_t p = 0; p < n_pols; ++p) {
    bool gated = true;
    for (uint32_t r = pols[p].child_begin; r < pols[p].child_end && r < n_rules && gated; ++r) {
      const NodeRec& Q = rules[r];
      if (Q.nflags & NF_NULL) continue;
      gated = (Q.nflags & NF_HAS_TARGET) && !(Q.tflags & TF_ACL_SKIP);
    }
    if (gated) gb[p >> 5] |= 1u << (p & 31);
  }
  for (uint32_t s = 0; s < n_sets; ++s) {  // bit 30: every policy has rules and is ACL-gated
    bool inert = true;
    for (uint32_t p = sets[s].child_begin; p < sets[s].child_end && p < n_pols && inert; ++p)
      inert = !(pols[p].nflags & NF_NULL) && pols[p].map_size != 0 && ((gb[p >> 5] >> (p & 31)) & 1u);
    if (inert) out[2 * s + 1] |= 0x40000000u;
  }
  uint32_t* clean = out + event_index_clean_off(n_sets, n_pols, n_rules);
  for (uint32_t w = 0; w < (n_sets + 31) / 32; ++w) clean[w] = 0;
  for (uint32_t s = 0; s < n_sets; ++s)
    if (sets[s].nflags & NF_CLEAN) clean[s >> 5] |= 1u << (s & 31);
}

// Set s cannot push for an ACL_NONE request: every policy of it has rules and is ACL-gated.
ACS_FN bool set_acl_inert(const Tables& T, uint32_t s) {
  return T.ev_index && ((T.ev_index[2 * s + 1] >> 30) & 1u);
}

// Policy p's rules can all be vetoed by verifyACL (event index, above).
ACS_FN bool acl_gated(const Tables& T, uint32_t p) {
  if (!T.ev_index) return false;
  const uint32_t* gb = T.ev_index + 2 * (size_t)T.n_sets + (T.n_rules + 31) / 32;
  return (gb[p >> 5] >> (p & 31)) & 1u;
}

#if defined(ACS_SCAN_COUNT)
// Counting build (bench.py's B_scan): bytes of every table read a wave issues, once per wave.
__device__ unsigned long long acs_scan_bytes;
#endif
#if defined(ACS_SCAN_COUNT) && defined(__HIP_DEVICE_COMPILE__)
__device__ inline void scan_count(uint32_t bytes) {
  const uint32_t lane = __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u));
  if (lane == (uint32_t)__builtin_ctzll(__ballot(1))) atomicAdd(&acs_scan_bytes, (unsigned long long)bytes);
}
#define ACS_SCAN(bytes) scan_count(bytes)
#elif defined(ACS_HOST_WORK) && !defined(__HIP_DEVICE_COMPILE__)
// Work-counting host build (tools/lane_work.py, test infrastructure): table bytes one request reads
extern thread_local unsigned long long acs_host_work;
#define ACS_SCAN(bytes) (acs_host_work += (bytes))
#else
#define ACS_SCAN(bytes)
#endif

// Table records are read as whole dwords through wave-uniform addresses and unpacked in
// registers.  Vector loads (exec-masked, so a block entered with no active lane loads
// nothing), then the wave-uniform record moves to SGPRs: its fields feed scalar compares and
// branches and free VGPRs (K1 VGPR spills 45 -> 1; A/B c3 +5 %).  Where the compiler itself
// proves the address uniform it emits s_load; nothing here forces a scalar load.  Rejected
// forms (A/B): one-lane vector loads (c3 K1 1.891 vs 1.851 ms, r03_g); plain s_load
// (a scalar load ignores EXEC, so in a region no lane entered it reads a stale address: faulted on
// c4, r03); scalar buffer loads clamped into the image (safe; c3 10M 2.978 vs 2.929 ms, c5 3.26 vs
// 3.08, c4 K2 3.89 vs 4.00, r06_a).
template <class X, int NW = sizeof(X) / 4>
ACS_FN X load_words(const Tables& T, const X* p) {
  static_assert(sizeof(X) == 4 * NW && sizeof(X) <= 64, "record must be whole dwords, at most 64 B");
  (void)T;
  ACS_SCAN(sizeof(X));
  const uint32_t* w = reinterpret_cast<const uint32_t*>(p);
  uint32_t v[NW];
#if defined(__HIP_DEVICE_COMPILE__)
#pragma unroll
  for (int k = 0; k < NW; ++k) v[k] = __builtin_amdgcn_readfirstlane(w[k]);
#else
#pragma unroll
  for (int k = 0; k < NW; ++k) v[k] = w[k];
#endif
  X out;
  __builtin_memcpy(&out, v, sizeof(X));
  return out;
}

// Node record `x` of a table section of `n` records.  (ACS_AB_PROBE_NR2, timing probe: every
// record read a second time after the first, through an opaque zero offset — the cost of one more
// dependent record round trip per node visit.)
ACS_FN NodeRec node_at(const Tables& T, const NodeRec* sec, uint32_t x, uint32_t n) {
  (void)n;
#if ACS_AB_PROBE_NR2
  NodeRec a = load_words(T, sec + x);  // the second read depends on the first: one more round trip
  const NodeRec b = load_words(T, sec + x + (a.child_end & acs_opaque0()));
  a.child_begin = b.child_begin == a.child_begin ? a.child_begin : b.child_begin;
  return a;
#else
  return load_words(T, sec + x);
#endif
}

// Rule r.  The device image stores each rule in a 128-B line (record + inline attributes).
ACS_FN NodeRec rule_at(const Tables& T, uint32_t r) {
  return node_at(T, T.rules, r * T.rstride, T.n_rules * T.rstride);
}

struct Batch {
  uint32_t n;
  const ReqHdr* hdr;      // [n]
  const ReqRes* res;      // [QMAX][n]
  const Pair* subj;       // [SMAX][n]
  const Pair* act;        // [AMAX][n]
  const uint32_t* roles;  // [RMAX][n]
  const uint32_t* arena;
  const uint8_t* rx;      // [cols][rx_rows]
  uint32_t rx_rows;
  const uint32_t* cand;   // [cand_rows][cand_words] candidate bitsets (sets | policies | rules) per class
  uint32_t cand_words, cand_wp, cand_wr;  // row length, word offsets of the policy / rule sections
  uint32_t cand_rows;     // number of request classes (class ids >= cand_rows: unfiltered)
  uint32_t cand_wsu, cand_wpu;  // isAllowed's useful sets / policies sections (0: absent)
  uint32_t cand_wv;             // target-verdict sections (0: absent)
  uint32_t no_verdicts;         // A/B runs (ACS_NO_VERDICTS=1): K1 ignores the verdicts
  uint32_t lds_pref;            // long rows (> LDS row capacity): words of the wave's LDS union prefix
  uint32_t role_major;          // coherence sort key [role key | class] instead of [class | role key]
  uint32_t no_cut;              // A/B runs (ACS_NO_CUT=1): combining loops always run to the end
  const uint32_t* role_key;   // [n] role-factor row per request (nullptr: no role factor)
  const uint32_t* role_bits;  // [role_rows][cand_words]
  uint32_t role_rows;
  const ReqLine* lines;       // [n] packed first rows (nullptr: read the SoA rows)
  const uint32_t* ext;        // compact batches (hdr == nullptr): extension records (ReqLine.ext)
};

// The second class row of request i (ReqLine.cls2, composed class rows) or nullptr.  A cls2
// outside the batch's rows leaves the request unfiltered (*bad), never narrower.
ACS_FN const uint32_t* second_row(const Batch& B, uint32_t i, bool* bad) {
  *bad = false;
  if (!B.lines || !B.cand) return nullptr;
  const uint32_t c2 = B.lines[i].cls2;
  if (!c2) return nullptr;
  if (c2 - 1u >= B.cand_rows) {
    *bad = true;
    return nullptr;
  }
  return B.cand + (size_t)(c2 - 1u) * B.cand_words;
}

// The role-factor rows of a request's role key (role_key: row | (1 + second row) << 16; a
// request with two required roles ORs its two rows).  Both nullptr: no role filtering (no
// factor, or a key outside the rows — never narrower).
ACS_FN void role_rows_of(const Batch& B, uint32_t rk, const uint32_t** r1, const uint32_t** r2) {
  *r1 = *r2 = nullptr;
  if (!B.role_key) return;
  const uint32_t a = rk & 0xFFFFu, b = rk >> 16;
  if (a >= B.role_rows || (b && b - 1u >= B.role_rows)) return;
  *r1 = B.role_bits + (size_t)a * B.cand_words;
  if (b) *r2 = B.role_bits + (size_t)(b - 1u) * B.cand_words;
}

// word w of the OR of a request's role rows (all ones: no role filtering)
ACS_FN uint32_t role_word(const uint32_t* r1, const uint32_t* r2, uint32_t w) {
  return r1 ? (r2 ? r1[w] | r2[w] : r1[w]) : ~0u;
}

// Target-verdict word of a lane with one or two class rows: a known-true section (exact /
// RegExp true, rules retried true) is true when either row knows it (the composed request holds
// both role sets); a known-false section (`conj`) only when both do.
ACS_FN uint32_t compose_verdict(uint32_t a, const uint32_t* row2, uint32_t at, bool conj) {
  if (!row2) return a;
  return conj ? a & row2[at] : a | row2[at];
}

// OR of x over the wave's ACTIVE lanes, returned in an SGPR.  A lane drops out once its bits
// are covered, so the loop runs once per lane that still adds bits (lanes sharing a row
// share the value: a few rounds).  Host build: x itself (one request).
ACS_FN uint32_t wave_or(uint32_t x) {
#if defined(__HIP_DEVICE_COMPILE__)
  uint32_t acc = 0;
  uint64_t pend = __ballot(x != 0u);
  while (pend) {
    acc |= __builtin_amdgcn_readlane(x, __builtin_ctzll(pend));
    pend &= ~__ballot((x & ~acc) == 0u);
  }
  return acc;
#else
  return x;
#endif
}

// Whether b holds on every ACTIVE lane of the wave.  Host build: b (one request).
ACS_FN bool wave_all(bool b) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __ballot(!b) == 0;
#else
  return b;
#endif
}

// General candidate filter (rows longer than the LDS row form takes, and the host build).
// Each lane holds pointers to its own request's rows.  GPU: words below lds_n come from the
// wave's OR row in LDS (built before any lane diverges); a later word is the OR of the
// ACTIVE lanes' own words — the lanes still inside the loop that asks for it, which is all
// the iteration needs (lanes that returned or skipped the enclosing policy read nothing).
struct Filter {
  const uint32_t* row;     // this request's class row
  const uint32_t* row2;    // its second class row (composed rows; nullptr: none)
  const uint32_t* rrow;    // its role-factor row (nullptr: no role filtering)
  const uint32_t* rrow2;   // its second role-factor row (two required roles; nullptr: none)
  const uint32_t* lds;     // GPU: the wave's OR of its (class & role) rows, words [0, lds_n)
  uint32_t lds_n;
  uint32_t wp, wr;         // word offsets of the policy / rule sections
  uint32_t wsu, wpu;       // isAllowed: useful sets / loop-2b policies (0 / wp without them)
  uint32_t wv;             // target-verdict sections (candidates.verdict_offset)
  bool vok;                // the verdicts apply: the rows are this request's own class rows
  bool all;                // no filtering
  // word w of the verdict section at word `sec` past wv (0 when the verdicts do not apply);
  // conj: a known-false section (AND over the request's rows); roles: the node's target tests
  // role associations (TF_SUBJ_ROLE) — else both class rows of a composed request hold the same
  // verdict (they differ only in the role) and the second is not read
  ACS_FN uint32_t vword(uint32_t sec, uint32_t w, bool conj = false, bool roles = true) const {
    return vok ? compose_verdict(row[wv + sec + w], roles ? row2 : nullptr, wv + sec + w, conj)
               : 0u;
  }
  ACS_FN bool verdict(uint32_t sec, uint32_t i, bool conj = false, bool roles = true) const {
    return (vword(sec, i >> 5, conj, roles) >> (i & 31)) & 1u;
  }
  // word w of THIS lane's own row (class | second class, & role rows): the nodes its target
  // filter keeps (a node outside it is inert for the lane)
  ACS_FN uint32_t own_word(uint32_t w) const {
    if (all) return ~0u;
    uint32_t x = row[w];
    if (row2) x |= row2[w];
    if (rrow) x &= role_word(rrow, rrow2, w);
    return x;
  }
  ACS_FN uint32_t word(uint32_t w) const {
    if (all) return ~0u;
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(3))) const uint32_t lds_u32;
    if (w < lds_n) return wave_uniform(((lds_u32*)lds)[w]);
#endif
    ACS_SCAN(8);  // a word of the lanes' class and role rows (counted once per wave)
    ACS_OPC(OP_WORD);
    uint32_t x = row[w];
    if (row2) x |= row2[w];
    if (rrow) x &= role_word(rrow, rrow2, w);
    return wave_or(x);
  }
};

// The filter forms the GPU kernels are instantiated with (the evaluation core takes any
// type with wp, wr and word(w)); each keeps only the state its form reads, so the wave's
// long-lived scalar state stays small.
// FilterAll: the batch carries no candidate rows — every node is a candidate.
struct FilterAll {
  uint32_t wp, wr, wsu, wpu;
  ACS_FN uint32_t word(uint32_t) const { return ~0u; }
  ACS_FN uint32_t own_word(uint32_t) const { return ~0u; }
  ACS_FN bool verdict(uint32_t, uint32_t, bool = false, bool = true) const { return false; }  // no class rows
  ACS_FN uint32_t vword(uint32_t, uint32_t, bool = false, bool = true) const { return 0u; }
};

// FilterLds: rows that fit in LDS — the wave's OR of its (class & role) rows, built by the
// kernel before any lane diverges (all ones for a wave holding an unfiltered request).  The
// target verdicts are class facts: a wave of one class reads them from its LDS row (`single`:
// there the verdict sections are that class's alone), a composed lane composing them with its
// second row (`own2`); in a wave that mixes classes each lane reads its own class row (`own`,
// L2-resident; nullptr for an unfiltered lane: no verdicts) and a composed lane also `own2`.
// (c3: most waves hold composed lanes; reading the class's verdicts from LDS there instead of
// two L2 gathers per lookup: same-call A/B K1 3.125 -> 3.106 ms, r04_q.)
struct FilterLds {
  const uint32_t* lds;
  uint32_t wp, wr, wsu, wpu, wv;
  const uint32_t* own;
  const uint32_t* own2;
  bool single;
  bool ownc;  // own (| own2) is the lane's whole filter row (no role factor rows to AND)
  // word w of THIS lane's own row (a node outside it is inert for the lane); all ones when the
  // lane's row is not at hand
  ACS_FN uint32_t own_word(uint32_t w) const { return ownc ? own[w] | (own2 ? own2[w] : 0u) : ~0u; }
  ACS_FN uint32_t word(uint32_t w) const {
    ACS_OPC(OP_WORD);
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(3))) const uint32_t lds_u32;
    return wave_uniform(((lds_u32*)lds)[w]);
#else
    return lds[w];
#endif
  }
  // word w of the verdict section at `sec` (wave-uniform in a one-class wave, else per lane);
  // conj: a known-false section
  // roles: the node's target tests role associations (TF_SUBJ_ROLE); else a composed lane's two
  // class rows hold the same verdict (same entity column and action, another role) and the
  // second row is not read
  ACS_FN uint32_t vword(uint32_t sec, uint32_t w, bool conj = false, bool roles = true) const {
    const uint32_t* o2 = roles ? own2 : nullptr;
#if defined(ACS_OP_COUNT)
    ACS_OPC(single ? OP_V_LDS : OP_V_OWN);
    if (o2) ACS_OPC(OP_V_OWN2);
#endif
    if (single) return compose_verdict(word(wv + sec + w), o2, wv + sec + w, conj);
    return own ? compose_verdict(own[wv + sec + w], o2, wv + sec + w, conj) : 0u;
  }
  ACS_FN bool verdict(uint32_t sec, uint32_t i, bool conj = false, bool roles = true) const {
    return (vword(sec, i >> 5, conj, roles) >> (i & 31)) & 1u;
  }
};

// Ascending iteration over the candidate indices in [b, e) of one bitset section.  Every
// lane that is still inside the loop holds the same iterator state.
template <class FL>
struct CandRange {
  const FL& F;
  uint32_t off, base, e, bits;
  ACS_FN CandRange(const FL& f, uint32_t section_off, uint32_t b, uint32_t e_)
      : F(f), off(section_off), base(b & ~31u), e(e_), bits(0) {
    if (b < e) bits = F.word(off + (b >> 5)) & (~0u << (b & 31));
  }
  ACS_FN bool next(uint32_t& out) {
    for (;;) {
      if (bits) {
        const uint32_t x = wave_uniform(base + (uint32_t)__builtin_ctz(bits));
        bits &= bits - 1;
        if (x >= e) return false;
        out = x;
        return true;
      }
      base += 32;
      if (base >= e) return false;
      bits = F.word(off + (base >> 5));
    }
  }
};

// Descending iteration over the candidate indices in [b, e) of one bitset section.
template <class FL>
struct CandRangeRev {
  const FL& F;
  uint32_t off, b, lo, base, bits;  // lo: base of the word holding index b (the last word read)
  ACS_FN CandRangeRev(const FL& f, uint32_t section_off, uint32_t b_, uint32_t e)
      : F(f), off(section_off), b(b_), lo(b_ & ~31u), base(b_ & ~31u), bits(0) {
    if (b < e) {
      base = (e - 1) & ~31u;
      const uint32_t top = (e - 1) & 31u;
      bits = F.word(off + (base >> 5)) & (top == 31u ? ~0u : ((1u << (top + 1)) - 1u));
    }
  }
  ACS_FN bool next(uint32_t& out) {
    for (;;) {
      if (bits) {
        const uint32_t hi = 31u - (uint32_t)__builtin_clz(bits);
        const uint32_t x = wave_uniform(base + hi);
        bits &= ~(1u << hi);
        if (x < b) return false;
        out = x;
        return true;
      }
      if (base <= lo) return false;
      base -= 32;
      bits = F.word(off + (base >> 5));
    }
  }
};

ACS_FN bool loose_eq(uint32_t a, uint32_t b) { return a == b || (a <= ID_NULL && b <= ID_NULL); }

// Target verdicts, F.verdict(sec, i) (candidates.verdict_offset): bit i of the section at
// word `sec` past the verdict base — policies known exact-true (sec 0), exact-false (WP),
// RegExp-true (2 WP), RegExp-false (3 WP), rules whose retried match is known true (4 WP);
// WP = ceil(P / 32).  False wherever the class's verdicts do not apply.  The known-false
// sections (WP, 3 WP) are read with conj = true: a composed request (two class rows) knows a
// target false only when both of its rows do.

// tri-state result: 1 true, 0 false, <0 -ErrKind (the reference throws)
typedef int tri;

struct Fold {  // streaming decide(): first X else last / first element
  uint8_t ca, n, locked, eff, ec;
  ACS_FN explicit Fold(uint8_t ca_) : ca(ca_), n(0), locked(0), eff(EFF_UNDEF), ec(EC_UNDEF) {}
  ACS_FN void push(uint8_t e, uint8_t c) {
    if (ca == CA_FIRST_APPLICABLE) {
      if (!n) { eff = e; ec = c; }
    } else if (!locked) {
      eff = e;
      ec = c;
      if (e == (ca == CA_DENY_OVERRIDES ? EFF_DENY : EFF_PERMIT)) locked = 1;
    }
    n = 1;
  }
  // no later push can change eff / ec
  ACS_FN bool final() const {
    return n && ((ca != CA_DENY_OVERRIDES && ca != CA_PERMIT_OVERRIDES) || locked);
  }
};

struct OblLog {  // whatIsAllowed maskedProperty pushes, in evaluation order
  uint32_t* out;  // [cap][2] or nullptr
  uint32_t n;     // entries written (<= cap)
  bool overflow;  // a push found the log full
  uint32_t cap = OBL_MAX;
  uint32_t total = 0;  // every push, written or not (sizes the overflow pass)
};


// ------------------------------------------------------------------ request views
// Context arena + headers shared by both request views.
struct ReqCtx {
  const Tables& T;
  const Batch& B;
  uint32_t i;
  ReqHdr h;
  // The arena view is recomputed from two packed count words at each use (HR / ACL only)
  // instead of being held as six pointers and six counts: K1's per-lane state stays small.
  uint32_t c0, c1;  // arena counts: [0] grants | rolese<<8 | slots<<16 | roots<<24, [1] tse | hrkeys<<8
  uint32_t ext;     // compact batch: 1 + 16-B unit offset of the extension record (0: none)
  bool soa;         // the rows past the line are SoA rows (else the extension record); false as a
                    // constant in the compact-batch kernels, so their SoA paths compile away
  uint32_t s0i, s0v, s1i, s1v, a0i, a0v, role0, role1;
  mutable uint32_t hrd = 0;  // checkHierarchicalScope digest (hr_digest below; 0: none)
#if defined(ACS_PHASE_PROF)
  mutable uint64_t prof[PH_N] = {};
#endif

  // ln: the request's packed line (acs_layout.h ReqLine), nullptr: the SoA rows
  ACS_FN ReqCtx(const Tables& t, const Batch& b, uint32_t idx, const ReqHdr& hd, const ReqLine* ln = nullptr,
                bool soa_ok = true)
      : T(t), B(b), i(idx), h(hd) {
    soa = soa_ok && B.hdr != nullptr;
    if (ln || !soa_ok) {
      ext = ln->ext;
      s0i = ln->s0.id; s0v = ln->s0.value; s1i = ln->s1.id; s1v = ln->s1.value;
      a0i = ln->a0.id; a0v = ln->a0.value;
      role0 = ln->r0;
      role1 = ln->r1;
      c0 = ln->ar0;
      c1 = ln->ar1;
      return;
    }
    ext = 0;
    const uint32_t* a = B.arena + h.arena_off;
    c0 = a[0];
    c1 = a[1];
    const Pair s0 = h.nsubj > 0 ? B.subj[i] : Pair{};
    const Pair s1 = h.nsubj > 1 ? B.subj[(size_t)B.n + i] : Pair{};
    const Pair a0 = h.nact > 0 ? B.act[i] : Pair{};
    s0i = s0.id; s0v = s0.value; s1i = s1.id; s1v = s1.value; a0i = a0.id; a0v = a0.value;
    role0 = h.nroles > 0 ? B.roles[i] : 0u;
    role1 = h.nroles > 1 ? B.roles[(size_t)B.n + i] : 0u;
  }
  ACS_FN const uint32_t* ar() const { return B.arena + h.arena_off; }
  ACS_FN const uint32_t* ex() const { return B.ext + (size_t)(ext - 1u) * 4u; }
  ACS_FN uint32_t n_grants() const { return c0 & 0xFFu; }
  ACS_FN uint32_t n_rolese() const { return (c0 >> 8) & 0xFFu; }
  ACS_FN uint32_t n_slots() const { return (c0 >> 16) & 0xFFu; }
  ACS_FN uint32_t n_roots() const { return c0 >> 24; }
  ACS_FN uint32_t n_tse() const { return c1 & 0xFFu; }
  ACS_FN uint32_t n_hrkeys() const { return (c1 >> 8) & 0xFFu; }
  ACS_FN const uint32_t* grants() const { return ar() + 2; }
  ACS_FN const uint32_t* rolese() const { return grants() + 3 * n_grants(); }
  ACS_FN const uint32_t* roots() const { return rolese() + 2 * n_rolese(); }
  ACS_FN const uint32_t* hrkeys() const { return roots() + n_roots(); }
  ACS_FN const uint32_t* slotoff() const { return hrkeys() + n_hrkeys(); }
  ACS_FN const uint32_t* tse() const { return slotoff() + n_slots(); }
  // The first subject / action / role attributes live in registers: target matching reads
  // them for every visited node, and the rows are gathered in sort order (uncoalesced).
  // Rows past the line: the SoA rows, or a compact batch's extension record.
  ACS_FN ExtGeom geom() const { return ext_geom(h.nres, h.nsubj, h.nact, h.nroles); }
  ACS_FN ReqRes res_row(uint32_t j) const {
    if (soa) return B.res[(size_t)j * B.n + i];
    const uint32_t* w = ex() + 4u * (j - (uint32_t)LINE_RES);
    ReqRes q;
    __builtin_memcpy(&q, w, sizeof q);
    return q;
  }
  ACS_FN Pair subj(uint32_t j) const {
    if (j >= 2) {
      if (soa) return B.subj[(size_t)j * B.n + i];
      const uint32_t* w = ex() + geom().subj + 2u * (j - 2u);
      return Pair{w[0], w[1]};
    }
    Pair p;
    p.id = j == 0 ? s0i : s1i;  // value selects (no address taken: stays in registers)
    p.value = j == 0 ? s0v : s1v;
    return p;
  }
  ACS_FN Pair act(uint32_t j) const {
    if (j >= 1) {
      if (soa) return B.act[(size_t)j * B.n + i];
      const uint32_t* w = ex() + geom().act + 2u * (j - 1u);
      return Pair{w[0], w[1]};
    }
    Pair p;
    p.id = a0i;
    p.value = a0v;
    return p;
  }
  ACS_FN uint32_t role(uint32_t j) const {
    if (j < 2) return j == 0 ? role0 : role1;
    return soa ? B.roles[(size_t)j * B.n + i] : ex()[geom().roles + (j - 2u)];
  }
  ACS_FN uint8_t rx(uint32_t col, uint32_t row) const { return B.rx[(size_t)col * B.rx_rows + row]; }
  ACS_FN bool flag(uint32_t f) const { return (h.flags & f) != 0; }
};

// Resource attributes staged in LDS by the kernel (slots < LDS_SLOTS, column = lane,
// stride = block size): dynamic indexing without scratch, one ds_read_b128 per use.
// LDS_SLOTS = LINE_RES: the slots are exactly the line's attributes, and res_row serves only
// attributes past the line (a compact batch's extension record).  4 x 16 B x 256 lanes = 16 KB:
// with a c3 filter row (832 words x 4 waves, 13 KB) a block fits 5 times into the CU's 160 KB of
// LDS, for K1's 5 waves/SIMD (A/B r02_q: 6 slots 1.98, 4 slots 1.95, 4 slots + 5 waves 1.87 ms at
// c3; 8 slots: 3 blocks/CU, round-2 A/B 20.6 vs 17.6 ms with 6).
constexpr int LDS_SLOTS = LINE_RES;

// NS: the LDS slots the kernel staged (LDS_SLOTS; K2 also stages the first extension attribute)
template <int NS = LDS_SLOTS>
struct ReqLds : ReqCtx {
  static_assert(NS >= LINE_RES, "slots past the line come from the extension record");
  const ReqRes* col;  // this lane's LDS column
  uint32_t stride;
  uint32_t e0_val, e0_col;  // the request's only entity attribute (RQ_ENT_SHIFT field 1..6)
  ACS_FN ReqLds(const Tables& t, const Batch& b, uint32_t idx, const ReqHdr& hd, const ReqRes* c, uint32_t st,
                const ReqLine* ln = nullptr, bool soa_ok = true)
      : ReqCtx(t, b, idx, hd, ln, soa_ok), col(c), stride(st) {
    const uint32_t e = (h.flags >> RQ_ENT_SHIFT) & 7u;
    e0_val = e0_col = 0;
    if (e >= 1 && e <= 6) {
      const ReqRes q = res((int)e - 1);
      e0_val = q.value;
      e0_col = q.col;
    }
  }
  ACS_FN ReqRes res(int j) const {
#if defined(__HIP_DEVICE_COMPILE__)
    typedef __attribute__((address_space(3))) const ReqRes lds_res;  // ds_read, not flat
    if (j < NS) return ((lds_res*)col)[j * stride];
#else
    if (j < NS) return col[j * stride];
#endif
    return res_row((uint32_t)j);
  }
};
static_assert(LDS_SLOTS == LINE_RES, "the kernels stage exactly the request line's attributes in LDS");

// Resource attributes read from HBM on every use (host build of the core).
struct ReqMem : ReqCtx {
  uint32_t e0_val, e0_col;
  const ReqLine* line;  // compact batch: the request's line (nullptr: SoA rows)
  ACS_FN ReqMem(const Tables& t, const Batch& b, uint32_t idx, const ReqHdr& hd, const ReqLine* ln = nullptr)
      : ReqCtx(t, b, idx, hd, ln), line(ln) {
    const uint32_t e = (h.flags >> RQ_ENT_SHIFT) & 7u;
    e0_val = e0_col = 0;
    if (e >= 1 && e <= 6) {
      const ReqRes q = res((int)e - 1);
      e0_val = q.value;
      e0_col = q.col;
    }
  }
  ACS_FN ReqRes res(int j) const { return line && j < LINE_RES ? line->res[j] : res_row((uint32_t)j); }
};

// The request's header and (compact batches) its line.
ACS_FN const ReqLine* req_line(const Batch& B, uint32_t i) { return B.hdr ? nullptr : B.lines + i; }
ACS_FN ReqHdr req_hdr(const Batch& B, uint32_t i) { return B.hdr ? B.hdr[i] : B.lines[i].h; }

// ------------------------------------------------------------------ attributesMatch (loose ==)
ACS_FN bool attrs_match(const Pair* rule, uint32_t rn, const ReqCtx& R, bool subjects) {
  const uint32_t qn = subjects ? R.h.nsubj : R.h.nact;
  for (uint32_t k = 0; k < rn; ++k) {
    const Pair a = load_words(R.T, rule + wave_uniform(k));
    bool found = false;
    for (uint32_t j = 0; j < qn && !found; ++j) {
      const Pair q = subjects ? R.subj(j) : R.act(j);
      found = loose_eq(q.id, a.id) && loose_eq(q.value, a.value);
    }
    if (!found) return false;
  }
  return true;
}

// ------------------------------------------------------------------ checkSubjectMatches
// sp: the target's subject pairs (R.T.pairs + t.subj_off, or a staged copy)
ACS_FN bool subject_match_at(const NodeRec& t, const Pair* sp, const ReqCtx& R) {
  if (t.tflags & TF_SUBJ_EMPTY) return true;
  if (t.tflags & TF_SUBJ_ROLE) {
    if (!R.flag(RQ_RA_TRUTHY)) return false;
    for (uint32_t k = 0; k < R.h.nroles; ++k)
      if (R.role(k) == t.role) return true;
    return false;
  }
  return attrs_match(sp, t.subj_n, R, true);
}
ACS_FN bool subject_match(const NodeRec& t, const ReqCtx& R) { return subject_match_at(t, R.T.pairs + t.subj_off, R); }

// ------------------------------------------------------------------ resourceAttributesMatch
#ifndef ACS_RA_CACHE
#define ACS_RA_CACHE 2  // rule resource attributes held in registers per resource_match call (A/B: 2 >= 4 > 0)
#endif
// Request attrs [j0, j1) with requestPropertiesExist = rpe.  wia: 'whatIsAllowed' op.
// ra: the target's resource attributes (R.T.rres + t.res_off, or a staged copy)
template <class RQ>
ACS_FN tri resource_match_at(const NodeRec& t, const RuleResAttr* ra, const RQ& R, uint8_t effect, bool regex,
                             bool wia, int j0, int j1, bool rpe, OblLog* obl) {
  if (t.tflags & TF_RES_EMPTY) return 1;
  const uint32_t ent = (R.h.flags >> RQ_ENT_SHIFT) & 7u;
  if ((t.tflags & TF_RES_ENT_ONLY) && ent != 7u && j0 == 0 && j1 == (int)R.h.nres) {
    // Target without property / operation attributes and a request with at most one entity
    // attribute: every property / mask / skipDenyRule branch needs a rule property, so the
    // ordered double loop reduces to entityMatch over the rule's entity attributes (exact:
    // sticky equality; RegExp: reset / hit in order, throws first-come) — same result.
    if (ent == 0) return 0;
    bool em = false;
    for (uint32_t k = 0; k < t.res_n; ++k) {
      const RuleResAttr r = k < ACS_RA_CACHE ? load_words(R.T, ra + k) : load_words(R.T, ra + wave_uniform(k));
      if (!(r.kind & K_ENT)) continue;
      if (!regex) {
        if (R.e0_val == r.value) em = true;
      } else {
        const uint8_t c = R.rx(R.e0_col, r.row);
        if (c & RX_THROW_TYPE) return -(tri)ERR_TYPE;
        if (c & RX_THROW_SYNTAX) return -(tri)ERR_REGEX_SYNTAX;
        if (c & RX_HOST) return -(tri)ERR_REGEX_HOST;
        if (c & RX_RESET) em = false;
        if (c & RX_HIT) em = true;
      }
    }
    return em ? 1 : 0;
  }
  bool em = false, pm = false, rp = false, om = false, skip_deny = true;
  int ent_j = 0;
  uint32_t ent_val = 0;
  // The target's attributes are the same for every lane: the first ACS_RA_CACHE are loaded
  // once per call (all in flight together) instead of once per request attribute.
  RuleResAttr rc[ACS_RA_CACHE > 0 ? ACS_RA_CACHE : 1];
#pragma unroll
  for (int k = 0; k < ACS_RA_CACHE; ++k)
    if (k < (int)t.res_n) rc[k] = load_words(R.T, ra + k);
  for (int j = j0; j < j1; ++j) {
    const ReqRes q = R.res(j);
    pm = false;
    // one (request attr, rule attr) step of the ordered double loop; <0: the reference throws
    auto step = [&](const RuleResAttr& r, int jj) -> tri {
      if (r.kind & K_PROP) rp = true;
      if (!regex) {
        if ((q.kind & K_ENT) && (r.kind & K_ENT) && q.value == r.value) {
          em = true;
          ent_j = jj;
          ent_val = q.value;
        } else if ((q.kind & K_OP) && (r.kind & K_OP) && q.value == r.value) {
          om = true;
        } else if (em && (q.kind & K_PROP) && (r.kind & K_PROP)) {
          if ((q.contains >> ent_j) & 1u) {
            if (r.value == q.value) pm = true;
          } else if (effect == EFF_PERMIT) {
            pm = true;
          }
        }
      } else {
        if ((q.kind & K_ENT) && (r.kind & K_ENT)) {
          const uint8_t c = R.rx(q.col, r.row);
          if (c & RX_THROW_TYPE) return -(tri)ERR_TYPE;
          if (c & RX_THROW_SYNTAX) return -(tri)ERR_REGEX_SYNTAX;
          if (c & RX_HOST) return -(tri)ERR_REGEX_HOST;
          ent_val = q.value;
          if (c & RX_RESET) em = false;
          if (c & RX_HIT) em = true;
        } else if (em && (q.kind & K_PROP) && (r.kind & K_PROP)) {
          if (r.hash_sfx == q.hash_sfx) pm = true;
        }
      }
      return 0;
    };
#pragma unroll
    for (int k = 0; k < ACS_RA_CACHE; ++k) {
      if (k < (int)t.res_n) {
        const tri e = step(rc[k], j);
        if (e < 0) return e;
      }
    }
    for (uint32_t k = ACS_RA_CACHE; k < t.res_n; ++k) {
      const tri e = step(load_words(R.T, ra + wave_uniform(k)), j);
      if (e < 0) return e;
    }
    const bool scope = (q.kind & K_PROP) || !rpe;
    if (!wia) {
      if (effect == EFF_DENY && scope && em && rp && pm) skip_deny = false;
      if (effect == EFF_PERMIT && scope && em && rp && !pm) return 0;
    } else {
      // maskedProperty pushes (accessController.ts:592-640)
      const bool permit_mask = effect == EFF_PERMIT && scope && em && rp && !pm;
      if (permit_mask && !rpe) return 0;
      const bool deny_mask = effect == EFF_DENY && scope && em && rp && (pm || !rpe);
      if (permit_mask || deny_mask) {
        uint32_t mask;
        bool no_hash;
        if (rpe && q.value > ID_EMPTY) {  // truthy request property value
          mask = q.value;
          no_hash = !(q.kind & K_HAS_HASH);
        } else if (!rpe) {
          mask = t.last_prop_value;
          no_hash = (t.tflags & TF_LASTPROP_STR) && !(t.tflags & TF_LASTPROP_HASH);
        } else {
          mask = ID_UNDEF;
          no_hash = false;
        }
        if (!no_hash && obl) {
          obl->total++;
          if (obl->n < obl->cap) {
            if (obl->out) {
              obl->out[2 * obl->n] = ent_val;
              obl->out[2 * obl->n + 1] = mask;
            }
            obl->n++;
          } else {
            obl->overflow = true;
          }
        }
      }
    }
  }
  if (!wia && skip_deny && rp && rpe && effect == EFF_DENY && !pm) return 0;
  if (!em && !om) return 0;
  return 1;
}
template <class RQ>
ACS_FN tri resource_match(const NodeRec& t, const RQ& R, uint8_t effect, bool regex, bool wia, int j0, int j1,
                          bool rpe, OblLog* obl) {
  return resource_match_at(t, R.T.rres + t.res_off, R, effect, regex, wia, j0, j1, rpe, obl);
}

// ------------------------------------------------------------------ targetMatches
template <class RQ>
ACS_FN tri target_match(const NodeRec& t, const RQ& R, uint8_t effect, bool regex, bool wia, OblLog* obl) {
  if (R.flag(RQ_NO_TARGET)) return -(tri)ERR_TYPE;  // requestTarget.subjects of undefined
  if (!subject_match(t, R)) return 0;
  if (!attrs_match(R.T.pairs + t.act_off, t.act_n, R, false)) return 0;
  return resource_match(t, R, effect == EFF_UNDEF ? (uint8_t)EFF_PERMIT : effect, regex, wia, 0, R.h.nres,
                        R.flag(RQ_ANY_PROP), obl);
}

// Rule targets: the exact pass, then the RegExp retry (accessController.ts:214-219, 400-409).
// Subjects and actions do not depend on the mode, so when they fail both passes are false.
// (Rejected A/B, r06_c: both resource modes in one pass over the attribute pairs — the RegExp
// cells then read even when the exact pass matches — c3 10M K1 3.25 vs 2.93 ms, c3r1 0.452 vs
// 0.404, c3adv 1.96 vs 1.75.)
// sp / ap / ra: the target's subject pairs, action pairs and resource attributes
template <class RQ>
ACS_FN tri target_match_retry_at(const NodeRec& t, const Pair* sp, const Pair* ap, const RuleResAttr* ra, const RQ& R,
                                 uint8_t effect, bool wia, OblLog* obl) {
  if (R.flag(RQ_NO_TARGET)) return -(tri)ERR_TYPE;
  if (!subject_match_at(t, sp, R)) return 0;
  if (!attrs_match(ap, t.act_n, R, false)) return 0;
  const uint8_t eff = effect == EFF_UNDEF ? (uint8_t)EFF_PERMIT : effect;
  const tri m = resource_match_at(t, ra, R, eff, false, wia, 0, R.h.nres, R.flag(RQ_ANY_PROP), obl);
  if (m != 0) return m;
  return resource_match_at(t, ra, R, eff, true, wia, 0, R.h.nres, R.flag(RQ_ANY_PROP), obl);
}
template <class RQ>
ACS_FN tri target_match_retry(const NodeRec& t, const RQ& R, uint8_t effect, bool wia, OblLog* obl) {
  return target_match_retry_at(t, R.T.pairs + t.subj_off, R.T.pairs + t.act_off, R.T.rres + t.res_off, R, effect, wia,
                               obl);
}

// ------------------------------------------------------------------ checkHierarchicalScope
ACS_FN const uint32_t* slot_rec(const ReqCtx& R, uint32_t slot) { return R.ar() + R.slotoff()[slot]; }

ACS_FN bool hr_direct(const ReqCtx& R, uint32_t slot, uint32_t role, uint32_t se) {
  const uint32_t* rec = slot_rec(R, slot);
  const uint32_t n_owners = rec[1];
  const uint32_t* p = rec + 2;
  for (uint32_t o = 0; o < n_owners; ++o) {
    const uint32_t w = p[0], val = p[1], na = w >> 8;
    const uint32_t* at = p + 2;
    if ((w & 1u) && val == se) {
      for (uint32_t g = 0; g < R.n_grants(); ++g) {
        const uint32_t* gr = R.grants() + 3 * g;
        if (gr[0] == role && gr[1] == se)
          for (uint32_t a = 0; a < na; ++a)
            if (at[3 * a] == gr[2]) return true;
      }
    }
    p = at + 3 * na;
  }
  return false;
}

ACS_FN bool hr_tree(const ReqCtx& R, uint32_t slot, uint32_t role, uint32_t se) {
  bool rse = false;
  for (uint32_t k = 0; k < R.n_rolese() && !rse; ++k) rse = R.rolese()[2 * k] == role && R.rolese()[2 * k + 1] == se;
  if (!rse) return false;
  uint32_t mask = 0;
  for (uint32_t r = 0; r < R.n_roots(); ++r)
    if (R.roots()[r] == role) mask |= 1u << r;
  if (!mask) return false;
  const uint32_t* rec = slot_rec(R, slot);
  const uint32_t n_owners = rec[1];
  const uint32_t* p = rec + 2;
  for (uint32_t o = 0; o < n_owners; ++o) {
    const uint32_t w = p[0], val = p[1], na = w >> 8;
    const uint32_t* at = p + 2;
    if ((w & 1u) && val == se)
      for (uint32_t a = 0; a < na; ++a)
        if ((at[3 * a + 1] & K_OI) && (at[3 * a + 2] & mask)) return true;
    p = at + 3 * na;
  }
  return false;
}

#ifndef ACS_AB_TIMING_NO_HR  // timing-only A/B builds: checkHierarchicalScope always true (wrong records)
#define ACS_AB_TIMING_NO_HR 0
#endif
// The owner tests of checkHierarchicalScope for one context slot: bit 0 the direct owner <->
// grant match (hierarchicalScope.ts:165-191), bit 1 the HR-tree match (:199-245, only when not
// direct).
ACS_FN uint32_t hr_owner_bits_walk(const ReqCtx& R, uint32_t slot, uint32_t role, uint32_t se) {
  const uint32_t d = hr_direct(R, slot, role, se) ? 1u : 0u;
  return d | ((!d && hr_tree(R, slot, role, se)) ? 2u : 0u);
}

// The owner tests of a request's context slots computed once per request, so that a rule's
// checkHierarchicalScope reads no slot record (the slot offset -> owners -> owner attributes chain
// of dependent arena reads).  hr_direct(slot, role, se) can hold only for the (role, se) of one of
// the request's grants and then depends on that pair alone: bit 8 slot + g for grant g.
// hr_tree(slot, role, se) needs (role, se) among the role scoping pairs and then depends on that
// pair alone: bit 8 slot + 4 + k for pair k.  Bit 16 + slot: the slot's owners are missing.  Bit
// 31: the digest holds (at most 2 slots, 4 grants, 4 pairs; else the tests walk the records).
// K1 computes it only in the instantiation for batches with ACL_NONE requests (c3adv 1M 1.76 ->
// 1.67 ms, r06_d): there the ACL lanes run many checks; in the plain one it cost more up front than
// the walk's on-demand tests, which run for ~13 lanes of a wave per check (c3 10M 2.94 -> 3.62 ms,
// c3r1 1M 0.403 -> 0.454).
constexpr uint32_t HRD_OK = 1u << 31;
#ifndef ACS_AN_HR_DIGEST
#define ACS_AN_HR_DIGEST 1  // 0: A/B builds without the digest
#endif
ACS_FN uint32_t hr_digest(const ReqCtx& R) {
  const uint32_t ns = R.n_slots(), ng = R.n_grants(), nk = R.n_rolese();
  if (ns == 0 || ns > 2 || ng > 4 || nk > 4) return 0u;
  uint32_t d = HRD_OK;
  for (uint32_t s = 0; s < ns; ++s) {
    if (slot_rec(R, s)[0]) d |= 1u << (16 + s);
    for (uint32_t g = 0; g < ng; ++g) {
      const uint32_t* gr = R.grants() + 3 * g;
      if (hr_direct(R, s, gr[0], gr[1])) d |= 1u << (8 * s + g);
    }
    for (uint32_t k = 0; k < nk; ++k) {
      const uint32_t* rs = R.rolese() + 2 * k;
      if (hr_tree(R, s, rs[0], rs[1])) d |= 1u << (8 * s + 4 + k);
    }
  }
  return d;
}

// hr_direct (bit 0) and, when not direct, hr_tree (bit 1) of slot `slot` for (role, se)
ACS_FN uint32_t hr_owner_bits(const ReqCtx& R, uint32_t slot, uint32_t role, uint32_t se) {
  if (!(R.hrd & HRD_OK)) return hr_owner_bits_walk(R, slot, role, se);
  for (uint32_t g = 0; g < R.n_grants(); ++g) {
    const uint32_t* gr = R.grants() + 3 * g;
    if (gr[0] == role && gr[1] == se && ((R.hrd >> (8 * slot + g)) & 1u)) return 1u;
  }
  for (uint32_t k = 0; k < R.n_rolese(); ++k) {
    const uint32_t* rs = R.rolese() + 2 * k;
    if (rs[0] == role && rs[1] == se) return ((R.hrd >> (8 * slot + 4 + k)) & 1u) ? 2u : 0u;
  }
  return 0u;
}

// slot `slot`'s owners are missing (the context resource's meta.owners is empty)
ACS_FN bool hr_owners_missing(const ReqCtx& R, uint32_t slot) {
  return (R.hrd & HRD_OK) ? ((R.hrd >> (16 + slot)) & 1u) != 0u : slot_rec(R, slot)[0] != 0u;
}

template <class RQ>
ACS_FN tri hierarchical_scope(const NodeRec& t, const RQ& R) {
  if (ACS_AB_TIMING_NO_HR || (t.tflags & TF_HR_TRIVIAL)) return 1;
  if (R.flag(RQ_CTX_EMPTY)) return 0;
  bool all_direct = true, all_ok = true;
  const RuleResAttr* ra = R.T.rres + t.res_off;
  for (uint32_t k = 0; k < t.res_n; ++k) {
    const RuleResAttr r = load_words(R.T, ra + wave_uniform(k));
    if (r.kind & K_ENT_LOOSE) {
      bool em = false;
      for (int j = 0; j < (int)R.h.nres; ++j) {
        const ReqRes q = R.res(j);
        if (q.kind & K_ENT_LOOSE) {
          if (loose_eq(q.value, r.value)) {
            em = true;
          } else {
            const uint8_t c = R.rx(q.col, r.row);
            if (c & RX_THROW_TYPE) return -(tri)ERR_TYPE;
            if (c & RX_THROW_SYNTAX) return -(tri)ERR_REGEX_SYNTAX;
            if (c & RX_HOST) return -(tri)ERR_REGEX_HOST;
            if (c & RX_RESET) em = false;
            if (c & RX_HIT) em = true;
          }
        } else if ((q.kind & K_RID_LOOSE) && em) {
          const uint32_t slot = q.slot_a;
          if (slot == NONE8) return 0;
          if (hr_owners_missing(R, slot)) return 0;
          const uint32_t b = hr_owner_bits(R, slot, t.role, t.se);
          all_direct = all_direct && (b & 1u);
          all_ok = all_ok && b != 0u;
        }
      }
    } else if (r.kind & K_OP) {
      for (int j = 0; j < (int)R.h.nres; ++j) {
        const ReqRes q = R.res(j);
        if (!((q.kind & K_OP) && q.value == r.value)) continue;
        const uint32_t slot = q.slot_b;
        if (slot == NONE8) return 0;
        if (hr_owners_missing(R, slot)) return 0;
        const uint32_t b = hr_owner_bits(R, slot, t.role, t.se);
        all_direct = all_direct && (b & 1u);
        all_ok = all_ok && b != 0u;
      }
    }
  }
  if (R.flag(RQ_RA_EMPTY)) return 0;
  if (all_direct) return 1;
  if (!(t.tflags & TF_HR_CHECK)) return 0;
  if (!R.flag(RQ_HRS_ITERABLE)) return -(tri)ERR_TYPE;  // getAllChildNodes(undefined)
  return all_ok ? 1 : 0;
}

// ------------------------------------------------------------------ verifyACLList
ACS_FN bool in_list(const uint32_t* l, uint32_t n, uint32_t v) {
  for (uint32_t k = 0; k < n; ++k)
    if (l[k] == v) return true;
  return false;
}

ACS_FN tri verify_acl(const NodeRec& t, const ReqCtx& R) {
  if (t.tflags & TF_ACL_SKIP) return 1;
  const uint32_t st = (R.h.flags >> RQ_ACL_SHIFT) & 3u;
  if (st == ACL_RET_TRUE) return 1;
  if (st == ACL_RET_FALSE || st == ACL_NONE) return 0;
  if (R.flag(RQ_SUBJ_MISSING)) return -(tri)ERR_TYPE;
  if (R.flag(RQ_RA_EMPTY)) return 0;
  if (!R.flag(RQ_HRS_ITERABLE)) return -(tri)ERR_TYPE;  // getRoleOrgMapping(undefined)
  const uint32_t* roles = R.T.u32pool + t.acl_roles_off;
  const uint32_t nr = t.acl_roles_n;
  if (R.flag(RQ_ACT_CREATE)) {
    if (R.n_tse() == 0) return 1;
    bool valid = false;
    for (uint32_t e = 0; e < R.n_tse(); ++e) {
      const uint32_t se = R.tse()[3 * e], ni = R.tse()[3 * e + 1];
      const uint32_t* inst = R.ar() + R.tse()[3 * e + 2];
      if (se == R.T.id_user) {
        valid = true;
        continue;
      }
      bool present = false;
      for (uint32_t k = 0; k < R.n_rolese() && !present; ++k)
        present = R.rolese()[2 * k + 1] == se && in_list(roles, nr, R.rolese()[2 * k]);
      if (!present) return 0;
      uint32_t validated = 0;  // bitmask over inst indices
      for (uint32_t kk = 0; kk < R.n_hrkeys(); ++kk) {
        if (!in_list(roles, nr, R.hrkeys()[kk])) continue;
        for (uint32_t x = 0; x < ni; ++x) {
          if ((inst[2 * x + 1] >> kk) & 1u) {
            valid = true;
            validated |= 1u << x;
            continue;
          }
          bool was = false;
          for (uint32_t y = 0; y < ni && !was; ++y) was = ((validated >> y) & 1u) && inst[2 * y] == inst[2 * x];
          if (!was) {
            valid = false;
            break;
          }
        }
      }
      if (!valid) return 0;
    }
    return valid ? 1 : 0;
  }
  if (R.flag(RQ_ACT_RMD)) {
    if (R.n_tse() == 0) return 1;
    for (uint32_t e = 0; e < R.n_tse(); ++e) {
      const uint32_t se = R.tse()[3 * e], ni = R.tse()[3 * e + 1];
      const uint32_t* inst = R.ar() + R.tse()[3 * e + 2];
      if (se == R.T.id_user)
        for (uint32_t x = 0; x < ni; ++x)
          if (inst[2 * x] == R.h.subject_id) return 1;
      for (uint32_t g = 0; g < R.n_grants(); ++g) {
        const uint32_t* gr = R.grants() + 3 * g;
        if (gr[1] != se || !in_list(roles, nr, gr[0])) continue;
        for (uint32_t x = 0; x < ni; ++x)
          if (inst[2 * x] == gr[2]) return 1;
      }
    }
    return 0;
  }
  return 0;
}

// ------------------------------------------------------------------ checkMultipleEntitiesMatch
template <class RQ>
ACS_FN tri multiple_entities(const NodeRec& S, const RQ& R) {
  for (int j = 0; j < (int)R.h.nres; ++j) {
    const ReqRes q = R.res(j);
    if (!(q.kind & K_ENT)) continue;
    bool multi = false;
    for (uint32_t p = S.child_begin; p < S.child_end; ++p) {
      const NodeRec P = node_at(R.T, R.T.pols, p, R.T.n_pols);
      if (P.nflags & NF_NULL) return -(tri)ERR_TYPE;  // policy.effect of null
      if (!(P.nflags & NF_HAS_TARGET) || P.res_n == 0) continue;
      const uint8_t pe = (P.nflags & NF_EFFECT_TRUTHY) ? P.effect : (uint8_t)EFF_UNDEF;  // no PERMIT default
      const tri m = resource_match(P, R, pe, false, false, j, j + 1, (q.kind & K_PROP) != 0, nullptr);
      if (m < 0) return m;
      if (m) multi = true;
    }
    if (!multi) return 0;
  }
  return 1;
}

// ------------------------------------------------------------------ isAllowed
// at = 1 + index of the policy set whose evaluation threw (0: request level); the
// rule-sharded reduction orders terminal events by it (shard_key below).
ACS_FN Decision make_err(tri e, uint32_t at = 0) {
  Decision d{};
  d.decision = DEC_INDETERMINATE;
  d.flags = OF_ERR;
  d.err = (uint8_t)(-e);
  d.aux = at;
  return d;
}

// AN: compile the ACL_NONE skips (acs_req_batch.hints); without them an ACL_NONE request is
// still decided exactly (verify_acl vetoes its pushes), the skips only cost registers.
template <bool AN = true, bool SK = false, class RQ, class FL>
ACS_FN Decision is_allowed_body(const RQ& R, const FL& F);

// SK: lanes skip the sets / policies / rules outside their own rows (ACS_OWN_SKIP bits) — the
// instantiation for waves that mix classes (spread small batches)
template <bool AN = true, bool SK = false, class RQ, class FL>
ACS_FN Decision is_allowed_t(const RQ& R, const FL& F) {
  PROF_T0(t_total);
  const Decision d = is_allowed_body<AN, SK>(R, F);
  PROF_ADD(PH_TOTAL, t_total);
  return d;
}

// One policy set of isAllowed (the body of accessController.ts:125-295's set loop): no
// effect, an effect (sf's eff / ec), or an event that ends the request there (an error the
// reference throws, or a reached rule condition: the record in *ev).
//
// events_only: the set lies below the deciding set (or an event) and the request is safe, so
// only an event it raises can still change the record (is_allowed_body).  For a safe request
// only three things raise one: a null policy in loop 2a, a reached rule condition and an
// invalid combining algorithm with a push.  So loop 2b skips the policies that have neither a
// condition rule nor an invalid algorithm (NF_COND_FREE, valid ca), and in a policy with a
// valid algorithm visits only its condition rules (a rule without one cannot raise an event,
// and reaching a condition does not depend on the rules before it).  Sets with an invalid
// algorithm are never evaluated this way (their event depends on any push).
enum SetOutcome { SET_NONE = 0, SET_EFFECT = 1, SET_EVENT = 2 };

template <bool AN, bool SK, class RQ, class FL>
ACS_FN int eval_set(const RQ& R, const FL& F, uint32_t s, const NodeRec& S, bool safe, bool events_only,
                    uint8_t* eff, uint8_t* ec, Decision* ev) {
  const Tables& T = R.T;
  const uint32_t WP = (T.n_pols + 31) >> 5;  // verdict section stride
  ACS_OPC(events_only ? OP_SET_EVENTS : OP_SET_EVAL);
  if (S.nflags & NF_HAS_TARGET) {
    PROF_T0(t0);
    ACS_OPC(OP_SET_TARGET);
    const tri m = target_match(S, R, EFF_PERMIT, false, false, nullptr);
    PROF_ADD(PH_SET_TARGET, t0);
    if (m < 0) return *ev = make_err(m, s + 1), SET_EVENT;
    if (!m) return SET_NONE;
  }
  // loop 2a: first exact policy match; policyEffect = precomputed prefix (accessController.ts:136-157)
  bool exact = false;
  uint8_t pe = S.pe_at;  // after a full scan
  PROF_T0(t2a);
  {
    CandRange pols(F, F.wp, S.child_begin, S.child_end);
    uint32_t p;
    while (pols.next(p)) {
      ACS_OPC(OP_P2A_ITER);
      const NodeRec P = node_at(T, T.pols, p, T.n_pols);
      if (P.nflags & NF_NULL) return *ev = make_err(-(tri)ERR_TYPE, s + 1), SET_EVENT;
      if (P.nflags & NF_HAS_TARGET) {
        const bool rl = (P.tflags & TF_SUBJ_ROLE) != 0;
        const bool vt = F.verdict(0, p, false, rl), vf = !vt && F.verdict(WP, p, true, rl);
#if defined(ACS_OP_COUNT)
        if (!vt && !vf) ACS_OPC(OP_P2A_TM);
#endif
        const tri m = vt ? 1 : vf ? 0 : target_match(P, R, P.pe_at, false, false, nullptr);
        if (m < 0) return *ev = make_err(m, s + 1), SET_EVENT;
        if (m) {
          exact = true;
          pe = P.pe_at;
          break;
        }
      }
    }
  }
  PROF_ADD(PH_POL_EXACT, t2a);
  if (exact && R.flag(RQ_MULTI_ENT)) {
    PROF_T0(tm);
    ACS_OPC(OP_MULTI);
    const tri m = multiple_entities(S, R);
    PROF_ADD(PH_MULTI, tm);
    if (m < 0) return *ev = make_err(m, s + 1), SET_EVENT;
    exact = m != 0;
  }
  Fold sf(S.ca);
  const bool cut_p = safe && (S.nflags & NF_COND_FREE);
  CandRange pols(F, F.wpu, S.child_begin, S.child_end);  // loop 2b: the useful policies
  uint32_t p;
  uint32_t pw = 0xFFFFFFFFu, pbits = 0;  // SK: the lane's own useful-policy word last read
  while (pols.next(p)) {
    if constexpr (SK && (ACS_OWN_SKIP & 2)) {
      if ((p >> 5) != pw) {  // a policy outside the lane's own useful row cannot change its record
        pw = p >> 5;
        pbits = F.own_word(F.wpu + pw);
      }
      if (!((pbits >> (p & 31u)) & 1u)) continue;
    }
    ACS_OPC(OP_P2B_ITER);
    const NodeRec P = node_at(T, T.pols, p, T.n_pols);
    if (P.nflags & NF_NULL) continue;
    if (events_only && (P.nflags & NF_COND_FREE) && P.ca != CA_INVALID) continue;  // raises no event
    // a safe request whose ACLs veto every rule's push (ACL_NONE): only rules that skip ACLs,
    // have no target (no verifyACL) or carry a condition (an event) can matter; in an ACL-gated
    // policy with rules only its condition rules, and with none the policy does nothing
    const bool acl_none = AN && safe && ((R.h.flags >> RQ_ACL_SHIFT) & 3u) == ACL_NONE;
    const bool gated = acl_none && P.map_size != 0 && acl_gated(T, p);
    if (gated && (P.nflags & NF_COND_FREE)) continue;
    const bool cond_rules_only = (events_only && P.ca != CA_INVALID) || gated;
    bool psm = true;
    if (P.nflags & NF_HAS_TARGET) {
      PROF_T0(tp);
      // the class's verdict for this lane's mode
      const bool rl = (P.tflags & TF_SUBJ_ROLE) != 0;
      const bool kt = exact ? F.verdict(0, p, false, rl) : F.verdict(2 * WP, p, false, rl);
      const bool kf = exact ? F.verdict(WP, p, true, rl) : F.verdict(3 * WP, p, true, rl);
#if defined(ACS_OP_COUNT)
      if (!kt && !kf) ACS_OPC(OP_P2B_TM);
#endif
      const tri m = kt ? 1 : kf ? 0 : target_match(P, R, pe, !exact, false, nullptr);
      if (m < 0) return *ev = make_err(m, s + 1), SET_EVENT;
      if (!m) {
        PROF_ADD(PH_POL_TARGET, tp);
        continue;
      }
      if (P.tflags & TF_HAS_SUBJECTS) {
        ACS_OPC(OP_P2B_HR);
        const tri h = hierarchical_scope(P, R);
        if (h < 0) return *ev = make_err(h, s + 1), SET_EVENT;
        psm = h != 0;
      }
      PROF_ADD(PH_POL_TARGET, tp);
    }
    if (P.map_size == 0 && (P.nflags & NF_EFFECT_TRUTHY)) {
      sf.push(P.effect, P.ec);
      if (cut_p && sf.final()) break;
      continue;
    }
    Fold rf(P.ca);
    const bool cut_r = safe && (P.nflags & NF_COND_FREE);
    ACS_OPC(OP_RULE_LOOP);
    CandRange rules(F, F.wr, P.child_begin, P.child_end);
    uint32_t r;
    uint32_t own_w = 0xFFFFFFFFu, own_bits = 0;  // SK: the lane's own rule-section word last read
    while (rules.next(r)) {
      ACS_OPC(OP_RULE_ITER);
      const NodeRec Q = rule_at(T, r);
      if (Q.nflags & NF_NULL) continue;
      if (cond_rules_only && !(Q.nflags & NF_HAS_CONDITION)) continue;
      if (acl_none && (Q.nflags & NF_HAS_TARGET) && !(Q.nflags & NF_HAS_CONDITION) && !(Q.tflags & TF_ACL_SKIP))
        continue;
      tri m = 1;
      if (Q.nflags & NF_HAS_TARGET) {
        PROF_T0(tr);
        const bool vt = F.verdict(4 * WP, r, false, (Q.tflags & TF_SUBJ_ROLE) != 0);
        // SK: the wave walks the union of its lanes' rows: a rule outside this lane's own row
        // cannot match its target (the filter keeps every node whose target can pass), so the
        // lane leaves it without target matching — a wave whose lanes all know the rule or do
        // not hold it skips the match altogether
        if constexpr (SK && (ACS_OWN_SKIP & 1)) {
          if (!vt) {
            if ((r >> 5) != own_w) {
              own_w = r >> 5;
              own_bits = F.own_word(F.wr + own_w);
            }
            if (!((own_bits >> (r & 31u)) & 1u)) continue;
          }
        }
#if defined(ACS_OP_COUNT)
        if (!vt) ACS_OPC(OP_RULE_TM);
#endif
        m = vt ? 1 : target_match_retry(Q, R, Q.effect, false, nullptr);
#if ACS_AB_PROBE_TM2
        if (!vt) {
          NodeRec Q2 = Q;
          Q2.role ^= acs_opaque0();
          const tri m2 = target_match_retry(Q2, R, Q.effect, false, nullptr);
          m = m2 == m ? m : m2;
        }
#endif
        if (m < 0) return *ev = make_err(m, s + 1), SET_EVENT;
        PROF_ADD(PH_RULE_TARGET, tr);
        if (!m) continue;
        PROF_T0(th);
        ACS_OPC(OP_RULE_HR);
        m = hierarchical_scope(Q, R);
#if ACS_AB_PROBE_HR2
        {
          NodeRec Q2 = Q;
          Q2.se ^= acs_opaque0();
          const tri m2 = hierarchical_scope(Q2, R);
          m = m2 == m ? m : m2;
        }
#endif
        PROF_ADD(PH_RULE_HR, th);
        if (m < 0) return *ev = make_err(m, s + 1), SET_EVENT;
      }
      if (m && (Q.nflags & NF_HAS_CONDITION)) {
        Decision d{};
        d.decision = DEC_INDETERMINATE;
        d.flags = OF_HOST_COND;
        d.aux = r;
        return *ev = d, SET_EVENT;
      }
      if (m && (Q.nflags & NF_HAS_TARGET)) {
        PROF_T0(ta);
        ACS_OPC(OP_RULE_ACL);
        m = verify_acl(Q, R);
        PROF_ADD(PH_RULE_ACL, ta);
        if (m < 0) return *ev = make_err(m, s + 1), SET_EVENT;
      }
      // evaluation_cacheable: the rule's own value while every non-null rule up to it was truthy
      if (m && psm) {
        rf.push(Q.effect, r < P.fe ? Q.ec : (uint8_t)EC_FALSE);
        if (cut_r && rf.final()) break;
      }
    }
    if (rf.n) {
      if (rf.ca == CA_INVALID) return *ev = make_err(-(tri)ERR_INVALID_CA, s + 1), SET_EVENT;
      sf.push(rf.eff, rf.ec);
      if (cut_p && sf.final()) break;
    }
  }
  if (!sf.n) return SET_NONE;
  if (sf.ca == CA_INVALID) return *ev = make_err(-(tri)ERR_INVALID_CA, s + 1), SET_EVENT;
  *eff = sf.eff;
  *ec = sf.ec;
  return SET_EFFECT;
}

// Whether set s can raise an event for a safe request of this filter (is_allowed_body below the
// deciding set): it holds a null policy or an invalid combining algorithm, or one of its rules
// that carries a condition is a candidate of some active lane (a rule no lane can match cannot be
// reached, and a safe request throws nowhere else).
template <class FL>
ACS_FN bool set_may_raise(const Tables& T, const FL& F, uint32_t s) {
  if (!T.ev_index) return true;
  const uint32_t r0 = T.ev_index[2 * s], w1 = T.ev_index[2 * s + 1];
  if (w1 >> 31) return true;
  const uint32_t r1 = w1 & 0x3FFFFFFFu;
  if (r0 >= r1) return false;
  const uint32_t* cb = T.ev_index + 2 * (size_t)T.n_sets;
  const uint32_t w0 = r0 >> 5, wl = (r1 - 1) >> 5;
  for (uint32_t w = w0; w <= wl; ++w) {
    uint32_t m = ~0u;
    if (w == w0) m &= ~0u << (r0 & 31);
    if (w == wl) m &= ~0u >> (31 - ((r1 - 1) & 31));
    const uint32_t c = cb[w] & m;
    ACS_SCAN(4);
    if (c && (F.word(F.wr + w) & c)) return true;
  }
  return false;
}

// isAllowed over the sets LAST TO FIRST.  Forward, the reference lets the last set with an
// effect decide (`effect` is overwritten per set, :293-295) unless an earlier set ends the
// request (the first error / reached condition).  So walking backwards, the first effect
// found is the answer unless a set below it has an event, and the lowest event found wins
// over everything.  Once something was found and every set below is clean (NF_CLEAN_BELOW)
// and the request safe (nothing of it can throw there: see `safe`), no set below can change
// the record and the lane stops; otherwise it walks on to set 0.
template <bool AN, bool SK, class RQ, class FL>
ACS_FN Decision is_allowed_body(const RQ& R, const FL& F) {
  const Tables& T = R.T;
  // Cutting a combining loop short: once a fold's result is final (Fold::final), the rest of
  // its loop can change the decision only by throwing or by reaching a rule condition.  A
  // request cannot throw there when its hierarchical_scopes is an array, context.subject is
  // present (checkHierarchicalScope / verifyACL TypeErrors) and no RegExp cell of its entity
  // values throws or needs the host (RES_RX_SAFE); NF_COND_FREE rules out conditions (and,
  // for a set, invalid combining algorithms).  Then the lane leaves the loop.
  bool safe = !R.B.no_cut && R.flag(RQ_HRS_ITERABLE) && !R.flag(RQ_SUBJ_MISSING);
  for (int j = 0; j < (int)R.h.nres && safe; ++j) {
    const ReqRes q = R.res(j);
    if ((q.kind & K_ENT_LOOSE) && !(q.pad & RES_RX_SAFE)) safe = false;
  }
  const bool acl_none = AN && safe && ((R.h.flags >> RQ_ACL_SHIFT) & 3u) == ACL_NONE;
  if constexpr (AN && ACS_AN_HR_DIGEST) {
    if (!R.flag(RQ_CTX_EMPTY)) R.hrd = hr_digest(R);
  }
  uint8_t eff = EFF_UNDEF, ec = EC_UNDEF;
  uint32_t last_set = 0;  // 1 + the last set with an effect (0: none yet)
  Decision ev{};
  bool have_ev = false;
  CandRangeRev sets(F, F.wsu, 0, T.n_sets);  // the useful sets (candidates.py), descending
  uint32_t s;
  uint32_t own_w = 0xFFFFFFFFu, own_bits = 0;  // SK: the lane's own useful-set word last read
  while (sets.next(s)) {
    if constexpr (SK && (ACS_OWN_SKIP & 4)) {
      // the wave walks the union of its lanes' useful sets; a set outside this lane's own useful
      // row cannot change its record (candidates.py: useful sections), so the lane leaves it —
      // and the wave, once no active lane holds it
      if ((s >> 5) != own_w) {
        own_w = s >> 5;
        own_bits = F.own_word(F.wsu + own_w);
      }
      if (!((own_bits >> (s & 31u)) & 1u)) continue;
    }
    ACS_OPC(OP_SET_ITER);
    const NodeRec S = node_at(T, T.sets, s, T.n_sets);
    // below the deciding set (or an event) only an event can change the record, and a clean
    // set cannot raise one for a safe request: skip it (the unclean ones below are walked)
    if ((have_ev || last_set) && safe && (S.nflags & NF_CLEAN)) {
      ACS_OPC(OP_SET_SKIP);
      continue;
    }
    uint8_t e2 = EFF_UNDEF, c2 = EC_UNDEF;
    Decision d2{};
    const bool events_only = (have_ev || last_set) && safe && S.ca != CA_INVALID;
    if (events_only && !set_may_raise(T, F, s)) continue;
    // an ACL_NONE request gets no push from an ACL-inert set: only its events matter
    if (acl_none && set_acl_inert(T, s) && !set_may_raise(T, F, s)) continue;
    const int o = eval_set<AN, SK>(R, F, s, S, safe, events_only, &e2, &c2, &d2);
    if (o == SET_EVENT) {
      ev = d2;  // lower than any event found so far
      have_ev = true;
    } else if (o == SET_EFFECT && !last_set) {
      eff = e2;
      ec = c2;
      last_set = s + 1;
    }
    if ((have_ev || last_set) && safe && (S.nflags & NF_CLEAN_BELOW)) break;
  }
  ACS_OPC(OP_LANE_DONE);
  if (have_ev) return ev;
  Decision out{};
  if (!last_set) {
    out.decision = DEC_INDETERMINATE;
    out.ec = EC_UNDEF;
    return out;
  }
  out.decision = (eff >= EFF_PERMIT && eff <= EFF_UNRECOGNIZED) ? eff : (uint8_t)DEC_INDETERMINATE;
  out.ec = ec;
  out.flags = OF_HAS_EFFECT;
  out.aux = last_set;
  return out;
}

ACS_FN Decision early_decision(const ReqHdr& h, bool* done) {
  Decision out{};
  *done = true;
  if (h.flags & RQ_HOST) {
    out.decision = DEC_INDETERMINATE;
    out.flags = OF_HOST_REQ;
    return out;
  }
  if (h.flags & RQ_NO_TARGET) {
    out.decision = DEC_DENY;
    out.ec = EC_FALSE;
    out.flags = OF_NO_TARGET;
    return out;
  }
  *done = false;
  return out;
}

// Filter of a single request (host build / per-lane reference).
ACS_FN Filter request_filter(const Batch& B, const ReqHdr& h) {
  Filter F{};
  F.wp = B.cand_wp;
  F.wr = B.cand_wr;
  F.wsu = B.cand_wsu;
  F.wpu = B.cand_wpu ? B.cand_wpu : B.cand_wp;
  F.wv = B.cand_wv;
  const uint32_t pc = h.flags >> RQ_PCOL_SHIFT;
  F.all = B.cand == nullptr || pc == PCOL_ALL || pc >= B.cand_rows || (h.flags & RQ_NO_TARGET);
  F.row = F.all ? nullptr : B.cand + (size_t)pc * B.cand_words;
  F.row2 = F.rrow = F.rrow2 = nullptr;
  F.vok = !F.all && B.cand_wv != 0;  // the request's own class row
  return F;
}

ACS_FN Filter request_filter(const Batch& B, const ReqHdr& h, uint32_t i) {
  Filter F = request_filter(B, h);
  if (F.all) return F;
  bool bad = false;
  F.row2 = second_row(B, i, &bad);
  if (bad) {  // a second class outside the rows: unfiltered, no verdicts
    F.all = true;
    F.vok = false;
    F.row2 = nullptr;
    return F;
  }
  if (B.role_key) role_rows_of(B, B.role_key[i], &F.rrow, &F.rrow2);
  return F;
}

ACS_FN Decision is_allowed(const Tables& T, const Batch& B, uint32_t i) {
  const ReqHdr h = req_hdr(B, i);
  bool done;
  Decision d = early_decision(h, &done);
  if (done) return d;
  return is_allowed_t(ReqMem(T, B, i, h, req_line(B, i)), request_filter(B, h, i));
}

// ------------------------------------------------------------------ whatIsAllowed
// Inclusion bitset row of one request: sets | policies | rules, each section starting on a
// 4-word (16-B) boundary, so a section's 16-B chunks belong to it alone.
struct BitsLayout {
  uint32_t wp, wr, words;  // word offsets of the policy / rule sections, row length (multiple of 4)
};
ACS_FN uint32_t up4(uint32_t x) { return (x + 3u) & ~3u; }
ACS_FN BitsLayout bits_layout(uint32_t n_sets, uint32_t n_pols, uint32_t n_rules) {
  BitsLayout L;
  L.wp = up4((n_sets + 31u) / 32u);
  L.wr = L.wp + up4((n_pols + 31u) / 32u);
  L.words = L.wr + up4((n_rules + 31u) / 32u);
  return L;
}

// Bit sinks.  whatIsAllowed visits sets, policies and rules in ascending index order within
// each section, so each section's bits arrive with non-decreasing word index.
struct NullSink {  // the obligation-only pass: no bitset
  template <int S> ACS_FN void set(uint32_t, uint32_t) {}
  ACS_FN void finish() {}
};
struct RowSink {   // host build: OR into a zeroed row
  uint32_t* row;
  template <int S> ACS_FN void set(uint32_t w, uint32_t bit) { row[w] |= bit; }
  ACS_FN void finish() {}
};
#if defined(__HIP_DEVICE_COMPILE__) || defined(__HIPCC__)
// GPU: each section's current 16-B chunk is accumulated in registers and stored once when the
// traversal moves past it; the chunks it skipped are stored as zeros.  Every word of the
// row is written exactly once (no zeroing pass, no read-modify-write, no scratch), 16 B per
// store, and a lane writes its row front to back, so L2 merges the pieces into whole lines.
struct ChunkSink {
  uint4* row;
  uint32_t cur[3], lim[3];
  uint4 buf[3];
  ACS_FN ChunkSink(uint32_t* r, const BitsLayout& L) : row(reinterpret_cast<uint4*>(r)) {
    cur[0] = 0; lim[0] = L.wp >> 2;
    cur[1] = L.wp >> 2; lim[1] = L.wr >> 2;
    cur[2] = L.wr >> 2; lim[2] = L.words >> 2;
    for (int k = 0; k < 3; ++k) buf[k] = make_uint4(0u, 0u, 0u, 0u);
  }
  template <int S> ACS_FN void flush(uint32_t upto) {
    row[cur[S]] = buf[S];
    for (uint32_t c = cur[S] + 1; c < upto; ++c) row[c] = make_uint4(0u, 0u, 0u, 0u);
    cur[S] = upto;
    buf[S] = make_uint4(0u, 0u, 0u, 0u);
  }
  template <int S> ACS_FN void set(uint32_t w, uint32_t bit) {
    const uint32_t c = w >> 2, q = w & 3u;
    if (c != cur[S]) flush<S>(c);
    buf[S].x |= q == 0u ? bit : 0u;
    buf[S].y |= q == 1u ? bit : 0u;
    buf[S].z |= q == 2u ? bit : 0u;
    buf[S].w |= q == 3u ? bit : 0u;
  }
  ACS_FN void finish() {
    if (cur[0] < lim[0]) flush<0>(lim[0]);
    if (cur[1] < lim[1]) flush<1>(lim[1]);
    if (cur[2] < lim[2]) flush<2>(lim[2]);
  }
};
#endif

// [s_begin, s_end): the policy sets evaluated (whatIsAllowed keeps no state across sets but the
// push log, so a request's log is the concatenation of the logs of consecutive set ranges).
template <class RQ, class Sink, class FL>
ACS_FN Decision what_is_allowed_t(const RQ& R, const FL& F, const BitsLayout& BL, Sink& bits, OblLog& obl,
                                  uint32_t s_begin = 0, uint32_t s_end = NONE32) {
  const Tables& T = R.T;
  const uint32_t WP = (T.n_pols + 31) >> 5;  // verdict section stride
  Decision out{};
  CandRange sets(F, 0, s_begin, s_end < T.n_sets ? s_end : T.n_sets);
  uint32_t s;
  while (sets.next(s)) {
    const NodeRec S = node_at(T, T.sets, s, T.n_sets);
    if (S.nflags & NF_HAS_TARGET) {
      const tri m = target_match(S, R, EFF_PERMIT, false, true, &obl);
      if (m < 0) return make_err(m, s + 1);
      if (!m) continue;
    }
    bool exact = false;
    uint8_t pe = S.pe_at;
    {
      CandRange pols(F, F.wp, S.child_begin, S.child_end);
      uint32_t p;
      while (pols.next(p)) {
        const NodeRec P = node_at(T, T.pols, p, T.n_pols);
        if (P.nflags & NF_NULL) return make_err(-(tri)ERR_TYPE, s + 1);
        if (P.nflags & NF_HAS_TARGET) {
          // a verdict-known target has no property attribute, so it pushes no obligation
          const bool rl = (P.tflags & TF_SUBJ_ROLE) != 0;
          const tri m = F.verdict(0, p, false, rl)     ? 1
                        : F.verdict(WP, p, true, rl) ? 0
                                                     : target_match(P, R, P.pe_at, false, true, &obl);
          if (m < 0) return make_err(m, s + 1);
          if (m) {
            exact = true;
            pe = P.pe_at;
            break;
          }
        }
      }
    }
    if (exact && R.flag(RQ_MULTI_ENT)) {
      const tri m = multiple_entities(S, R);
      if (m < 0) return make_err(m, s + 1);
      exact = m != 0;
    }
    bool any_pol = false;
    CandRange pols(F, F.wp, S.child_begin, S.child_end);
    uint32_t p;
    while (pols.next(p)) {
      const NodeRec P = node_at(T, T.pols, p, T.n_pols);
      if (P.nflags & NF_NULL) continue;
      if (P.nflags & NF_HAS_TARGET) {
        const bool rl = (P.tflags & TF_SUBJ_ROLE) != 0;
        const bool kt = exact ? F.verdict(0, p, false, rl) : F.verdict(2 * WP, p, false, rl);
        const bool kf = exact ? F.verdict(WP, p, true, rl) : F.verdict(3 * WP, p, true, rl);
        const tri m = kt ? 1 : kf ? 0 : target_match(P, R, pe, !exact, true, &obl);
        if (m < 0) return make_err(m, s + 1);
        if (!m) continue;
      }
      // Rules a word at a time: the candidates whose retried target match the lane's class
      // already knows to be true (verdict section 4 WP: targets without properties, so they
      // push no obligation) are included as a whole word, unread; the wave visits only the
      // rules some lane does not know (accessController.ts:389-418).
      bool any_rule = false;
      const uint32_t rb = P.child_begin, re = P.child_end;
      for (uint32_t base = rb & ~31u; base < re; base += 32) {
        const uint32_t w = base >> 5;
        uint32_t m = F.word(F.wr + w);
        if (base < rb) m &= ~0u << (rb & 31u);
        if (re - base < 32u) m &= (1u << (re - base)) - 1u;
        const uint32_t mine = m;
        const uint32_t known = mine & F.vword(4 * WP, w);  // this lane's
        if (known) {
          bits.template set<2>(BL.wr + w, known);
          any_rule = true;
        }
        uint32_t rest = wave_or(mine & ~known);
        while (rest) {
          const uint32_t r = wave_uniform(base + (uint32_t)__builtin_ctz(rest));
          rest &= rest - 1u;
          if (!((mine >> (r & 31u)) & 1u) || ((known >> (r & 31u)) & 1u)) continue;  // inert for it / included above
          const NodeRec Q = rule_at(T, r);
          if (Q.nflags & NF_NULL) continue;
          tri mt = 1;
          if (Q.nflags & NF_HAS_TARGET) {
            mt = target_match_retry(Q, R, Q.effect, true, &obl);
            if (mt < 0) return make_err(mt, s + 1);
          }
          if (mt) {
            bits.template set<2>(BL.wr + w, 1u << (r & 31u));
            any_rule = true;
          }
        }
      }
      if ((P.nflags & NF_EFFECT_TRUTHY) || any_rule) {
        bits.template set<1>(BL.wp + (p >> 5), 1u << (p & 31));
        any_pol = true;
      }
    }
    if (any_pol) bits.template set<0>(s >> 5, 1u << (s & 31));
  }
  if (obl.overflow) out.flags |= OF_OBL_OVERFLOW;
  return out;
}

// ------------------------------------------------------------------ whatIsAllowed templates
// Most of a whatIsAllowed walk (accessController.ts:343-419) is decided by a request's class row
// alone: which candidate sets are reached (sets without a target), loop 2a's `exact` (the first
// candidate policy whose exact target match the class knows to be true, every one before it
// known false), the loop-2b policy gates in that mode (verdict-known targets), and the rules
// whose retried match the class knows to be true (targets without properties: no obligation).
// A class's TEMPLATE records those inclusion bits; its WORK is the candidate rules of reached
// policies whose match depends on the request (a property attribute: these are the only targets
// that push maskedProperty obligations).  whatIsAllowed keeps no state across the walk but the
// push log, so a request whose class has a template is decided by copying the template and
// evaluating its work rules in index (= walk) order; its log is the same push sequence.  A class
// is not templated (TPL_OK clear) when some reached node is not verdict-known, a set has a
// target, or loop 2a meets a null policy (the walk throws there).  A composed request (two class
// rows, two role associations) is templated when both classes are, neither class's walk reads a
// target that tests role associations (TPL_ROLE_FREE: the two walks then take the same
// decisions, and the composed walk is their union), and they agree on `exact` for the sets both
// hold.  Anything else — no template, a multi-entity request (checkMultipleEntitiesMatch), a
// work rule that throws — takes the full walk (what_is_allowed_t).
enum TplFlags : uint32_t { TPL_OK = 1u, TPL_ROLE_FREE = 2u };

// Per-class template record (u32 words): [BitsLayout row | work rule bits (R) | exact sets (S) |
// work-word mask (a bit per nonzero work word) | flags], each section 4-word aligned.
struct TplLayout {
  uint32_t words;   // inclusion row (bits_layout(...).words), at 0
  uint32_t work;    // offset of the work bits, ceil(R / 32) words
  uint32_t exact;   // offset of the exact-set bits, ceil(S / 32) words
  uint32_t mask;    // offset of the work-word mask, ceil(work words / 32) words
  uint32_t flags;   // offset of the flags word
  uint32_t stride;  // record length (multiple of 4)
};
ACS_FN TplLayout tpl_layout(uint32_t n_sets, uint32_t n_pols, uint32_t n_rules) {
  TplLayout L;
  L.words = bits_layout(n_sets, n_pols, n_rules).words;
  const uint32_t ww = (n_rules + 31u) / 32u;
  L.work = L.words;
  L.exact = L.work + up4(ww);
  L.mask = L.exact + up4((n_sets + 31u) / 32u);
  L.flags = L.mask + up4((ww + 31u) / 32u);
  L.stride = L.flags + 4u;
  return L;
}

ACS_FN bool row_bit(const uint32_t* row, uint32_t off, uint32_t i) { return (row[off + (i >> 5)] >> (i & 31u)) & 1u; }

// The template of candidate set s for class row `row` (batch layout wp / wr / wv): its inclusion
// bits, work rules and exact decision go through acc (or_bits(word, bits) on the record);
// *role_free cleared when a target it reads tests role associations.  false: s makes the class
// untemplated.  Plain (per-lane) loads: the lanes of a template pass walk different sets.
template <class Acc>
ACS_FN bool wia_template_set(const Tables& T, const uint32_t* row, uint32_t wp, uint32_t wr, uint32_t wv,
                             const BitsLayout& BL, const TplLayout& TL, uint32_t s, Acc& acc, bool* role_free) {
  const uint32_t WP = (T.n_pols + 31) >> 5;
  const NodeRec S = T.sets[s];
  if (S.nflags & NF_HAS_TARGET) return false;
  bool exact = false;
  // the set's candidate policies a word at a time from the policy bitsets: loop 2a stops at the
  // first candidate that is null (untemplated), has a target the class does not decide
  // (untemplated) or has a target it knows exact (`exact`); role-testing targets up to there
  // clear role_free
  const uint32_t* pnull = policy_bits(T, 0);
  const uint32_t* ptgt = policy_bits(T, 1);
  const uint32_t* prole = policy_bits(T, 2);
  auto range_mask = [&](uint32_t base) {
    uint32_t m = ~0u;
    if (base < S.child_begin) m &= ~0u << (S.child_begin & 31u);
    if (S.child_end - base < 32u) m &= (1u << (S.child_end - base)) - 1u;
    return m;
  };
  for (uint32_t base = S.child_begin & ~31u; base < S.child_end; base += 32u) {
    const uint32_t w = base >> 5;
    const uint32_t cand = row[wp + w] & range_mask(base);
    const uint32_t nul = cand & pnull[w], tg = cand & ptgt[w] & ~nul;
    const uint32_t xt = tg & row[wv + w], xf = tg & row[wv + WP + w];
    const uint32_t stop = nul | (tg & ~xt & ~xf) | xt;
    if (!stop) {
      if (tg & prole[w]) *role_free = false;
      continue;
    }
    const uint32_t b = (uint32_t)__builtin_ctz(stop), upto = b == 31u ? ~0u : (2u << b) - 1u;
    if (tg & prole[w] & upto) *role_free = false;
    if (!((xt >> b) & 1u)) return false;  // a null policy or an undecided target
    exact = true;
    break;
  }
  if (exact) acc.or_bits(TL.exact + (s >> 5), 1u << (s & 31u));
  bool any_pol = false;
  // loop 2b: the candidate non-null policies whose target the class knows true in this mode (or
  // that have none) are kept, those it knows false skipped; an undecided one leaves the class
  // untemplated.  A kept policy's candidate non-null rules go a word at a time: known true (no
  // target, or a retried match the class knows) into the row, the others are work.
  const uint32_t* rlive = rule_live_bits(T);
  const uint32_t* rtgt = rule_target_bits(T);
  const uint32_t kts = exact ? 0u : 2u * WP, kfs = exact ? WP : 3u * WP;
  for (uint32_t base = S.child_begin & ~31u; base < S.child_end; base += 32u) {
    const uint32_t w = base >> 5;
    const uint32_t live = row[wp + w] & range_mask(base) & ~pnull[w], tg = live & ptgt[w];
    if (tg & prole[w]) *role_free = false;
    const uint32_t kt = row[wv + kts + w], kf = row[wv + kfs + w];
    if (tg & ~kt & ~kf) return false;
    for (uint32_t kept = live & ~(tg & ~kt); kept; kept &= kept - 1u) {
      const uint32_t p = base + (uint32_t)__builtin_ctz(kept);
      const NodeRec P = T.pols[p];
      bool any_rule = false;
      for (uint32_t rb = P.child_begin & ~31u; rb < P.child_end; rb += 32u) {
        const uint32_t rw = rb >> 5;
        uint32_t m = row[wr + rw] & rlive[rw];
        if (rb < P.child_begin) m &= ~0u << (P.child_begin & 31u);
        if (P.child_end - rb < 32u) m &= (1u << (P.child_end - rb)) - 1u;
        const uint32_t known = m & (~rtgt[rw] | row[wv + 4u * WP + rw]), work = m & ~known;
        if (known) {
          acc.or_bits(BL.wr + rw, known);
          any_rule = true;
        }
        if (work) acc.or_bits(TL.work + rw, work);
      }
      if ((P.nflags & NF_EFFECT_TRUTHY) || any_rule) {
        acc.or_bits(BL.wp + (p >> 5), 1u << (p & 31u));
        any_pol = true;
      }
    }
  }
  if (any_pol) acc.or_bits(s >> 5, 1u << (s & 31u));
  return true;
}

// Sink for a templated request: every 16-B chunk of the row is written once, as the template(s)
// OR the bits the work rules add (ChunkSink's order rule: each section's bits arrive with
// non-decreasing word index).
struct TplSink {
  uint32_t* row;
  const uint32_t* t1;  // template rows (t2: the second class's, or nullptr)
  const uint32_t* t2;
  uint32_t cur[3], lim[3];
  uint32_t buf[3][4];
  ACS_FN TplSink(uint32_t* r, const BitsLayout& L, const uint32_t* a, const uint32_t* b) : row(r), t1(a), t2(b) {
    cur[0] = 0; lim[0] = L.wp >> 2;
    cur[1] = L.wp >> 2; lim[1] = L.wr >> 2;
    cur[2] = L.wr >> 2; lim[2] = L.words >> 2;
    for (int k = 0; k < 3; ++k)
      for (int q = 0; q < 4; ++q) buf[k][q] = 0u;
  }
  ACS_FN void put(uint32_t c, const uint32_t* extra) {
    ACS_SCAN(t2 ? 32 : 16);  // the template chunk(s), shared by the class's lanes
    uint32_t v[4];
    for (int q = 0; q < 4; ++q) v[q] = t1[4 * c + q] | (t2 ? t2[4 * c + q] : 0u) | (extra ? extra[q] : 0u);
#if defined(__HIP_DEVICE_COMPILE__)
    reinterpret_cast<uint4*>(row)[c] = make_uint4(v[0], v[1], v[2], v[3]);
#else
    for (int q = 0; q < 4; ++q) row[4 * c + q] = v[q];
#endif
  }
  template <int S> ACS_FN void flush(uint32_t upto) {
    put(cur[S], buf[S]);
    for (uint32_t c = cur[S] + 1; c < upto; ++c) put(c, nullptr);
    cur[S] = upto;
    for (int q = 0; q < 4; ++q) buf[S][q] = 0u;
  }
  template <int S> ACS_FN void set(uint32_t w, uint32_t bit) {
    const uint32_t c = w >> 2;
    if (c != cur[S]) flush<S>(c);
    buf[S][w & 3u] |= bit;
  }
  ACS_FN void finish() {
    if (cur[0] < lim[0]) flush<0>(lim[0]);
    if (cur[1] < lim[1]) flush<1>(lim[1]);
    if (cur[2] < lim[2]) flush<2>(lim[2]);
  }
};

// Whether request R (class rows c1, c2: template records t1 / t2, nullptr for none) is decided
// from templates: both templated, composition exact (see above), not a multi-entity request.
ACS_FN bool tpl_usable(const TplLayout& TL, const uint32_t* t1, const uint32_t* t2, const uint32_t* row1,
                       const uint32_t* row2, uint32_t n_sets, uint32_t req_flags) {
  if (!t1 || !(t1[TL.flags] & TPL_OK) || (req_flags & (RQ_MULTI_ENT | RQ_HOST | RQ_NO_TARGET))) return false;
  if (!row2) return true;
  if (!t2 || !(t2[TL.flags] & TPL_OK) || !(t1[TL.flags] & t2[TL.flags] & TPL_ROLE_FREE)) return false;
  for (uint32_t w = 0; w < (n_sets + 31u) / 32u; ++w)
    if ((t1[TL.exact + w] ^ t2[TL.exact + w]) & row1[w] & row2[w]) return false;
  return true;
}

// A templated request: the template row(s) plus its work rules (t1 / t2's work bits, less the
// rules the other class's template already includes — known true there, so the full walk would
// not match them either), evaluated in index order with the pushes they make.  Work words are
// visited wave-uniformly (the union of the active lanes' work-word masks), a word's rules for the
// lanes that hold them.  Returns false when a work rule throws: the caller re-runs the request
// with the full walk (the row is then rewritten from scratch).
template <class RQ, class SINK>
ACS_FN bool what_is_allowed_tpl(const RQ& R, const TplLayout& TL, const BitsLayout& BL, const uint32_t* t1,
                                const uint32_t* t2, SINK& sink, OblLog& obl) {
  const Tables& T = R.T;
  const uint32_t MW = (TL.flags - TL.mask);  // mask words (padded)
  ACS_OPC(OP_TPL_REQ);
  for (uint32_t k = 0; k < MW; ++k) {
    ACS_SCAN(t2 ? 8 : 4);
    uint32_t u = wave_or(t1[TL.mask + k] | (t2 ? t2[TL.mask + k] : 0u));
    while (u) {
      const uint32_t w = wave_uniform(32u * k + (uint32_t)__builtin_ctz(u));
      u &= u - 1u;
      ACS_OPC(OP_TPL_WORD);
      ACS_SCAN(t2 ? 16 : 4);
      uint32_t mine = t1[TL.work + w] & ~(t2 ? t2[BL.wr + w] : 0u);
      if (t2) mine |= t2[TL.work + w] & ~t1[BL.wr + w];
      uint32_t rest = wave_or(mine);
      while (rest) {
        const uint32_t r = wave_uniform(32u * w + (uint32_t)__builtin_ctz(rest));
        rest &= rest - 1u;
        ACS_OPC(OP_TPL_RULE);
        if (!((mine >> (r & 31u)) & 1u)) continue;
        ACS_OPC(OP_TPL_TM);
        const NodeRec Q = rule_at(T, r);
        const tri m = target_match_retry(Q, R, Q.effect, true, &obl);
        if (m < 0) return false;
        if (m) {
          ACS_OPC(OP_TPL_HIT);
          const uint32_t p = T.parents[r + T.n_pols], s = T.parents[p];
          sink.template set<0>(s >> 5, 1u << (s & 31u));
          sink.template set<1>(BL.wp + (p >> 5), 1u << (p & 31u));
          sink.template set<2>(BL.wr + w, 1u << (r & 31u));
        }
      }
    }
  }
  sink.finish();
  return true;
}

// Host build: row = this request's zeroed BitsLayout row.
ACS_FN Decision what_is_allowed(const Tables& T, const Batch& B, uint32_t i, uint32_t* row, uint32_t* obl_out,
                                uint32_t* obl_n) {
  const ReqHdr h = req_hdr(B, i);
  OblLog obl{obl_out, 0, false};
  Decision d{};
  if (h.flags & RQ_HOST) {
    d.flags = OF_HOST_REQ;
  } else {
    RowSink sink{row};
    d = what_is_allowed_t(ReqMem(T, B, i, h, req_line(B, i)), request_filter(B, h, i),
                          bits_layout(T.n_sets, T.n_pols, T.n_rules),
                          sink, obl);
  }
  *obl_n = (d.flags & OF_ERR) ? 0u : obl.n;
  return d;
}

// ------------------------------------------------------------------ rule-sharded isAllowed (C1)
// whole policy sets are partitioned over ranks and every rank evaluates every
// request against its own sets.  Sets are independent except for two cross-set rules of
// isAllowed (accessController.ts:125-295): the LAST set with a policy effect decides
// (`effect` is overwritten per set, :293-295), and the FIRST set whose evaluation throws or
// reaches a rule condition ends the request.  One 64-bit key per request and rank turns
// both into a plain integer MAX across ranks:
//   bit 62       terminal event (error, rule condition, request-level host / no target)
//   bits 61..33  terminal: SHARD_ORDER_MAX - at (at = 1 + global set index; 0: request level)
//                else    : 1 + global index of the last applicable set (0: none)
//   bit 32       payload is a global rule index (a rule condition was reached)
//   bits 31..0   payload: decision | ec << 8 | flags << 16 | err << 24, or that rule index
// Keys stay below 2^63, so a signed int64 all-reduce MAX (RCCL, gloo) orders them as well.
struct ShardBase {
  uint32_t set_base, pol_base, rule_base;  // global index of the rank's first set / policy / rule
};
constexpr uint32_t SHARD_ORDER_MAX = (1u << 29) - 1;

// Policy set that holds (local) rule r: child ranges are contiguous and ascending.
ACS_FN uint32_t set_of_rule(const Tables& T, uint32_t r) {
  uint32_t lo = 0, hi = T.n_pols;
  while (hi - lo > 1) {
    const uint32_t mid = (lo + hi) / 2;
    if (T.pols[mid].child_begin <= r) lo = mid; else hi = mid;
  }
  uint32_t a = 0, b = T.n_sets;
  while (b - a > 1) {
    const uint32_t mid = (a + b) / 2;
    if (T.sets[mid].child_begin <= lo) a = mid; else b = mid;
  }
  return a;
}

ACS_FN uint64_t shard_key(const Tables& T, const Decision& d, const ShardBase& b) {
  const uint64_t term = 1ull << 62;
  const uint64_t payload = (uint64_t)d.decision | (uint64_t)d.ec << 8 | (uint64_t)d.flags << 16 |
                           (uint64_t)d.err << 24;
  if (d.flags & OF_HOST_COND) {
    const uint32_t at = set_of_rule(T, d.aux) + b.set_base + 1;
    return term | (uint64_t)(SHARD_ORDER_MAX - at) << 33 | (1ull << 32) | (uint64_t)(d.aux + b.rule_base);
  }
  if (d.flags & OF_ERR) {
    const uint32_t at = d.aux ? d.aux + b.set_base : 0u;
    return term | (uint64_t)(SHARD_ORDER_MAX - at) << 33 | payload;
  }
  if (d.flags & (OF_HOST_REQ | OF_NO_TARGET)) return term | (uint64_t)SHARD_ORDER_MAX << 33 | payload;
  const uint32_t last = d.aux ? d.aux + b.set_base : 0u;
  return (uint64_t)last << 33 | payload;
}

// A rule-sharded handle's class rows (acs_compile_sharded): the batch's rows in the global
// layout [S | P | useful S | useful P | R | verdicts: 4 x P, R] cut to one shard's nodes —
// each section's bits [bit0, bit0 + nbits) moved to bit 0 of the shard's section.
struct RowSlice {
  uint32_t n;                                // sections present
  uint32_t src[10], dst[10], bit0[10], nbits[10];
  uint32_t words;                            // the shard's row length
  uint32_t wp, wr, wsu, wpu, wv;             // its section offsets (acs_req_batch.cand_*)
};

// Build the slice of a global layout (offsets as in acs_req_batch; 0: section absent) for a
// shard holding sets / policies / rules [b.*_base, + n_*).
inline RowSlice make_row_slice(uint32_t g_pols, uint32_t cand_wp, uint32_t cand_wr, uint32_t cand_wsu,
                               uint32_t cand_wpu, uint32_t cand_wv, const ShardBase& b, uint32_t ns,
                               uint32_t np, uint32_t nr) {
  RowSlice L{};
  const uint32_t ws = (ns + 31) / 32, wp = (np + 31) / 32, wr = (nr + 31) / 32, gwp = (g_pols + 31) / 32;
  uint32_t at = 0;
  auto add = [&](uint32_t src, uint32_t bit0, uint32_t nbits, uint32_t w) {
    L.src[L.n] = src;
    L.dst[L.n] = at;
    L.bit0[L.n] = bit0;
    L.nbits[L.n] = nbits;
    ++L.n;
    const uint32_t d = at;
    at += w;
    return d;
  };
  add(0, b.set_base, ns, ws);
  L.wp = add(cand_wp, b.pol_base, np, wp);
  if (cand_wsu) L.wsu = add(cand_wsu, b.set_base, ns, ws);
  if (cand_wpu) L.wpu = add(cand_wpu, b.pol_base, np, wp);
  L.wr = add(cand_wr, b.rule_base, nr, wr);
  if (cand_wv) {
    L.wv = at;
    for (uint32_t k = 0; k < 4; ++k) add(cand_wv + k * gwp, b.pol_base, np, wp);
    add(cand_wv + 4 * gwp, b.rule_base, nr, wr);
  }
  L.words = at;
  return L;
}

// Word w of the shard's row cut from global row `row` (src_words long).
ACS_FN uint32_t slice_word(const uint32_t* row, uint32_t src_words, const RowSlice& L, uint32_t w) {
  uint32_t k = 0;
  while (k + 1 < L.n && L.dst[k + 1] <= w) ++k;
  const uint32_t j = w - L.dst[k];
  if (32 * j >= L.nbits[k]) return 0u;
  const uint32_t bit = L.bit0[k] + 32 * j, sw = L.src[k] + (bit >> 5), sh = bit & 31u;
  uint32_t x = sw < src_words ? row[sw] >> sh : 0u;
  if (sh && sw + 1 < src_words) x |= row[sw + 1] << (32u - sh);
  const uint32_t left = L.nbits[k] - 32 * j;
  return left >= 32 ? x : x & ((1u << left) - 1u);
}

// Reduced key -> the decision record an unsharded evaluation writes (global indices).
ACS_FN Decision shard_decode(uint64_t key) {
  Decision d{};
  if (key & (1ull << 32)) {
    d.decision = DEC_INDETERMINATE;
    d.flags = OF_HOST_COND;
    d.aux = (uint32_t)key;
    return d;
  }
  const uint32_t order = (uint32_t)(key >> 33) & SHARD_ORDER_MAX;
  d.decision = (uint8_t)key;
  d.ec = (uint8_t)(key >> 8);
  d.flags = (uint8_t)(key >> 16);
  d.err = (uint8_t)(key >> 24);
  if (key & (1ull << 62)) {
    d.aux = (d.flags & OF_ERR) ? SHARD_ORDER_MAX - order : 0u;
  } else {
    d.aux = order;
  }
  return d;
}

}  // namespace acs
