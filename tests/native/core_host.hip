// core_host.hip — TEST INFRASTRUCTURE: the evaluator core (csrc/acs_eval.h) run on the
// host CPU, request by request, over the same packed tables/batches the GPU kernels
// consume.  Lets the not-gpu test tier check the host compiler + encoder + core
// logic against the oracle in a container without a GPU.  Never linked into the
// product library (libacs_mi355x.so has no CPU path).
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/acs_mi355x.h"
#include "../../access-control-srv_amd/csrc/acs_eval.h"

using namespace acs;

static size_t a16(size_t x) { return (x + 15) & ~size_t(15); }

static bool host_tables(const void* blob, size_t n, Tables* T) {
  acs_blob_header h;
  if (n < sizeof h) return false;
  std::memcpy(&h, blob, sizeof h);
  if (h.magic != ACS_BLOB_MAGIC) return false;
  const char* p = (const char*)blob + a16(sizeof h);
  const size_t sz[6] = {h.n_sets * sizeof(NodeRec), h.n_pols * sizeof(NodeRec), h.n_rules * sizeof(NodeRec),
                        h.n_rres * sizeof(RuleResAttr), h.n_pairs * sizeof(Pair), h.n_u32pool * sizeof(uint32_t)};
  const char* s[6];
  for (int k = 0; k < 6; ++k) {
    s[k] = p;
    p += a16(sz[k]);
  }
  T->sets = (const NodeRec*)s[0];
  T->pols = (const NodeRec*)s[1];
  T->rules = (const NodeRec*)s[2];
  T->rres = (const RuleResAttr*)s[3];
  T->pairs = (const Pair*)s[4];
  T->u32pool = (const uint32_t*)s[5];
  T->n_sets = h.n_sets;
  T->n_pols = h.n_pols;
  T->n_rules = h.n_rules;
  T->id_user = h.id_user;
  T->rstride = 1;  // blob layout: 64-B rule records, separate pools
  // the event index (one per thread: the host entry points are called one batch at a time)
  static thread_local std::vector<uint32_t> evx;
  evx.assign(event_index_words(h.n_sets, h.n_pols, h.n_rules), 0u);
  build_event_index(T->sets, h.n_sets, T->pols, h.n_pols, T->rules, h.n_rules, evx.data());
  T->ev_index = getenv("ACS_HOST_NO_EV_INDEX") ? nullptr : evx.data();
  static thread_local std::vector<uint32_t> par;
  par.assign(parent_index_words(h.n_pols, h.n_rules), 0u);
  build_parents(T->sets, h.n_sets, T->pols, h.n_pols, T->rules, h.n_rules, par.data());
  T->parents = par.data();
  return true;
}

static Batch host_batch(const acs_req_batch* b) {
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
  B.cand_rows = b->cand ? b->cand_rows : 0u;
  B.role_key = b->cand ? b->role_key : nullptr;
  B.role_bits = b->role_rows_bits;
  B.role_rows = b->role_key ? b->role_rows : 0u;
  B.lines = (const ReqLine*)b->lines;  // a compact batch reads its lines + extension records
  B.ext = b->ext;
  // cut-invariance tests (tests/test_cut.py): ACS_NO_CUT=1 in this test build only; the product
  // library fixes it at compile time (ACS_AB_NO_CUT)
  const char* no_cut = getenv("ACS_NO_CUT");
  B.no_cut = no_cut && *no_cut == '1' ? 1u : 0u;
  return B;
}

extern "C" int acs_host_is_allowed(const void* blob, size_t n, const acs_req_batch* b, acs_decision* out) {
  Tables T;
  if (!host_tables(blob, n, &T)) return -1;
  Batch B = host_batch(b);
  for (uint32_t i = 0; i < B.n; ++i) {
    Decision d = is_allowed(T, B, i);
    std::memcpy(&out[i], &d, sizeof d);
  }
  return 0;
}

// Rule-sharded reduction keys / decode (csrc/acs_eval.h shard_key) on the host, for the
// world-size-2 gloo tests of the sharded path.
extern "C" int acs_host_shard_keys(const void* blob, size_t n, const acs_decision* dec, size_t m,
                                   const acs_shard* s, uint64_t* keys) {
  Tables T;
  if (!host_tables(blob, n, &T)) return -1;
  const ShardBase b{s->set_base, s->pol_base, s->rule_base};
  for (size_t i = 0; i < m; ++i) {
    Decision d;
    std::memcpy(&d, &dec[i], sizeof d);
    keys[i] = shard_key(T, d, b);
  }
  return 0;
}

extern "C" void acs_host_shard_decode(const uint64_t* keys, size_t m, acs_decision* out) {
  for (size_t i = 0; i < m; ++i) {
    const Decision d = shard_decode(keys[i]);
    std::memcpy(&out[i], &d, sizeof d);
  }
}

extern "C" int acs_host_what_is_allowed(const void* blob, size_t n, const acs_req_batch* b, uint32_t* bits,
                                        uint32_t* obl, uint32_t* obl_n, acs_decision* out) {
  Tables T;
  if (!host_tables(blob, n, &T)) return -1;
  Batch B = host_batch(b);
  const uint32_t words = bits_layout(T.n_sets, T.n_pols, T.n_rules).words;
  for (uint32_t i = 0; i < B.n; ++i) {
    uint32_t* mb = bits + (size_t)i * words;
    for (uint32_t w = 0; w < words; ++w) mb[w] = 0;
    Decision d = what_is_allowed(T, B, i, mb, obl + (size_t)i * 2 * OBL_MAX, obl_n + i);
    std::memcpy(&out[i], &d, sizeof d);
  }
  return 0;
}

// Obligation-only pass (acs_what_is_allowed_obl's CPU twin): requests idx[0..m) with the
// policy sets cut into `chunks` ranges, a cap-entry log per (range, request) and no bitset;
// obl_n[c][j] = total pushes of range c of request j.
// g_sets / set_base: the ranges cut the whole store's sets, this image holding [set_base, + its
// n_sets) of them (a shard of a rule-sharded handle); the plain form passes n_sets / 0.
extern "C" int acs_host_what_is_allowed_obl_shard(const void* blob, size_t n, const acs_req_batch* b,
                                                  const uint32_t* idx, size_t m, uint32_t chunks, uint32_t cap,
                                                  uint32_t* obl, uint32_t* obl_n, uint32_t g_sets, uint32_t set_base);

extern "C" int acs_host_what_is_allowed_obl(const void* blob, size_t n, const acs_req_batch* b, const uint32_t* idx,
                                            size_t m, uint32_t chunks, uint32_t cap, uint32_t* obl,
                                            uint32_t* obl_n) {
  acs_blob_header h;
  std::memcpy(&h, blob, sizeof h);
  return acs_host_what_is_allowed_obl_shard(blob, n, b, idx, m, chunks, cap, obl, obl_n, h.n_sets, 0);
}

static uint32_t clip_local(uint32_t g, uint32_t base, uint32_t n) {
  return g <= base ? 0u : (g - base < n ? g - base : n);
}

extern "C" int acs_host_what_is_allowed_obl_shard(const void* blob, size_t n, const acs_req_batch* b,
                                                  const uint32_t* idx, size_t m, uint32_t chunks, uint32_t cap,
                                                  uint32_t* obl, uint32_t* obl_n, uint32_t g_sets, uint32_t set_base) {
  Tables T;
  if (!host_tables(blob, n, &T)) return -1;
  Batch B = host_batch(b);
  for (uint32_t c = 0; c < chunks; ++c)
    for (size_t j = 0; j < m; ++j) {
      const uint32_t i = idx[j];
      if (i >= B.n) return -1;
      const size_t k = (size_t)c * m + j;
      const ReqHdr h = req_hdr(B, i);
      OblLog log{obl + k * 2 * (size_t)cap, 0, false, cap, 0};
      uint32_t total = 0;
      if (!(h.flags & RQ_HOST)) {
        const uint32_t s0 = clip_local((uint32_t)((uint64_t)g_sets * c / chunks), set_base, T.n_sets);
        const uint32_t s1 = clip_local((uint32_t)((uint64_t)g_sets * (c + 1) / chunks), set_base, T.n_sets);
        NullSink none;
        const Decision d =
            what_is_allowed_t(ReqMem(T, B, i, h, req_line(B, i)), request_filter(B, h, i), BitsLayout{}, none, log, s0,
                              s1);
        total = (d.flags & OF_ERR) ? 0u : log.total;
      }
      obl_n[k] = total;
    }
  return 0;
}

#if defined(ACS_HOST_WORK)
namespace acs {
thread_local unsigned long long acs_host_work = 0;
}
// Per request: its record and the table bytes its evaluation read (tools/lane_work.py).
extern "C" int acs_host_is_allowed_work(const void* blob, size_t n, const acs_req_batch* b, acs_decision* out,
                                        unsigned long long* work) {
  Tables T;
  if (!host_tables(blob, n, &T)) return -1;
  Batch B = host_batch(b);
  for (uint32_t i = 0; i < B.n; ++i) {
    acs_host_work = 0;
    Decision d = is_allowed(T, B, i);
    std::memcpy(&out[i], &d, sizeof d);
    work[i] = acs_host_work;
  }
  return 0;
}

extern "C" int acs_host_what_is_allowed_work(const void* blob, size_t n, const acs_req_batch* b, unsigned long long* work) {
  Tables T;
  if (!host_tables(blob, n, &T)) return -1;
  Batch B = host_batch(b);
  const uint32_t words = bits_layout(T.n_sets, T.n_pols, T.n_rules).words;
  std::vector<uint32_t> row(words), obl(2 * OBL_MAX);
  for (uint32_t i = 0; i < B.n; ++i) {
    acs_host_work = 0;
    uint32_t on = 0;
    for (uint32_t& w : row) w = 0;
    what_is_allowed(T, B, i, row.data(), obl.data(), &on);
    work[i] = acs_host_work;
  }
  return 0;
}
#endif

// whatIsAllowed templates (csrc/acs_eval.h wia_template_set): the template record of every class
// row of the batch, as the GPU's template pass writes them; out: [cand_rows][stride] words.
extern "C" int acs_host_wia_templates(const void* blob, size_t n, const acs_req_batch* b, uint32_t* out,
                                      uint32_t* stride) {
  Tables T;
  if (!host_tables(blob, n, &T)) return -1;
  const TplLayout TL = tpl_layout(T.n_sets, T.n_pols, T.n_rules);
  const BitsLayout BL = bits_layout(T.n_sets, T.n_pols, T.n_rules);
  *stride = TL.stride;
  if (!out) return 0;
  if (!b->cand || !b->cand_wv) return -1;
  struct Acc {
    uint32_t* rec;
    void or_bits(uint32_t w, uint32_t bit) { rec[w] |= bit; }
  };
  for (uint32_t c = 0; c < b->cand_rows; ++c) {
    uint32_t* rec = out + (size_t)c * TL.stride;
    for (uint32_t w = 0; w < TL.stride; ++w) rec[w] = 0;
    const uint32_t* row = b->cand + (size_t)c * b->cand_words;
    Acc acc{rec};
    bool ok = true, role_free = true;
    for (uint32_t s = 0; s < T.n_sets && ok; ++s)
      if (row_bit(row, 0, s)) ok = wia_template_set(T, row, b->cand_wp, b->cand_wr, b->cand_wv, BL, TL, s, acc, &role_free);
    if (!ok) {
      for (uint32_t w = 0; w < TL.stride; ++w) rec[w] = 0;
      continue;
    }
    for (uint32_t w = 0; w < TL.exact - TL.work; ++w)
      if (rec[TL.work + w]) rec[TL.mask + (w >> 5)] |= 1u << (w & 31u);
    rec[TL.flags] = TPL_OK | (role_free ? TPL_ROLE_FREE : 0u);
  }
  return 0;
}

// acs_host_set_tpl_which(w): acs_host_what_is_allowed_tpl also sets w[i] = 1 for each request i
// a template decided (tools: which waves keep a full-walk lane)
static uint8_t* g_tpl_which = nullptr;
extern "C" void acs_host_set_tpl_which(uint8_t* w) { g_tpl_which = w; }

// whatIsAllowed from the templates where usable (tpl_usable), else the full walk: the outputs
// of acs_host_what_is_allowed; *templated: how many requests took a template.
extern "C" int acs_host_what_is_allowed_tpl(const void* blob, size_t n, const acs_req_batch* b, const uint32_t* tpl,
                                            uint32_t* bits, uint32_t* obl, uint32_t* obl_n, acs_decision* out,
                                            size_t* templated) {
  Tables T;
  if (!host_tables(blob, n, &T)) return -1;
  Batch B = host_batch(b);
  const TplLayout TL = tpl_layout(T.n_sets, T.n_pols, T.n_rules);
  const BitsLayout BL = bits_layout(T.n_sets, T.n_pols, T.n_rules);
  *templated = 0;
  for (uint32_t i = 0; i < B.n; ++i) {
    uint32_t* row = bits + (size_t)i * BL.words;
    const ReqHdr h = req_hdr(B, i);
    const uint32_t c1 = h.flags >> RQ_PCOL_SHIFT;
    const uint32_t c2 = B.lines ? B.lines[i].cls2 : 0u;
    const uint32_t* t1 = B.cand && c1 < B.cand_rows ? tpl + (size_t)c1 * TL.stride : nullptr;
    const uint32_t* t2 = t1 && c2 && c2 - 1u < B.cand_rows ? tpl + (size_t)(c2 - 1u) * TL.stride : nullptr;
    const uint32_t* r1 = t1 ? B.cand + (size_t)c1 * B.cand_words : nullptr;
    const uint32_t* r2 = t2 ? B.cand + (size_t)(c2 - 1u) * B.cand_words : nullptr;
    if (!(c2 && !t2) && tpl_usable(TL, t1, t2, r1, r2, T.n_sets, h.flags)) {
      OblLog log{obl + (size_t)i * 2 * OBL_MAX, 0, false};
      TplSink sink(row, BL, t1, t2);
      if (what_is_allowed_tpl(ReqMem(T, B, i, h, req_line(B, i)), TL, BL, t1, t2, sink, log)) {
        Decision d{};
        if (log.overflow) d.flags |= OF_OBL_OVERFLOW;
        std::memcpy(&out[i], &d, sizeof d);
        obl_n[i] = log.n;
        ++*templated;
        if (g_tpl_which) g_tpl_which[i] = 1;
        continue;
      }
    }
    for (uint32_t w = 0; w < BL.words; ++w) row[w] = 0;
    Decision d = what_is_allowed(T, B, i, row, obl + (size_t)i * 2 * OBL_MAX, obl_n + i);
    std::memcpy(&out[i], &d, sizeof d);
  }
  return 0;
}
