// acs_validate.cpp — host-side structural checks of what the kernels dereference.
//
// The kernels index the compiled tables and the request batch without bounds checks (every
// record load is on the hot path).  A malformed image or batch handed to the host-buffer
// entry points (acs_compile, acs_is_allowed, acs_what_is_allowed, acs_what_is_allowed_obl)
// would turn into out-of-bounds device reads, so they are walked here first, once, on the
// host copy: every child range, pool offset, arena offset and regex-matrix coordinate the
// device code follows must land inside its buffer.  The *_device entry points take
// device-resident batches (normally from acs_codec_encode, which writes them consistent)
// and are not walked.
#include <cstring>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <cstddef>
#include <thread>
#include <vector>

#include "acs_pool.h"
#include "../../include/acs_mi355x.h"
#include "acs_layout.h"

using namespace acs;

extern "C" void acs_internal_set_error(const char* msg);

namespace {

int bad(const char* what, size_t at) {
  char msg[192];
  snprintf(msg, sizeof msg, "malformed %s (at %zu)", what, at);
  acs_internal_set_error(msg);
  return -1;
}

size_t align16(size_t x) { return (x + 15) & ~size_t(15); }
uint32_t words32(uint32_t n) { return (n + 31) >> 5; }

// f(lo, hi) over [0, n) on up to 16 host threads (acs_pool.h workers) (one per 64k items); returns the smallest item
// index any call reported (f returns its first bad index, or n when none), so the error message
// names the same request as a serial walk would.
template <class F>
size_t parallel_first_bad(size_t n, F f) {
  size_t T = std::thread::hardware_concurrency();
  T = T < 1 ? 1 : (T > 16 ? 16 : T);
  if (T > n / 65536 + 1) T = n / 65536 + 1;
  std::vector<size_t> bad(T, n);
  // inline when the pool is busy (a pipeline encoding the next chunk): the check does not wait for it
  acs_pool::run((int)T, [&](int t) { bad[t] = f(n * t / T, n * (t + 1) / T); }, true);
  size_t m = n;
  for (size_t b : bad) m = b < m ? b : m;
  return m;
}

}  // namespace

extern "C" {

// Image checks for acs_compile; *rx_rows_min = 1 + the largest regex-matrix row any rule
// resource attribute reads (0: none).
int acs_internal_check_blob(const void* blob, size_t n_bytes, uint32_t* rx_rows_min) {
  acs_blob_header h;
  memcpy(&h, blob, sizeof h);
  const char* p = (const char*)blob + align16(sizeof h);
  const NodeRec* sets = (const NodeRec*)p;
  p += align16((size_t)h.n_sets * sizeof(NodeRec));
  const NodeRec* pols = (const NodeRec*)p;
  p += align16((size_t)h.n_pols * sizeof(NodeRec));
  const NodeRec* rules = (const NodeRec*)p;
  p += align16((size_t)h.n_rules * sizeof(NodeRec));
  const RuleResAttr* rres = (const RuleResAttr*)p;
  (void)n_bytes;  // the caller checked that every section lies inside the blob
  auto node_ok = [&](const NodeRec& t) {
    return (uint64_t)t.subj_off + t.subj_n <= h.n_pairs && (uint64_t)t.act_off + t.act_n <= h.n_pairs &&
           (uint64_t)t.res_off + t.res_n <= h.n_rres && (uint64_t)t.acl_roles_off + t.acl_roles_n <= h.n_u32pool;
  };
  for (uint32_t s = 0; s < h.n_sets; ++s) {
    const NodeRec t = sets[s];
    if (!node_ok(t) || t.child_begin > t.child_end || t.child_end > h.n_pols) return bad("image: policy set", s);
  }
  for (uint32_t q = 0; q < h.n_pols; ++q) {
    const NodeRec t = pols[q];
    if (!node_ok(t) || t.child_begin > t.child_end || t.child_end > h.n_rules || t.fe < t.child_begin ||
        t.fe > t.child_end)
      return bad("image: policy", q);
  }
  // rules and rule attributes over the host threads (c5: 1M rules)
  const size_t first_bad = parallel_first_bad(h.n_rules, [&](size_t lo, size_t hi) {
    for (size_t r = lo; r < hi; ++r)
      if (!node_ok(rules[r])) return r;
    return (size_t)h.n_rules;
  });
  if (first_bad < h.n_rules) return bad("image: rule", first_bad);
  std::atomic<uint32_t> rows{0};
  parallel_first_bad(h.n_rres, [&](size_t lo, size_t hi) {
    uint32_t m = 0;
    for (size_t k = lo; k < hi; ++k)
      if ((rres[k].kind & K_ENT_LOOSE) && (uint32_t)rres[k].row + 1 > m) m = (uint32_t)rres[k].row + 1;
    for (uint32_t v = rows.load(); v < m && !rows.compare_exchange_weak(v, m);) {
    }
    return (size_t)h.n_rres;
  });
  *rx_rows_min = rows.load();
  return 0;
}

// Batch checks for the host-buffer entry points.  SoA batches (+ optional lines equal to
// their rows) and compact batches (lines + extension records) alike.
int acs_internal_check_batch2(const acs_req_batch* b, uint32_t n_sets, uint32_t n_pols, uint32_t n_rules,
                              uint32_t rx_rows_min, uint32_t* arena_end);

int acs_internal_check_batch(const acs_req_batch* b, uint32_t n_sets, uint32_t n_pols, uint32_t n_rules,
                             uint32_t rx_rows_min) {
  return acs_internal_check_batch2(b, n_sets, n_pols, n_rules, rx_rows_min, nullptr);
}

// arena_end (optional, [n]): one past the last arena word request i's records occupy (the
// multi-device split uploads each shard's arena words only).
int acs_internal_check_batch2(const acs_req_batch* b, uint32_t n_sets, uint32_t n_pols, uint32_t n_rules,
                              uint32_t rx_rows_min, uint32_t* arena_end) {
  const size_t n = b->n;
  if (n == 0) return 0;
  const bool compact = b->hdr == nullptr;
  if (compact) {
    if (b->res || b->subj || b->act || b->roles) return bad("batch: partial SoA rows", 0);
    if (!b->lines) return bad("batch: compact batch without request lines", 0);
  } else if (!b->res || !b->subj || !b->act || !b->roles) {
    return bad("batch: null request buffer", 0);
  }
  if (!b->arena) return bad("batch: null request buffer", 0);
  if (rx_rows_min && (!b->rx || b->rx_rows < rx_rows_min)) return bad("batch: regex matrix rows", b->rx_rows);
  if (b->cand) {
    if (b->cand_wp < words32(n_sets) || b->cand_wr < b->cand_wp + words32(n_pols) ||
        b->cand_words < b->cand_wr + words32(n_rules))
      return bad("batch: candidate row layout", b->cand_words);
    if ((b->cand_wsu && b->cand_wsu + words32(n_sets) > b->cand_words) ||
        (b->cand_wpu && b->cand_wpu + words32(n_pols) > b->cand_words) ||
        (b->cand_wv && (uint64_t)b->cand_wv + 4ull * words32(n_pols) + words32(n_rules) > b->cand_words))
      return bad("batch: candidate row layout", b->cand_words);
    if (b->role_key && !b->role_rows_bits && b->role_rows) return bad("batch: role factor rows", 0);
    // role keys pack two row indices in 16 bits each, 0xFFFF meaning "no role filtering"
    if (b->role_key && b->role_rows >= 0xFFFFu) return bad("batch: role factor rows", b->role_rows);
  }
  // the encoder's coherence order: every request exactly once, holes 0xFFFFFFFF (the kernels
  // skip an index >= n; a request missing from it would leave its record unwritten)
  if (b->perm) {
    if (b->perm_lanes < n || b->perm_lanes > 0xFFFFFFFFull) return bad("batch: perm_lanes", b->perm_lanes);
    std::vector<std::atomic<uint8_t>> seen(n);
    for (auto& x : seen) x.store(0, std::memory_order_relaxed);
    std::atomic<size_t> got{0};
    const size_t at = parallel_first_bad(b->perm_lanes, [&](size_t lo, size_t hi) -> size_t {
      size_t mine = 0;
      for (size_t x = lo; x < hi; ++x) {
        const uint32_t i = b->perm[x];
        if (i == 0xFFFFFFFFu) continue;
        if (i >= n || seen[i].exchange(1, std::memory_order_relaxed)) return x;
        ++mine;
      }
      got += mine;
      return b->perm_lanes;
    });
    if (at < b->perm_lanes) return bad("batch: perm (an index outside the batch, or twice)", at);
    if (got != n) return bad("batch: perm misses requests", got);
  }
  // RES_RX_SAFE on an attribute lets K1 stop early (the clean-below set walk, the final-fold
  // cuts): it claims that no cell of the value's regex-matrix column throws or needs the host.
  // Checked per column once (RX_THROW_TYPE | RX_THROW_SYNTAX | RX_HOST = 4 | 8 | 16).
  std::vector<uint8_t> col_unsafe;
  if (rx_rows_min && b->rx) {
    col_unsafe.assign(b->rx_cols, 0);
    for (size_t c = 0; c < b->rx_cols; ++c)
      for (size_t r = 0; r < b->rx_rows; ++r)
        if (b->rx[c * b->rx_rows + r] & 0x1Cu) {
          col_unsafe[c] = 1;
          break;
        }
  }
  const ReqHdr* hdr = (const ReqHdr*)b->hdr;
  const ReqRes* res = (const ReqRes*)b->res;
  const size_t W = b->arena_words;
  const ReqLine* lines = (const ReqLine*)b->lines;
  // one request's checks: nullptr, or what is malformed (the per-request loop runs on host threads)
  auto check_one = [&](size_t i) -> const char* {
    const ReqHdr hd = compact ? lines[i].h : hdr[i];
    if (hd.nres > QMAX || hd.nsubj > SMAX || hd.nact > AMAX || hd.nroles > RMAX) return "batch: counts";
    const size_t o = hd.arena_off;
    if (o + 2 > W) return "batch: arena offset";
    const uint32_t* ar = b->arena + o;
    const size_t room = W - o;
    const bool live = !(hd.flags & (RQ_HOST | RQ_NO_TARGET));
    // the rows past the line: extension record of a compact batch
    const uint32_t* ex = nullptr;
    if (compact) {
      const ExtGeom g = ext_geom(hd.nres, hd.nsubj, hd.nact, hd.nroles);
      if (g.words) {
        const uint32_t e = lines[i].ext;
        if (!e || !b->ext || ((size_t)e - 1) * 4 + g.words > b->ext_words) return "batch: extension record";
        ex = b->ext + ((size_t)e - 1) * 4;
      }
      if (lines[i].ar0 != (live ? ar[0] : 0u) || lines[i].ar1 != (live ? ar[1] : 0u))
        return "batch: request line arena counts";
    } else if (lines) {  // the packed line must equal the SoA rows (K1 trusts it for addressing)
      ReqLine want{};
      want.h = hd;
      for (uint32_t j = 0; j < hd.nres && j < (uint32_t)LINE_RES; ++j) want.res[j] = res[j * n + i];
      const Pair* subj = (const Pair*)b->subj;
      const Pair* act = (const Pair*)b->act;
      if (hd.nsubj > 0) want.s0 = subj[i];
      if (hd.nsubj > 1) want.s1 = subj[n + i];
      if (hd.nact > 0) want.a0 = act[i];
      if (hd.nroles > 0) want.r0 = b->roles[i];
      if (hd.nroles > 1) want.r1 = b->roles[n + i];
      if (live) {
        want.ar0 = ar[0];
        want.ar1 = ar[1];
      }
      want.ext = lines[i].ext;  // (an SoA batch reads its rows, not extension records)
      want.cls2 = lines[i].cls2;  // (a class fact, not a row: checked below)
      if (std::memcmp(&want, &lines[i], sizeof want) != 0) return "batch: request line differs from its rows";
    }
    auto res_at = [&](uint32_t j) -> ReqRes {
      if (!compact) return res[(size_t)j * n + i];
      if (j < (uint32_t)LINE_RES) return lines[i].res[j];
      ReqRes q;
      std::memcpy(&q, ex + 4 * (j - LINE_RES), sizeof q);
      return q;
    };
    const uint32_t c0 = ar[0], c1 = ar[1];
    const uint32_t ng = c0 & 0xFF, nre = (c0 >> 8) & 0xFF, ns = (c0 >> 16) & 0xFF, nro = c0 >> 24;
    const uint32_t nt = c1 & 0xFF, nh = (c1 >> 8) & 0xFF;
    if (nro > MAX_ROOTS || nh > MAX_HRKEYS || ns > MAX_SLOTS) return "batch: arena header";
    const size_t head = 2 + 3 * (size_t)ng + 2 * (size_t)nre + nro + nh + ns + 3 * (size_t)nt;
    if (head > room) return "batch: arena header";
    size_t used = head;  // words of this request's records past its offset
    const uint32_t* slotoff = ar + 2 + 3 * ng + 2 * nre + nro + nh;
    const uint32_t* tse = slotoff + ns;
    for (uint32_t s = 0; s < ns; ++s) {  // [owners_empty, n_owners, owner...]
      size_t at = slotoff[s];
      if (at + 2 > room) return "batch: arena slot record";
      const uint32_t no = ar[at + 1];
      at += 2;
      for (uint32_t k = 0; k < no; ++k) {  // [is_oe | n_attrs << 8, value, n_attrs x 3]
        if (at + 2 > room) return "batch: arena owner record";
        at += 2 + 3 * (size_t)(ar[at] >> 8);
        if (at > room) return "batch: arena owner record";
      }
      if (at > used) used = at;
    }
    for (uint32_t e = 0; e < nt; ++e) {  // (se, n_inst, inst_rel_off) -> n_inst x 2
      const uint32_t ni = tse[3 * e + 1];
      if (ni > 32 || (size_t)tse[3 * e + 2] + 2 * (size_t)ni > room) return "batch: arena instance list";
      if ((size_t)tse[3 * e + 2] + 2 * (size_t)ni > used) used = (size_t)tse[3 * e + 2] + 2 * (size_t)ni;
    }
    if (arena_end) arena_end[i] = (uint32_t)(o + used);
    // composed class rows: a second class needs a valid first one, and no role factor
    if (lines && lines[i].cls2) {
      const uint32_t c1 = hd.flags >> RQ_PCOL_SHIFT, c2 = lines[i].cls2 - 1u;
      if (!b->cand || b->role_key || c1 >= b->cand_rows || c2 >= b->cand_rows) return "batch: second class row";
    }
    const uint32_t ent = (hd.flags >> RQ_ENT_SHIFT) & 7u;
    const uint32_t e0 = ent >= 1 && ent <= 6 ? ent - 1 : (uint32_t)QMAX;  // the lone entity attr's slot
    if (compact && e0 < QMAX && e0 >= hd.nres) return "batch: entity slot";
    for (uint32_t j = 0; j < QMAX; ++j) {
      if (j >= hd.nres && j != e0) continue;
      const ReqRes q = res_at(j);
      if (rx_rows_min && ((q.kind & K_ENT_LOOSE) || j == e0) && q.col >= b->rx_cols)
        return "batch: regex matrix column";
      if (!col_unsafe.empty() && (q.kind & K_ENT_LOOSE) && (q.pad & RES_RX_SAFE) && col_unsafe[q.col])
        return "batch: RES_RX_SAFE on a regex column that throws or needs the host";
      if ((q.slot_a != NONE8 && q.slot_a >= ns) || (q.slot_b != NONE8 && q.slot_b >= ns))
        return "batch: context resource slot";
    }
    return nullptr;
  };
  const size_t first = parallel_first_bad(n, [&](size_t lo, size_t hi) -> size_t {
    for (size_t i = lo; i < hi; ++i)
      if (check_one(i)) return i;
    return n;
  });
  if (first < n) return bad(check_one(first), first);
  return 0;
}

// ACL_NONE (acs_layout.h) is a claim K1 acts on (it skips ACL-gated rules and ACL-inert sets):
// verifyACL (verifyACL.ts:89-251) is false for every rule, rule-independently, without an error.
// Recomputed here from what verify_acl itself reads — the flags, the ACL instance lists, the
// grants and the role-scoping pairs of the request's arena (encoder._acl_none,
// acs_codec.cpp's ACL_NONE block) — and a request whose arena does not support it is rejected.
// id_user: the image's interned urns.user.  Run after acs_internal_check_batch (arena bounds).
int acs_internal_check_acl_none(const acs_req_batch* b, uint32_t id_user) {
  const size_t n = b->n;
  const bool compact = b->hdr == nullptr;
  const ReqHdr* hdr = (const ReqHdr*)b->hdr;
  const ReqLine* lines = (const ReqLine*)b->lines;
  // one request: nullptr, or why its ACL_NONE claim does not hold (the loop runs on host threads)
  auto check_one = [&](size_t i) -> const char* {
    const ReqHdr hd = compact ? lines[i].h : hdr[i];
    if (((hd.flags >> RQ_ACL_SHIFT) & 3u) != ACL_NONE || (hd.flags & (RQ_HOST | RQ_NO_TARGET))) return nullptr;
    const uint32_t f = hd.flags;
    if ((f & RQ_SUBJ_MISSING) || !((f & RQ_RA_EMPTY) || (f & RQ_HRS_ITERABLE)))
      return "batch: ACL_NONE on a request whose verifyACL can throw";
    if ((f & RQ_RA_EMPTY) || !(f & (RQ_ACT_CREATE | RQ_ACT_RMD))) return nullptr;  // false for every rule
    const uint32_t* ar = b->arena + hd.arena_off;
    const uint32_t c0 = ar[0], c1 = ar[1];
    const uint32_t ng = c0 & 0xFF, nre = (c0 >> 8) & 0xFF, ns = (c0 >> 16) & 0xFF, nro = c0 >> 24;
    const uint32_t nt = c1 & 0xFF, nh = (c1 >> 8) & 0xFF;
    const uint32_t* grants = ar + 2;
    const uint32_t* rolese = grants + 3 * ng;
    const uint32_t* tse = rolese + 2 * nre + nro + nh + ns;
    bool none;
    if (nt == 0) {
      none = false;  // verifyACL returns true when no ACL entity is left to check
    } else if (f & RQ_ACT_CREATE) {
      none = false;
      for (uint32_t e = 0; e < nt && !none; ++e) {
        const uint32_t se = tse[3 * e];
        if (se == id_user) continue;
        bool scoped = false;
        for (uint32_t k = 0; k < nre && !scoped; ++k) scoped = rolese[2 * k + 1] == se;
        if (!scoped) none = true;
      }
    } else {  // read / modify / delete: no instance is the subject (user entity) or a grant's
      none = true;
      for (uint32_t e = 0; e < nt && none; ++e) {
        const uint32_t se = tse[3 * e], ni = tse[3 * e + 1];
        const uint32_t* inst = ar + tse[3 * e + 2];
        for (uint32_t x = 0; x < ni && none; ++x) {
          if (se == id_user && inst[2 * x] == hd.subject_id) none = false;
          for (uint32_t g = 0; g < ng && none; ++g)
            if (grants[3 * g + 1] == se && grants[3 * g + 2] == inst[2 * x]) none = false;
        }
      }
    }
    return none ? nullptr : "batch: ACL_NONE on a request whose ACLs can let a rule pass";
  };
  const size_t first = parallel_first_bad(n, [&](size_t lo, size_t hi) -> size_t {
    for (size_t i = lo; i < hi; ++i)
      if (check_one(i)) return i;
    return n;
  });
  if (first < n) return bad(check_one(first), first);
  return 0;
}

// The slices of a compact batch that requests [lo, hi) read (the multi-device split uploads
// only these): plan[0..1] = arena words [a0, a1), plan[2..3] = extension words [e0, e1).
// arena_end from acs_internal_check_batch2.  Empty ranges are [0, 0).
void acs_internal_shard_plan(const acs_req_batch* b, size_t lo, size_t hi, const uint32_t* arena_end, size_t plan[4]) {
  const ReqLine* L = (const ReqLine*)b->lines;
  // min / max over the range, in parts over the pool (a 625k-request chunk reads 80 MB of lines)
  const size_t m = hi > lo ? hi - lo : 0;
  size_t T = std::thread::hardware_concurrency();
  T = T < 1 ? 1 : (T > 16 ? 16 : T);
  if (T > m / 16384 + 1) T = m / 16384 + 1;
  std::vector<size_t> part(4 * T);
  acs_pool::run((int)T, [&](int t) {
    size_t a0 = ~size_t(0), a1 = 0, e0 = ~size_t(0), e1 = 0;
    for (size_t i = lo + m * t / T; i < lo + m * (t + 1) / T; ++i) {
      const ReqHdr& h = L[i].h;
      if (arena_end[i] > h.arena_off) {
        a0 = h.arena_off < a0 ? h.arena_off : a0;
        a1 = arena_end[i] > a1 ? arena_end[i] : a1;
      }
      if (L[i].ext) {
        const size_t x = (size_t)(L[i].ext - 1) * 4, w = ext_geom(h.nres, h.nsubj, h.nact, h.nroles).words;
        e0 = x < e0 ? x : e0;
        e1 = x + w > e1 ? x + w : e1;
      }
    }
    part[4 * t] = a0;
    part[4 * t + 1] = a1;
    part[4 * t + 2] = e0;
    part[4 * t + 3] = e1;
  }, true);
  size_t a0 = ~size_t(0), a1 = 0, e0 = ~size_t(0), e1 = 0;
  for (size_t t = 0; t < T; ++t) {
    a0 = std::min(a0, part[4 * t]);
    a1 = std::max(a1, part[4 * t + 1]);
    e0 = std::min(e0, part[4 * t + 2]);
    e1 = std::max(e1, part[4 * t + 3]);
  }
  if (a0 > a1) a0 = a1 = 0;
  if (e0 > e1) e0 = e1 = 0;
  plan[0] = a0;
  plan[1] = a1;
  plan[2] = e0;
  plan[3] = e1;
}

}  // extern "C"
