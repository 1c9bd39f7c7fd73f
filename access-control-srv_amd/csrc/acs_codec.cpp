// acs_codec.cpp — native request codec of the MI355X evaluator (C ABI: include/acs_mi355x.h).
//
// JSON requests in the shape the reference's AccessControlService hands to
// AccessController.isAllowed / whatIsAllowed (src/accessControlService.ts:62-125) ->
// the packed batch the kernels read (csrc/acs_layout.h), on host threads.  It restates
// acs_mi355x/encoder.py + candidates.py (the Python encoder the tests pin against the
// oracle) function for function; every sub-expression of the reference that depends on
// the request alone is evaluated here once:
//
//   attribute-id kinds against the URN config            accessController.ts:493-574
//   lodash _.find context-resource lookups -> slots      hierarchicalScope.ts:106-133, verifyACL.ts:40-48
//   the verifyACL request loop -> 2-bit outcome + map    verifyACL.ts:37-88
//   role associations -> grants / (role, entity) pairs   hierarchicalScope.ts:166-181,222-238, verifyACL.ts:104-125
//   hierarchical_scopes -> per-root / per-role org sets  hierarchicalScope.ts:199-245, verifyACL.ts:129-145
//   indexOf / '#'-suffix / namespace-RegExp cells        accessController.ts:509-574
//   candidate classes (entity x roles x action)          candidates.py
//
// Per-subject HR cache (accessController.ts:735-783 keeps HR scopes per subject in Redis):
// a forest is flattened ONCE per distinct version — keyed by its exact JSON text for inline
// `hierarchical_scopes`, or registered per subject key (acs_codec_set_subject_scopes, the
// createHRScope / evictHRScopes counterpart) — into its root / role-key lists and, per org
// id, the bit masks of the roots whose subtree (Euler interval of the DFS) holds it.  A
// request then costs one hash lookup per owner instance instead of a tree walk.
#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cstring>
#include <deque>
#include <memory>
#include <mutex>
#include <regex>
#include <shared_mutex>
#include <string>
#include <string_view>
#include <thread>
#include <emmintrin.h>
#include <sys/mman.h>
#include <unordered_map>
#include <vector>

#include "../../include/acs_mi355x.h"
#include "acs_json.h"
#include "acs_layout.h"
#include "acs_pool.h"

extern "C" void acs_internal_set_error(const char* msg);
// acs_kernels.hip: page-locked (portable) host memory when a device is present, else malloc
extern "C" void* acs_internal_host_alloc(size_t bytes, int* pinned);
extern "C" void acs_internal_host_free(void* p, int pinned);

using namespace acs;
using namespace acs_json;

namespace {

struct Unsup {
  const char* why;
};
[[noreturn]] void unsup(const char* why) { throw Unsup{why}; }

enum UrnName {
  U_ENT, U_PROP, U_OP, U_RID, U_ACTID, U_ROLE, U_RSE, U_RSI, U_HRS, U_OE, U_OI, U_ACLIE, U_ACLI, U_CREATE,
  U_READ, U_MODIFY, U_DELETE, U_USER, U_SKIPACL, U_MASKED, U_COUNT
};

constexpr uint32_t CODEC_MAGIC = 0x43534341u, CODEC_VERSION = 2u;
constexpr uint8_t HIT_LIKE = 1 | 4 | 8 | 16;  // RX_HIT | RX_THROW_TYPE | RX_THROW_SYNTAX | RX_HOST
constexpr uint8_t C_RX_HIT = 1, C_RX_RESET = 2, C_RX_THROW_TYPE = 4, C_RX_THROW_SYNTAX = 8, C_RX_HOST = 16;
constexpr uint32_t LOCAL_BITS = 24;  // per-thread batch-local id range

inline uint32_t words_of(uint32_t n) { return (n + 31) / 32; }

// ------------------------------------------------------------------ regex cells
// regex.py restated: literal patterns by substring search, a metacharacter subset by
// std::regex (ECMAScript: `$` is end of input, as in V8) after rejecting the stacked
// quantifiers V8 rejects, everything else (and any non-ASCII text) -> the host.  Pinned
// against V8 by tests/golden/regex_cells.json (tests/test_codec.py).
bool in_literal_set(unsigned char c) {
  if ((c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9')) return true;
  return strchr("_- \t\n\r\f\v\x1c\x1d\x1e\x1f#@%&=,;'\"<>~`!", c) != nullptr && c != 0;
}
bool in_safe_set(unsigned char c) {
  if ((c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9')) return true;
  return c != 0 && strchr("_-*+?|()[]^$", c) != nullptr;
}
bool is_ascii(std::string_view s) {
  for (unsigned char c : s)
    if (c >= 0x80) return false;
  return true;
}

struct RxPattern {  // one rule entity value (a regex-matrix row), prepared once
  bool nullish = false, ascii = true;
  std::string prefix, last;  // namespace prefix (before the last ':'), last dot segment
  bool has_ns = false;
  std::string ns_upper;
  int mode = 0;  // 0 literal, 1 regex, 2 host, 3 syntax error
  std::unique_ptr<std::regex> rx;
};

std::string upper_ascii(std::string_view s) {
  std::string o(s);
  for (char& c : o)
    if (c >= 'a' && c <= 'z') c = (char)(c - 32);
  return o;
}

void split_entity(std::string_view v, std::string& prefix, std::string_view& first, std::string_view& last) {
  const size_t c = v.rfind(':');
  prefix = c == std::string_view::npos ? std::string() : std::string(v.substr(0, c));
  const std::string_view pat = c == std::string_view::npos ? v : v.substr(c + 1);
  const size_t d0 = pat.find('.'), d1 = pat.rfind('.');
  first = d0 == std::string_view::npos ? pat : pat.substr(0, d0);
  last = d1 == std::string_view::npos ? pat : pat.substr(d1 + 1);
}

void prepare_pattern(RxPattern& P, bool nullish_v, std::string_view v) {
  P.nullish = nullish_v;
  if (nullish_v) return;
  P.ascii = is_ascii(v);
  if (!P.ascii) return;
  std::string_view first, last;
  split_entity(v, P.prefix, first, last);
  P.last = std::string(last);
  const std::string fu = upper_ascii(first), lu = upper_ascii(last);
  P.has_ns = fu != lu && !fu.empty();
  if (P.has_ns) P.ns_upper = fu;
  const std::string& p = P.last;
  bool lit = true, safe = true;
  for (unsigned char c : p) {
    lit = lit && in_literal_set(c);
    safe = safe && in_safe_set(c);
  }
  if (lit) {
    P.mode = 0;
    return;
  }
  if (!safe || p.find("(?") != std::string::npos || p.find("[]") != std::string::npos ||
      p.find("[^]") != std::string::npos) {
    P.mode = 2;
    return;
  }
  // a quantifier right after a quantifier (other than one lazy '?') is a V8 SyntaxError
  bool in_class = false;
  int quant = 0;
  for (char c : p) {
    if (in_class) {
      in_class = c != ']';
      continue;
    }
    if (c == '*' || c == '+' || c == '?') {
      if (quant == 1 && c == '?') quant = 2;
      else if (quant) {
        P.mode = 3;
        return;
      } else quant = 1;
      continue;
    }
    quant = 0;
    if (c == '[') in_class = true;
  }
  try {
    P.rx.reset(new std::regex(p, std::regex::ECMAScript));
    P.mode = 1;
  } catch (const std::regex_error&) {
    P.mode = 3;
  }
}

uint8_t rx_cell(const RxPattern& R, bool q_nullish, std::string_view q) {
  if (R.nullish || q_nullish) return C_RX_THROW_TYPE;
  if (!R.ascii || !is_ascii(q)) return C_RX_HOST;
  std::string qprefix;
  std::string_view qfirst, qlast;
  split_entity(q, qprefix, qfirst, qlast);
  uint8_t bits = qprefix != R.prefix ? C_RX_RESET : 0;
  const std::string qfu = upper_ascii(qfirst), qlu = upper_ascii(qlast);
  const bool q_ns = qfu != qlu && !qfu.empty();
  if ((q_ns && R.has_ns && qfu == R.ns_upper) || (!q_ns && !R.has_ns)) {
    switch (R.mode) {
      case 0:
        if (qlast.find(R.last) != std::string_view::npos) bits |= C_RX_HIT;
        break;
      case 1:
        if (std::regex_search(qlast.begin(), qlast.end(), *R.rx)) bits |= C_RX_HIT;
        break;
      case 2: bits |= C_RX_HOST; break;       // (regex.py keeps the reset bit beside it; the
      default: bits |= C_RX_THROW_SYNTAX;     //  kernel tests the throw / host bits first)
    }
  }
  return bits;
}

// ------------------------------------------------------------------ string hashing
// 8 bytes per multiply-xorshift step: the codec hashes ~25 URNs / ids per request, and
// std::hash's bytewise loop over 40-60 byte URNs was a visible share of encode time.
inline uint64_t fast_hash(const char* p, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xC2B2AE3D27D4EB4Full);
  size_t k = 0;
  for (; k + 8 <= n; k += 8) {
    uint64_t w;
    memcpy(&w, p + k, 8);
    h = (h ^ w) * 0xFF51AFD7ED558CCDull;
    h ^= h >> 31;
  }
  uint64_t w = 0;
  memcpy(&w, p + k, n - k);
  h = (h ^ w) * 0xC4CEB9FE1A85EC53ull;
  h ^= h >> 29;
  return h;
}
struct FastHash {
  size_t operator()(std::string_view s) const { return (size_t)fast_hash(s.data(), s.size()); }
  size_t operator()(const std::string& s) const { return (size_t)fast_hash(s.data(), s.size()); }
};

// String -> V, open addressing with the hash stored in the slot: a lookup is one probe run
// over a flat array (no node chasing, no allocation per insert).  Keys are views: their bytes
// must outlive the map (the dictionary's bytes, a StrPool, or the request text of a batch).
template <class V>
class StrMap {
 public:
  struct Slot {
    uint64_t h;
    const char* p;
    uint32_t n;  // 0xFFFFFFFF: empty
    V v;
  };
  explicit StrMap(size_t expect = 16) { rehash(expect); }
  const Slot* find(uint64_t h, std::string_view s) const {
    for (size_t x = h & mask_;; x = (x + 1) & mask_) {
      const Slot& e = t_[x];
      if (e.n == EMPTY) return nullptr;
      if (e.h == h && e.n == s.size() && memcmp(e.p, s.data(), s.size()) == 0) return &e;
    }
  }
  const Slot* find(std::string_view s) const { return find(fast_hash(s.data(), s.size()), s); }
  Slot* insert(uint64_t h, const char* p, uint32_t n, const V& v) {  // the key must be absent
    if (2 * (size_ + 1) > t_.size()) rehash(size_ + 1);
    size_t x = h & mask_;
    while (t_[x].n != EMPTY) x = (x + 1) & mask_;
    t_[x] = Slot{h, p, n, v};
    ++size_;
    return &t_[x];
  }
  size_t size() const { return size_; }
  void clear() {
    for (Slot& e : t_) e.n = EMPTY;
    size_ = 0;
  }

 private:
  static constexpr uint32_t EMPTY = 0xFFFFFFFFu;
  void rehash(size_t expect) {
    size_t cap = 16;
    while (cap < 2 * expect) cap <<= 1;
    std::vector<Slot> old(std::move(t_));
    t_.assign(cap, Slot{0, nullptr, EMPTY, V{}});
    mask_ = cap - 1;
    size_ = 0;
    for (const Slot& e : old)
      if (e.n != EMPTY) insert(e.h, e.p, e.n, e.v);
  }
  std::vector<Slot> t_;
  size_t mask_ = 0, size_ = 0;
};

// Stable bump storage for strings (chunks never move).
class StrPool {
 public:
  const char* put(std::string_view s) {
    if (s.size() > CHUNK) {
      big_.emplace_back(s);
      return big_.back().data();
    }
    if (chunks_.empty() || used_ + s.size() > CHUNK) {
      chunks_.emplace_back(new char[CHUNK]);
      used_ = 0;
    }
    char* d = chunks_.back().get() + used_;
    memcpy(d, s.data(), s.size());
    used_ += s.size();
    return d;
  }

 private:
  static constexpr size_t CHUNK = size_t(1) << 16;
  std::vector<std::unique_ptr<char[]>> chunks_;
  std::deque<std::string> big_;
  size_t used_ = 0;
};

// ------------------------------------------------------------------ HR forests
struct Scalar {
  uint8_t kind = 0;  // 0 undefined, 1 null, 2 string
  std::string s;
};

struct HrForest {
  const char* why = nullptr;  // non-null: the request goes to the host (Unsupported)
  bool is_array = false;
  std::vector<Scalar> roots;  // hierarchical_scopes[i].role
  std::vector<Scalar> keys;   // verifyACL effective-role keys, first-seen order
  StrPool ids;                // storage of the org ids `masks` is keyed by
  StrMap<uint64_t> masks;     // org id -> root bits | key bits << 32 (flat: one probe run per owner lookup)
  std::string text;           // inline forests: the exact JSON text they were built from
  size_t bytes() const { return text.size() + masks.size() * 64 + 256; }
  uint64_t mask(std::string_view id) const {
    const auto* e = masks.find(id);
    return e ? e->v : 0;
  }
};

Scalar scalar_of(const JV* v) {
  Scalar s;
  if (v->t == J_UNDEF) s.kind = 0;
  else if (v->t == J_NULL) s.kind = 1;
  else if (v->t == J_STR) {
    s.kind = 2;
    s.s.assign(v->s, v->n);
  } else unsup("non-string attribute scalar");
  return s;
}

bool scalar_eq(const Scalar& a, const Scalar& b) { return a.kind == b.kind && (a.kind != 2 || a.s == b.s); }

// hierarchicalScope.ts:199-245 / verifyACL.ts:129-145, as encoder.py's walk(): a preorder
// DFS of every root (the root's Euler interval), collecting per org id the bits of the roots
// whose subtree holds it and of its effective role key (the nearest ancestor-or-self
// `role`, first-seen order across the forest, verifyACL's roleWithOrgScopesMap keys).
void build_forest(HrForest& F, const JV* hrs) {
  try {
    if (hrs->t != J_ARR) {
      if (!nullish(hrs)) unsup("hierarchical_scopes is not an array");
      return;
    }
    F.is_array = true;
    if (hrs->n > (uint32_t)MAX_ROOTS) unsup("too many HR scope roots");
    for (uint32_t r = 0; r < hrs->n; ++r)
      if (hrs->a[r].t != J_OBJ) unsup("non-object entry in hierarchical_scopes");
    std::vector<Scalar> vals(1);   // distinct inherited role values; [0] = undefined
    std::vector<int> val_key(1, -1);
    auto val_index = [&](const JV* role) -> int {
      const Scalar x = scalar_of(role);
      for (size_t k = 0; k < vals.size(); ++k)
        if (scalar_eq(vals[k], x)) return (int)k;
      vals.push_back(x);
      val_key.push_back(-1);
      return (int)vals.size() - 1;
    };
    struct Item {
      const JV* node;
      int vi;
    };
    std::vector<Item> stack;
    for (uint32_t r = 0; r < hrs->n; ++r) {
      const JV* root = &hrs->a[r];
      F.roots.push_back(scalar_of(get(root, "role")));
      stack.assign(1, Item{root, 0});
      while (!stack.empty()) {
        const Item it = stack.back();
        stack.pop_back();
        const JV* h = it.node;
        if (h->t != J_OBJ) unsup("non-object entry in hierarchical scope nodes");
        const JV* role = get(h, "role");
        const int vi = nullish(role) ? it.vi : val_index(role);
        const JV* hid = get(h, "id");
        if (truthy(hid)) {
          if (val_key[vi] < 0) {
            if (F.keys.size() >= (size_t)MAX_HRKEYS) unsup("too many HR effective roles");
            val_key[vi] = (int)F.keys.size();
            F.keys.push_back(vals[vi]);
          }
          if (hid->t == J_STR) {
            const std::string_view sid = hid->str();
            const uint64_t h = fast_hash(sid.data(), sid.size());
            auto* e = const_cast<StrMap<uint64_t>::Slot*>(F.masks.find(h, sid));
            if (!e) e = F.masks.insert(h, F.ids.put(sid), (uint32_t)sid.size(), 0ull);
            e->v |= (1ull << r) | (1ull << (32 + val_key[vi]));
          }
        }
        const JV* ch = get(h, "children");
        if (ch->t == J_ARR) {
          for (uint32_t k = ch->n; k-- > 0;) stack.push_back({&ch->a[k], vi});
        } else if (ch->t == J_STR) {
          if (ch->n) unsup("hierarchical scope nodes is not an array");
        } else if (ch->t == J_OBJ) {
          if (truthy(get(ch, "length"))) unsup("hierarchical scope nodes is not an array");
        }
      }
    }
  } catch (const Unsup& u) {
    F.why = u.why;
  }
}

}  // namespace

// ------------------------------------------------------------------ host buffers
namespace {
// The big arrays of an encoded batch (request lines, extension records, arena, class rows)
// live in page-locked host memory, so acs_is_allowed's copies to the device run at full PCIe
// speed without a staging copy.  Pinning is slow, so blocks are recycled across batches.
struct HostBlock {
  void* p = nullptr;
  size_t bytes = 0;
  int pinned = 0;
};

class HostPool {
 public:
  ~HostPool() {
    for (HostBlock& b : free_) acs_internal_host_free(b.p, b.pinned);
  }
  HostBlock acquire(size_t bytes) {
    if (bytes < 256) bytes = 256;
    {
      std::lock_guard<std::mutex> lock(mu_);
      size_t best = free_.size();
      for (size_t k = 0; k < free_.size(); ++k)
        if (free_[k].bytes >= bytes && free_[k].bytes <= 4 * bytes &&
            (best == free_.size() || free_[k].bytes < free_[best].bytes))
          best = k;
      if (best < free_.size()) {
        HostBlock b = free_[best];
        free_.erase(free_.begin() + (ptrdiff_t)best);
        held_ -= b.bytes;
        return b;
      }
    }
    HostBlock b;
    b.bytes = ((bytes + bytes / 8) + 4095) & ~size_t(4095);  // headroom for the next, slightly larger batch
    b.p = acs_internal_host_alloc(b.bytes, &b.pinned);
    if (!b.p) throw std::bad_alloc();
    return b;
  }
  void release(HostBlock& b) {
    if (!b.p) return;
    std::lock_guard<std::mutex> lock(mu_);
    while (!free_.empty() && held_ + b.bytes > HOLD_MAX) {  // drop the oldest
      acs_internal_host_free(free_.front().p, free_.front().pinned);
      held_ -= free_.front().bytes;
      free_.erase(free_.begin());
    }
    free_.push_back(b);
    held_ += b.bytes;
    b = HostBlock{};
  }

 private:
  static constexpr size_t HOLD_MAX = size_t(8) << 30;
  std::mutex mu_;
  std::vector<HostBlock> free_;
  size_t held_ = 0;
};
}  // namespace

namespace {
// Candidate-class rows, cached per codec (= per store version) across batches: a class row
// is a pure function of its key (entity value, action, role-association set, key level) and
// of the image, so a steady stream of requests computes each row once (c3: ~15k keys, each
// ~200 us of bit work; per-batch recomputation was 0.39 s per 1M requests on 16 threads).
// Rows are interned by content: keys whose rows coincide share one entry (one class).
struct ClassEntry {
  std::vector<uint32_t> row;
  uint32_t cost = 0;  // candidate nodes in the filter sections (heaviest classes first)
};
struct ClassCache {
  std::shared_mutex mu;
  std::unordered_map<std::string, std::shared_ptr<const ClassEntry>> by_key;
  std::unordered_map<uint64_t, std::vector<std::shared_ptr<const ClassEntry>>> by_row;
  std::unordered_map<std::string, std::shared_ptr<const std::vector<uint32_t>>> role_rows;  // role factor
  size_t bytes = 0;
  static constexpr size_t MAX_BYTES = size_t(2) << 30;
  void clear_locked() {  // batches hold their own references to the rows they use
    by_key.clear();
    by_row.clear();
    role_rows.clear();
    bytes = 0;
  }
};
}  // namespace

// ------------------------------------------------------------------ the codec (per store image)
struct acs_codec {
  // store image
  uint32_t S = 0, P = 0, R = 0, ws = 0, wp = 0, wr = 0, W = 0;
  // sets | policies | rules (uninitialised storage: codec_load fills it, in parallel)
  // Large stores: 2-MB pages (MADV_HUGEPAGE) — a c5 load faulted in 65 MB of 4-KB pages, the
  // kernel's page-fault path serialising the copy (~70 ms, no gain from more threads)
  struct NodeTable {
    struct Free {
      void operator()(NodeRec* q) const { free(q); }
    };
    std::unique_ptr<NodeRec, Free> p;
    size_t n = 0;
    void alloc(size_t k) {
      const size_t huge = size_t(2) << 20, bytes = std::max<size_t>(k * sizeof(NodeRec), 64);
      void* q = nullptr;
      if (bytes >= huge) {
        q = aligned_alloc(huge, (bytes + huge - 1) / huge * huge);
        if (q) madvise(q, (bytes + huge - 1) / huge * huge, MADV_HUGEPAGE);
      }
      if (!q) q = malloc(bytes);
      if (!q) throw std::bad_alloc();
      p.reset((NodeRec*)q);
      n = k;
    }
    NodeRec& operator[](size_t i) { return p.get()[i]; }
    const NodeRec& operator[](size_t i) const { return p.get()[i]; }
    NodeRec* data() { return p.get(); }
    size_t size() const { return n; }
  } nodes;
  std::vector<Pair> pairs;
  // dictionary
  std::string sbytes;
  std::vector<uint32_t> soff;
  StrMap<uint32_t> dict;
  uint32_t n_dict = 0;
  uint32_t urn[U_COUNT] = {};
  std::string_view urn_s[U_COUNT];
  std::string ec_json;  // JSON array of the evaluation_cacheable values with codes 4..
  // regex rows
  std::vector<uint32_t> rx_row_id;
  std::vector<RxPattern> rx_pat;
  std::unordered_map<uint32_t, uint32_t> row_of_id;  // dictionary id of a row's value -> row
  // candidate specs (candidates.py): per rx row the nodes whose entity spec lists it; nodes
  // always a candidate; per required role the nodes requiring it
  std::vector<uint32_t> row_ptr, row_nodes;
  std::vector<uint32_t> always_bits;          // [W]
  std::vector<uint32_t> role_ids;             // sorted
  std::vector<int32_t> node_role;             // per node: index into role_ids or -1
  std::vector<uint32_t> norole_bits;          // [W]
  std::vector<std::vector<uint32_t>> role_node_list;  // per role row: node indices
  std::vector<uint8_t> node_need_act;
  // per-node target facts as [W] bitsets (the word-parallel verdict sections): a target, an
  // empty subjects list, a role-requiring subjects list, a target listing actions
  std::vector<uint32_t> tgt_bits, subj_empty_bits, subj_role_bits, need_act_bits;
  std::vector<uint32_t> need_act_nodes;  // nodes whose target lists actions
  // resource verdict statics per section (policy / rule local bits): an empty resources list,
  // an entity-only list (not empty)
  std::vector<uint32_t> res_empty_p, res_empty_r, ent_only_p, ent_only_r;
  // useful sections (candidates.useful_static): policies useful wherever they are candidates,
  // sets holding a null policy; output row layout [S | P | useful S | useful P | R]
  std::vector<uint8_t> pol_static, set_null;
  uint32_t W2 = 0, WV = 0;  // row length; offset of the target-verdict sections
  std::vector<uint8_t> spec_kind;              // per node: 0 rows list (maybe empty), 1 always, 2 rows list
  std::vector<uint32_t> spec_ptr, spec_idx;    // per node: its entity rows, in attribute order
  // caches
  std::shared_mutex hr_mu;
  std::unordered_map<uint64_t, std::vector<std::shared_ptr<const HrForest>>> hr_inline;
  std::unordered_map<std::string, std::shared_ptr<const HrForest>, FastHash> hr_subject;
  size_t hr_bytes = 0;
  std::mutex col_mu;
  std::unordered_map<std::string, std::shared_ptr<const std::vector<uint8_t>>> rx_cols;     // value key -> cells
  std::unordered_map<std::string, std::shared_ptr<const std::vector<uint32_t>>> ent_rows;   // value key -> [W]
  std::unordered_map<uint64_t, std::shared_ptr<const std::vector<uint32_t>>> act_rows;      // pair -> [W]
  std::atomic<uint64_t> hr_hits{0}, hr_misses{0};
  int force_level = -1;  // tests only (acs_internal_codec_force_level): pin the class key level
  // the largest batch whose level-0 keys (entity + roles + action) were given up (too many keys
  // per request): a batch no larger starts at level 1 — keys per request only fall as batches
  // grow (c3: level 0 was tried and dropped on every batch, ≈ 40 % of the class work)
  std::atomic<uint32_t> level0_given_up{0};
  // recycled page-locked blocks of the batches' arrays (shared: a batch may be freed after its
  // codec, e.g. by a garbage collector that finalises both in either order)
  std::shared_ptr<HostPool> pool = std::make_shared<HostPool>();
  ClassCache classes;    // candidate-class rows per key, across batches of this store version

  // global node index -> (section word offset, bit)
  uint32_t node_word(uint32_t g) const {
    if (g < S) return g >> 5;
    if (g < S + P) return ws + ((g - S) >> 5);
    return ws + wp + ((g - S - P) >> 5);
  }
  uint32_t node_bit(uint32_t g) const {
    const uint32_t l = g < S ? g : (g < S + P ? g - S : g - S - P);
    return 1u << (l & 31);
  }
  std::string_view string_of(uint32_t id) const {
    if (id >= n_dict) return {};
    return std::string_view(sbytes.data() + soff[id], soff[id + 1] - soff[id]);
  }
  uint32_t lookup(std::string_view s) const {
    auto e = dict.find(s);
    return e ? e->v : NONE32;
  }
};

namespace {

template <class T>
bool take(const uint8_t*& p, const uint8_t* e, std::vector<T>& out, size_t n, size_t align = 4) {
  const size_t bytes = n * sizeof(T);
  if ((size_t)(e - p) < bytes) return false;
  out.resize(n);
  if (n) memcpy(out.data(), p, bytes);
  p += (bytes + align - 1) / align * align;
  return true;
}

// host threads for a store load (the pool's workers; at most 16)
size_t load_threads() {
#if defined(ACS_CODEC_TIMING)
  if (const char* e = getenv("ACS_LOAD_THREADS")) return (size_t)atoi(e);
#endif
  const size_t h = std::thread::hardware_concurrency();
  return h < 1 ? 1 : (h > 16 ? 16 : h);
}

#if defined(ACS_CODEC_TIMING)
#define LOAD_T(name)                                                                                \
  do {                                                                                              \
    const auto t_ = std::chrono::steady_clock::now();                                               \
    if (getenv("ACS_LOAD_DEBUG"))                                                                   \
      fprintf(stderr, "codec_load %s %.1f ms\n", name,                                              \
              std::chrono::duration<double, std::milli>(t_ - load_t0_).count());                   \
    load_t0_ = t_;                                                                                  \
  } while (0)
#else
#define LOAD_T(name) \
  do {               \
  } while (0)
#endif
bool codec_load(acs_codec* c, const void* blob, size_t n_bytes, std::string& err) {
#if defined(ACS_CODEC_TIMING)
  auto load_t0_ = std::chrono::steady_clock::now();
#endif
  acs_blob_header h;
  if (!blob || n_bytes < sizeof h) return err = "blob too small", false;
  memcpy(&h, blob, sizeof h);
  if (h.magic != ACS_BLOB_MAGIC || h.version != ACS_ABI_VERSION) return err = "bad blob magic/version", false;
  const uint32_t off = h.reserved[0], len = h.reserved[1];
  if (!off || (size_t)off + len > n_bytes) return err = "blob has no codec section (compiler.store_blob)", false;
  c->S = h.n_sets;
  c->P = h.n_pols;
  c->R = h.n_rules;
  c->ws = words_of(c->S);
  c->wp = words_of(c->P);
  c->wr = words_of(c->R);
  c->W = c->ws + c->wp + c->wr;
  // node tables (16-B aligned sections after the 64-B header)
  const uint8_t* base = (const uint8_t*)blob;
  const uint8_t* p = base + 64;
  const uint8_t* e = base + off;
  auto a16 = [](size_t x) { return (x + 15) & ~size_t(15); };
  const size_t nn = (size_t)c->S + c->P + c->R;
  if ((size_t)(e - p) < a16(nn * 64)) return err = "truncated node tables", false;
  c->nodes.alloc(nn);
  {  // the three sections, copied in 4-MB pieces over the pool (c5: 65 MB, page faults included)
    const uint8_t* src[3] = {p, p + a16(c->S * 64ull), p + a16(c->S * 64ull) + a16(c->P * 64ull)};
    uint8_t* dst[3] = {(uint8_t*)c->nodes.data(), (uint8_t*)(c->nodes.data() + c->S),
                       (uint8_t*)(c->nodes.data() + c->S + c->P)};
    const size_t len[3] = {c->S * 64ull, c->P * 64ull, c->R * 64ull};
    constexpr size_t PIECE = size_t(4) << 20;
    std::vector<std::array<size_t, 3>> pieces;  // (section, offset, bytes)
    for (int k = 0; k < 3; ++k)
      for (size_t o = 0; o < len[k]; o += PIECE) pieces.push_back({(size_t)k, o, std::min(PIECE, len[k] - o)});
    std::atomic<size_t> next{0};
    acs_pool::run((int)std::min<size_t>(load_threads(), std::max<size_t>(pieces.size(), 1)), [&](int) {
      for (size_t x; (x = next.fetch_add(1)) < pieces.size();) {
        const auto& q = pieces[x];
        memcpy(dst[q[0]] + q[1], src[q[0]] + q[1], q[2]);
      }
    });
    p = src[2] + a16(c->R * 64ull);
  }
  p += a16(h.n_rres * 16ull);
  if ((size_t)(e - p) < h.n_pairs * 8ull) return err = "truncated pair pool", false;
  c->pairs.resize(h.n_pairs);
  if (h.n_pairs) memcpy(c->pairs.data(), p, h.n_pairs * 8ull);
  LOAD_T("tables");
  // codec section
  p = base + off;
  e = p + len;
  uint32_t hd[8];
  if (len < sizeof hd) return err = "truncated codec section", false;
  memcpy(hd, p, sizeof hd);
  p += sizeof hd;
  if (hd[0] != CODEC_MAGIC || hd[1] != CODEC_VERSION) return err = "bad codec section magic/version", false;
  const uint32_t n_str = hd[2], n_urn = hd[3], n_rx = hd[4], n_spec = hd[5], n_idx = hd[6], n_sb = hd[7];
  if (n_urn != U_COUNT || n_spec != nn) return err = "codec section does not match the tables", false;
  std::vector<uint32_t> urns, spec_ptr, spec_idx;
  std::vector<uint8_t> kind;
  if (!take(p, e, urns, n_urn) || !take(p, e, c->rx_row_id, n_rx) || !take(p, e, kind, n_spec) ||
      !take(p, e, spec_ptr, n_spec + 1) || !take(p, e, spec_idx, n_idx) || !take(p, e, c->soff, n_str + 1))
    return err = "truncated codec section", false;
  if ((size_t)(e - p) < n_sb || c->soff.back() != n_sb) return err = "bad codec string table", false;
  c->sbytes.assign((const char*)p, n_sb);
  p += (n_sb + 3) / 4 * 4;
  uint32_t ecn = 0;
  if ((size_t)(e - p) < 4) return err = "truncated codec section", false;
  memcpy(&ecn, p, 4);
  p += 4;
  if ((size_t)(e - p) < ecn) return err = "truncated codec section", false;
  c->ec_json.assign((const char*)p, ecn);
  LOAD_T("sections");
  c->n_dict = n_str;
  c->dict = StrMap<uint32_t>(n_str);
  for (uint32_t i = ID_EMPTY; i < n_str; ++i) {
    const std::string_view v = c->string_of(i);
    const uint64_t h = fast_hash(v.data(), v.size());
    if (!c->dict.find(h, v)) c->dict.insert(h, v.data(), (uint32_t)v.size(), i);  // first id of a string
  }
  LOAD_T("dict");
  for (int k = 0; k < U_COUNT; ++k) {
    c->urn[k] = urns[k];
    c->urn_s[k] = c->string_of(urns[k]);
  }
  c->rx_pat.resize(n_rx);
  for (uint32_t r = 0; r < n_rx; ++r) {
    const uint32_t id = c->rx_row_id[r];
    c->row_of_id.emplace(id, r);
    prepare_pattern(c->rx_pat[r], id <= ID_NULL, c->string_of(id));
  }
  LOAD_T("rx");
  // candidate specs
  c->always_bits.assign(c->W, 0);
  std::vector<std::vector<uint32_t>> per_row(n_rx);
  for (uint32_t g = 0; g < nn; ++g) {
    if (kind[g] == 1) c->always_bits[c->node_word(g)] |= c->node_bit(g);
    else if (kind[g] == 2)
      for (uint32_t k = spec_ptr[g]; k < spec_ptr[g + 1]; ++k)
        if (spec_idx[k] < n_rx) per_row[spec_idx[k]].push_back(g);
  }
  c->row_ptr.assign(n_rx + 1, 0);
  for (uint32_t r = 0; r < n_rx; ++r) {
    c->row_ptr[r + 1] = c->row_ptr[r] + (uint32_t)per_row[r].size();
    c->row_nodes.insert(c->row_nodes.end(), per_row[r].begin(), per_row[r].end());
  }
  LOAD_T("specs");
  // useful-section statics (candidates.useful_static)
  c->WV = 2 * c->ws + 2 * c->wp + c->wr;
  c->W2 = c->WV + 4 * c->wp + c->wr;
  c->spec_kind = kind;
  c->spec_ptr = spec_ptr;
  c->spec_idx = spec_idx;
  c->pol_static.assign(c->P, 0);
  c->set_null.assign(c->S, 0);
  for (uint32_t q = 0; q < c->P; ++q) {
    const NodeRec& N = c->nodes[c->S + q];
    const bool eff_only = (N.nflags & NF_EFFECT_TRUTHY) && N.map_size == 0;
    const bool tgt = (N.nflags & NF_HAS_TARGET) && ((N.tflags & TF_HAS_SUBJECTS) || kind[c->S + q] == 1);
    c->pol_static[q] = eff_only || tgt;
  }
  for (uint32_t s = 0; s < c->S; ++s) {
    const NodeRec& N = c->nodes[s];
    for (uint32_t q = N.child_begin; q < N.child_end && q < c->P; ++q)
      if (c->nodes[c->S + q].nflags & NF_NULL) c->set_null[s] = 1;
  }
  // role requirements (candidates.role_requirements), action requirements and the per-node
  // bit rows, in parallel over pieces of whole words of each section (a word's bits belong to one
  // piece; c5: 1M nodes, 150 -> ~30 ms)
  LOAD_T("useful statics");
  c->node_role.assign(nn, -1);
  c->node_need_act.assign(nn, 0);
  std::vector<uint32_t> req_role(nn, NONE32);
  c->tgt_bits.assign(c->W, 0);
  c->subj_empty_bits.assign(c->W, 0);
  c->subj_role_bits.assign(c->W, 0);
  c->need_act_bits.assign(c->W, 0);
  c->res_empty_p.assign(c->wp ? c->wp : 1, 0);
  c->ent_only_p.assign(c->wp ? c->wp : 1, 0);
  c->res_empty_r.assign(c->wr ? c->wr : 1, 0);
  c->ent_only_r.assign(c->wr ? c->wr : 1, 0);
  c->norole_bits.assign(c->W, 0);
  std::vector<std::pair<uint32_t, uint32_t>> pieces;  // node ranges, word-aligned per section
  {
    const uint32_t sec[4] = {0, c->S, c->S + c->P, (uint32_t)nn};
    for (int k = 0; k < 3; ++k)
      for (uint32_t g = sec[k]; g < sec[k + 1]; g += 8192) pieces.push_back({g, std::min(sec[k + 1], g + 8192)});
  }
  const int LT = (int)std::min<size_t>(load_threads(), std::max<size_t>(pieces.size(), 1));
  std::vector<std::vector<uint32_t>> roles_t(LT);
  LOAD_T("alloc");
  {
    std::atomic<size_t> next{0};
    acs_pool::run(LT, [&](int t) {
      std::vector<uint32_t>& mine = roles_t[t];
      uint32_t seen[256];  // direct-mapped: roles this thread already listed
      for (uint32_t& v : seen) v = NONE32;
      for (size_t x; (x = next.fetch_add(1)) < pieces.size();) {
        for (uint32_t g = pieces[x].first; g < pieces[x].second; ++g) {
          const NodeRec& N = c->nodes[g];
          const bool tgt = (N.nflags & NF_HAS_TARGET) != 0;
          if (tgt && (N.tflags & TF_SUBJ_ROLE) && !(N.tflags & TF_SUBJ_EMPTY)) {
            req_role[g] = N.role;
            uint32_t& sl = seen[(N.role * 2654435761u) >> 24];
            if (sl != N.role) {
              sl = N.role;
              if (std::find(mine.begin(), mine.end(), N.role) == mine.end()) mine.push_back(N.role);
            }
          }
          c->node_need_act[g] = tgt && N.act_n > 0;
          if (tgt) {
            const uint32_t w = c->node_word(g), b = c->node_bit(g);
            c->tgt_bits[w] |= b;
            if (N.tflags & TF_SUBJ_EMPTY) c->subj_empty_bits[w] |= b;
            else if (N.tflags & TF_SUBJ_ROLE) c->subj_role_bits[w] |= b;
            if (c->node_need_act[g]) c->need_act_bits[w] |= b;
          }
          if (g >= c->S) {
            const bool pol = g < c->S + c->P;
            const uint32_t l = pol ? g - c->S : g - c->S - c->P;
            const uint16_t tf = (uint16_t)N.tflags;
            if (tf & TF_RES_EMPTY) (pol ? c->res_empty_p : c->res_empty_r)[l >> 5] |= 1u << (l & 31);
            else if (tf & TF_RES_ENT_ONLY) (pol ? c->ent_only_p : c->ent_only_r)[l >> 5] |= 1u << (l & 31);
          }
        }
      }
    });
  }
#if defined(ACS_CODEC_TIMING)
  if (getenv("ACS_LOAD_DEBUG")) {
    size_t used = 0;
    for (const auto& v : roles_t) used += !v.empty();
    fprintf(stderr, "pass1: LT %d, threads with roles %zu, pieces %zu\n", LT, used, pieces.size());
  }
#endif
  LOAD_T("pass1");
  for (const auto& v : roles_t) c->role_ids.insert(c->role_ids.end(), v.begin(), v.end());
  std::sort(c->role_ids.begin(), c->role_ids.end());
  c->role_ids.erase(std::unique(c->role_ids.begin(), c->role_ids.end()), c->role_ids.end());
  {
    std::atomic<size_t> next{0};
    acs_pool::run(LT, [&](int) {
      uint32_t memo_role[256], memo_idx[256];  // direct-mapped role id -> row
      for (uint32_t& v : memo_role) v = NONE32;
      for (size_t x; (x = next.fetch_add(1)) < pieces.size();)
        for (uint32_t g = pieces[x].first; g < pieces[x].second; ++g) {
          const uint32_t r = req_role[g];
          if (r == NONE32) {
            c->norole_bits[c->node_word(g)] |= c->node_bit(g);
            continue;
          }
          const uint32_t h = (r * 2654435761u) >> 24;
          if (memo_role[h] != r) {
            memo_role[h] = r;
            memo_idx[h] = (uint32_t)(std::lower_bound(c->role_ids.begin(), c->role_ids.end(), r) - c->role_ids.begin());
          }
          c->node_role[g] = (int)memo_idx[h];
        }
    });
  }
  LOAD_T("pass2");
  for (uint32_t g = 0; g < nn; ++g)
    if (c->node_need_act[g]) c->need_act_nodes.push_back(g);
  c->role_node_list.assign(c->role_ids.size(), {});
  for (uint32_t g = 0; g < nn; ++g)
    if (c->node_role[g] >= 0) c->role_node_list[c->node_role[g]].push_back(g);
  LOAD_T("statics");
  return true;
}

}  // namespace

// ------------------------------------------------------------------ encoded batch
struct ThreadStrings {  // one encoder thread's batch-local strings (ids base + k)
  uint32_t base = 0;
  StrPool bytes;
  std::vector<std::string_view> strs;  // views into `bytes`
};

// An encoded batch in the compact form (acs_layout.h): request lines, extension records,
// context arena, regex matrix, class rows — the arrays the kernels read, in page-locked host
// memory.  The SoA rows (hdr / res / subj / act / roles) are only materialised on request
// (acs_codec_batch_expand: tests, the CPU build of the core).
struct acs_codec_batch {
  acs_codec* codec = nullptr;
  std::shared_ptr<HostPool> pool;
  uint32_t n = 0;
  HostBlock lines_b, ext_b, arena_b, cand_b, perm_b;
  ReqLine* lines = nullptr;   // [n]
  uint32_t* ext = nullptr;    // extension records (ReqLine.ext)
  size_t ext_words = 0;
  uint32_t* arena = nullptr;  // context arena
  size_t arena_words = 0;
  std::vector<uint8_t> rx;  // [rx_cols][rx_rows]
  uint32_t rx_cols = 1, rx_rows = 1;
  uint32_t* cand = nullptr;  // [cand_rows][cand_words]
  uint32_t cand_rows = 0, cand_words = 0, cand_wp = 0, cand_wr = 0, cand_wsu = 0, cand_wpu = 0, cand_wv = 0;
  std::vector<uint32_t> role_key, role_bits;
  uint32_t role_rows = 0;
  uint32_t* perm = nullptr;  // coherence order (candidates.coherence_order), perm_lanes entries
  size_t perm_lanes = 0;
  uint32_t hints = 0;  // acs_req_batch.hints
  // SoA rows (acs_codec_batch_expand)
  bool expanded = false;
  std::vector<ReqHdr> hdr;
  std::vector<ReqRes> res;  // [QMAX][n]
  std::vector<Pair> subj, act;
  std::vector<uint32_t> roles;
  std::vector<const char*> reason;  // per request: why it goes to the host (nullptr: it does not)
  std::deque<ThreadStrings> strings;  // (a deque: StrPool does not move)
  double seconds[4] = {};  // parse+encode, regex matrix, candidate classes, total
  uint64_t hr_hits = 0, hr_misses = 0;
  uint32_t classes_new = 0;  // class keys computed by this batch (the rest came from the cache)
  ~acs_codec_batch() {
    if (!pool) return;
    pool->release(lines_b);
    pool->release(ext_b);
    pool->release(arena_b);
    pool->release(cand_b);
    pool->release(perm_b);
  }
  // request rows of the compact form
  const ReqHdr& h(uint32_t i) const { return lines[i].h; }
  ReqRes res_at(uint32_t i, uint32_t j) const {
    if (j < (uint32_t)LINE_RES) return lines[i].res[j];
    ReqRes q;
    memcpy(&q, ext + (size_t)(lines[i].ext - 1) * 4 + 4 * (j - LINE_RES), sizeof q);
    return q;
  }
  ReqRes* res_ptr(uint32_t i, uint32_t j) {
    if (j < (uint32_t)LINE_RES) return &lines[i].res[j];
    return (ReqRes*)(ext + (size_t)(lines[i].ext - 1) * 4 + 4 * (j - LINE_RES));
  }
  uint32_t role_at(uint32_t i, uint32_t k) const {
    if (k == 0) return lines[i].r0;
    if (k == 1) return lines[i].r1;
    const ReqHdr& hd = lines[i].h;
    return ext[(size_t)(lines[i].ext - 1) * 4 + ext_geom(hd.nres, hd.nsubj, hd.nact, hd.nroles).roles + (k - 2)];
  }
};

namespace {

uint64_t hash_bytes(const char* p, size_t n) {
  uint64_t h = 0x9E3779B97F4A7C15ull ^ (n * 0xC2B2AE3D27D4EB4Full);
  size_t k = 0;
  for (; k + 8 <= n; k += 8) {
    uint64_t w;
    memcpy(&w, p + k, 8);
    h = (h ^ w) * 0xFF51AFD7ED558CCDull;
    h ^= h >> 31;
  }
  uint64_t w = 0;
  memcpy(&w, p + k, n - k);
  h = (h ^ w) * 0xC4CEB9FE1A85EC53ull;
  h ^= h >> 29;
  return h;
}

constexpr size_t HR_CACHE_BYTES = size_t(512) << 20;

struct Col {  // one distinct entity value of the batch (a regex-matrix column)
  std::string key;  // 'm' undefined, 'n' null, 's' + value
  uint32_t first;   // first use: request index * QMAX + attribute index
};

struct Shared {  // batch-wide state of the encoder threads
  std::mutex mu;
  std::unordered_map<std::string, uint32_t> col_index;
  std::vector<Col> cols;
};

class Encoder {
 public:
  Encoder(acs_codec& c, acs_codec_batch& b, Shared& sh, uint32_t t) : C(c), B(b), SH(sh), parser_(ar_) {
    strs_ = &B.strings[t];
  }
  void encode(uint32_t i, const char* p, const char* e);
  std::vector<uint32_t> arena;  // this thread's context arena words
  std::vector<uint32_t> ext;    // this thread's extension records
  uint64_t hits = 0, misses = 0;
  uint32_t hints = 0;  // ACS_HINT_* of the requests this encoder wrote

 private:
  // String -> id: the store dictionary, else this thread's batch-local strings.  A
  // direct-mapped cache of recent strings (hash, canonical bytes, id) in front of both: a
  // request interns ~25 strings, most of them URNs every request repeats, and a miss in the
  // node-based maps costs a few cache misses (~500 cycles measured) where a hit here costs
  // one hash and one compare against bytes that are already in cache.
  uint32_t intern_sv(std::string_view s) {
    const uint64_t h = fast_hash(s.data(), s.size());
    RecentString& x = recent_[h & (RECENT - 1)];
    if (x.h == h && x.n == s.size() && memcmp(x.p, s.data(), s.size()) == 0) return x.id;
    uint32_t id;
    const char* canon;
    if (auto d = C.dict.find(h, s)) {
      id = d->v;
      canon = d->p;
    } else if (auto l = local_.find(h, s)) {
      id = l->v;
      canon = l->p;
    } else {
      if (strs_->strs.size() >= (1u << LOCAL_BITS)) unsup("too many batch-local strings");
      canon = strs_->bytes.put(s);
      strs_->strs.emplace_back(canon, s.size());
      id = strs_->base + (uint32_t)strs_->strs.size() - 1;
      local_.insert(h, canon, (uint32_t)s.size(), id);
    }
    x.h = h;
    x.p = canon;
    x.n = (uint32_t)s.size();
    x.id = id;
    return id;
  }
  uint32_t intern(const JV* v) {
    if (v->t == J_UNDEF) return ID_UNDEF;
    if (v->t == J_NULL) return ID_NULL;
    if (v->t != J_STR) unsup("non-string attribute scalar");
    return intern_sv(v->str());
  }
  uint32_t intern(const Scalar& s) { return s.kind == 0 ? ID_UNDEF : s.kind == 1 ? ID_NULL : intern_sv(s.s); }
  // strict equality with a URN (undefined URN: only an absent value equals it)
  bool eq_urn(const JV* v, int u) const {
    if (C.urn[u] == ID_UNDEF) return v->t == J_UNDEF;
    return v->t == J_STR && v->str() == C.urn_s[u];
  }
  bool loose_urn(const JV* v, int u) const {  // (nullish(v) && nullish(urn)) || v === urn
    return (nullish(v) && C.urn[u] == ID_UNDEF) || eq_urn(v, u);
  }
  static void check_scalar(const JV* v) {
    if (!(v->t == J_UNDEF || v->t == J_NULL || v->t == J_STR)) unsup("non-string attribute scalar");
  }
  static const JV* attr_list(const JV* v, uint32_t& n) {  // _attr_list
    n = 0;
    if (!truthy(v)) return nullptr;
    if (v->t != J_ARR) unsup("non-array list value");
    for (uint32_t k = 0; k < v->n; ++k) {
      const JV* a = &v->a[k];
      if (a->t != J_OBJ) unsup("non-object attribute entry");
      check_scalar(get(a, "id"));
      check_scalar(get(a, "value"));
    }
    n = v->n;
    return v->a;
  }
  static const JV* dict_list(const JV* v, uint32_t& n) {  // _dict_list
    n = 0;
    if (nullish(v)) return nullptr;
    if (v->t != J_ARR) unsup("list value is not an array");
    for (uint32_t k = 0; k < v->n; ++k)
      if (v->a[k].t != J_OBJ) unsup("non-object list entry");
    n = v->n;
    return v->a;
  }
  // lodash _.find(coll, [path, value]) for a string / null / undefined value
  static const JV* find_by(const JV* coll, uint32_t nc, bool instance_id, const JV* value) {
    for (uint32_t k = 0; k < nc; ++k) {
      const JV* o = &coll[k];
      const JV* ov = instance_id ? get(get(o, "instance"), "id") : get(o, "id");
      if (ov->t == J_UNDEF) continue;  // an absent path never equals (JSON has no undefined members)
      if (ov->t == J_OBJ || ov->t == J_ARR) continue;
      if (value->t == J_NULL ? ov->t == J_NULL : (value->t == J_STR && ov->t == J_STR && ov->str() == value->str()))
        return o;
    }
    return &kUndef;
  }
  uint32_t column(const JV* v, uint32_t i) {  // i: request index * QMAX + attribute index
    uint32_t* memo = v->t == J_UNDEF ? &col_undef_ : v->t == J_NULL ? &col_null_ : nullptr;
    if (memo && *memo != NONE32) return *memo;
    if (!memo) {
      auto it = cols_.find(v->str());
      if (it != cols_.end()) return it->second;
    }
    std::string key = v->t == J_UNDEF ? std::string("m") : v->t == J_NULL ? std::string("n") : "s" + std::string(v->str());
    std::lock_guard<std::mutex> lock(SH.mu);
    auto g = SH.col_index.find(key);
    uint32_t c;
    if (g == SH.col_index.end()) {
      if (SH.cols.size() >= 0xFFFE) unsup("too many distinct entity values in batch");
      c = (uint32_t)SH.cols.size();
      SH.col_index.emplace(key, c);
      SH.cols.push_back({key, i});
    } else {
      c = g->second;
      if (i < SH.cols[c].first) SH.cols[c].first = i;
    }
    if (memo) *memo = c;
    else cols_.emplace(v->str(), c);
    return c;
  }
  // A registered forest as this thread sees it: the forest and its roots / effective-role
  // keys interned once per thread and batch
  struct Registered {
    std::shared_ptr<const HrForest> f;
    std::vector<uint32_t> root_ids, key_ids;
  };
  // The subject's HR forest for one request: one forest (inline or registered), or the parts of
  // a "$hrs" key list composed in place — roots concatenated, keys merged in first-seen order,
  // owner masks read from the parts and remapped — without building a forest per request
  struct SubjectForest {
    const HrForest* one = nullptr;
    const Registered* part[MAX_ROOTS];
    uint32_t n = 0;
    uint32_t root_off[MAX_ROOTS];
    uint8_t key_map[MAX_ROOTS][MAX_HRKEYS];
    bool is_array = false;
    uint64_t mask(std::string_view id) const {
      if (one) return one->mask(id);
      uint64_t m = 0;
      for (uint32_t p = 0; p < n; ++p) {
        const uint64_t x = part[p]->f->mask(id);
        if (!x) continue;
        m |= (x & 0xFFFFFFFFull) << root_off[p];
        for (uint32_t k = (uint32_t)(x >> 32); k; k &= k - 1) m |= 1ull << (32 + key_map[p][__builtin_ctz(k)]);
      }
      return m;
    }
  };
  std::shared_ptr<const HrForest> inline_forest(const JV* raw);
  void subject_forest(const JV* key, SubjectForest& out, std::vector<uint32_t>& roots, std::vector<uint32_t>& keys);
  const Registered& registered_forest(const JV* key);
  void encode_one(uint32_t i, const JV* req);

  acs_codec& C;
  acs_codec_batch& B;
  Shared& SH;
  ThreadStrings* strs_;
  Arena ar_, ar2_;
  Parser parser_;
  StrMap<uint32_t> local_{4096};  // batch-local strings of this thread (bytes: strs_->bytes)
  struct RecentString {
    uint64_t h = 0;
    const char* p = nullptr;  // the dictionary's or pool_'s bytes (stable for the batch)
    uint32_t n = 0xFFFFFFFFu, id = 0;
  };
  static constexpr size_t RECENT = 4096;
  std::unique_ptr<RecentString[]> recent_{new RecentString[RECENT]};
  // this thread's view of batch-wide state, keyed by views into the request text (valid for
  // the batch): entity value -> regex-matrix column, "$hrs" subject key (or key list) ->
  // forest (the maps' shared_ptrs keep the forests alive), so the shared maps and their locks
  // are touched once per distinct value per thread, not once per request
  std::unordered_map<std::string_view, uint32_t, FastHash> cols_;
  uint32_t col_undef_ = NONE32, col_null_ = NONE32;
  std::unordered_map<std::string_view, Registered, FastHash> forests_;
  // per-request scratch (cleared, never freed)
  std::vector<const JV*> slot_objs_;
  std::vector<std::pair<uint32_t, uint8_t>> keys_a_, keys_b_;
  std::vector<uint32_t> rolese_, grants_, roots_, hr_keys_, w_;
  std::vector<std::pair<uint32_t, std::vector<const JV*>>> tse_;
  size_t tse_n_ = 0;
};

std::shared_ptr<const HrForest> Encoder::inline_forest(const JV* raw) {
  const uint64_t h = hash_bytes(raw->s, raw->n);
  {
    std::shared_lock<std::shared_mutex> lock(C.hr_mu);
    auto it = C.hr_inline.find(h);
    if (it != C.hr_inline.end())
      for (const auto& f : it->second)
        if (f->text.size() == raw->n && memcmp(f->text.data(), raw->s, raw->n) == 0) {
          ++hits;
          return f;
        }
  }
  ++misses;
  auto F = std::make_shared<HrForest>();
  F->text.assign(raw->s, raw->n);
  ar2_.reset();
  Parser p2(ar2_);
  const JV* v = p2.parse(raw->s, raw->s + raw->n);
  build_forest(*F, v);
  std::unique_lock<std::shared_mutex> lock(C.hr_mu);
  if (C.hr_bytes + F->bytes() > HR_CACHE_BYTES) {
    C.hr_inline.clear();
    C.hr_bytes = 0;
  }
  C.hr_bytes += F->bytes();
  C.hr_inline[h].push_back(F);
  return F;
}

// A "$hrs" key: one registered forest (createHRScope's per-subject cache), or a list of them
// whose root arrays concatenate into the subject's hierarchical_scopes (e.g. one cached forest
// per role association: compose_forests' semantics, composed in place per request).  Fills the
// request's roots and effective-role keys (interned); unsupported forests send it to the host.
void Encoder::subject_forest(const JV* key, SubjectForest& out, std::vector<uint32_t>& roots,
                             std::vector<uint32_t>& keys) {
  ++hits;
  if (key->t != J_ARR) {
    const Registered& r = registered_forest(key);
    if (r.f->why) unsup(r.f->why);
    out.one = r.f.get();
    out.is_array = r.f->is_array;
    if (out.is_array) {
      roots.insert(roots.end(), r.root_ids.begin(), r.root_ids.end());
      keys.insert(keys.end(), r.key_ids.begin(), r.key_ids.end());
    }
    return;
  }
  if (key->n > (uint32_t)MAX_ROOTS) unsup("too many HR scope roots");
  out.is_array = true;
  for (uint32_t k = 0; k < key->n; ++k) {
    const Registered& r = registered_forest(&key->a[k]);
    if (r.f->why) unsup(r.f->why);
    if (!r.f->is_array) unsup("registered HR scopes are not an array");
    if (roots.size() + r.root_ids.size() > (size_t)MAX_ROOTS) unsup("too many HR scope roots");
    const uint32_t p = out.n++;
    out.part[p] = &r;
    out.root_off[p] = (uint32_t)roots.size();
    roots.insert(roots.end(), r.root_ids.begin(), r.root_ids.end());
    for (size_t q = 0; q < r.key_ids.size(); ++q) {
      size_t at = 0;
      while (at < keys.size() && keys[at] != r.key_ids[q]) ++at;
      if (at == keys.size()) {
        if (keys.size() >= (size_t)MAX_HRKEYS) unsup("too many HR effective roles");
        keys.push_back(r.key_ids[q]);
      }
      out.key_map[p][q] = (uint8_t)at;
    }
  }
}

const Encoder::Registered& Encoder::registered_forest(const JV* key) {
  if (key->t != J_STR) unsup("$hrs subject key is not a string");
  auto mine = forests_.find(key->str());
  if (mine == forests_.end()) {
    std::shared_ptr<const HrForest> f;
    {
      std::shared_lock<std::shared_mutex> lock(C.hr_mu);
      auto it = C.hr_subject.find(std::string(key->str()));
      if (it != C.hr_subject.end()) f = it->second;
    }
    if (!f) unsup("subject HR scopes not in the codec cache (acs_codec_set_subject_scopes)");
    Registered r;
    if (!f->why && f->is_array) {
      for (const Scalar& x : f->roots) r.root_ids.push_back(intern(x));
      for (const Scalar& x : f->keys) r.key_ids.push_back(intern(x));
    }
    r.f = std::move(f);
    mine = forests_.emplace(key->str(), std::move(r)).first;
  }
  return mine->second;
}

#if defined(ACS_CODEC_TIMING)  // profiling harness only: cycles in parse / encode_one
std::atomic<uint64_t> g_cyc_parse{0}, g_cyc_encode{0};
#endif

void Encoder::encode(uint32_t i, const char* p, const char* e) {
  ar_.reset();
#if defined(ACS_CODEC_TIMING)
  const uint64_t c0 = __builtin_ia32_rdtsc();
#endif
  const JV* req = parser_.parse(p, e, "hierarchical_scopes");
#if defined(ACS_CODEC_TIMING)
  const uint64_t c1 = __builtin_ia32_rdtsc();
  g_cyc_parse += c1 - c0;
  struct Tail {
    uint64_t t;
    ~Tail() { g_cyc_encode += __builtin_ia32_rdtsc() - t; }
  } tail{c1};
#endif
  try {
    encode_one(i, req);
  } catch (const Unsup& u) {
    ReqLine& L = B.lines[i];
    L = ReqLine{};
    L.h.flags = RQ_HOST;
    L.h.arena_off = (uint32_t)arena.size();  // (thread-local until the batch is assembled)
    arena.push_back(0);
    arena.push_back(0);
    B.reason[i] = u.why;
  }
}

#if defined(ACS_CODEC_TIMING)
std::atomic<uint64_t> g_cyc_sect[8];
#define SECT(k)                                            \
  do {                                                     \
    const uint64_t t_ = __builtin_ia32_rdtsc();            \
    g_cyc_sect[k].fetch_add(t_ - t_sect_, std::memory_order_relaxed); \
    t_sect_ = t_;                                          \
  } while (0)
#else
#define SECT(k) \
  do {          \
  } while (0)
#endif

// encoder.py Encoder._encode_one, restated.
void Encoder::encode_one(uint32_t i, const JV* req) {
#if defined(ACS_CODEC_TIMING)
  uint64_t t_sect_ = __builtin_ia32_rdtsc();
#endif
  uint32_t flags = 0;
  if (req->t != J_OBJ) unsup("request is not an object");
  const JV* target = get(req, "target");
  const JV *subjects = nullptr, *resources = nullptr, *actions = nullptr;
  uint32_t ns = 0, nr = 0, na = 0;
  if (!truthy(target)) {
    flags |= RQ_NO_TARGET;
  } else {
    if (target->t != J_OBJ) unsup("target is not an object");
    subjects = attr_list(get(target, "subjects"), ns);
    resources = attr_list(get(target, "resources"), nr);
    actions = attr_list(get(target, "actions"), na);
  }
  if (ns > (uint32_t)SMAX || nr > (uint32_t)QMAX || na > (uint32_t)AMAX) unsup("request list exceeds packed capacity");

  const JV* ctx = get(req, "context");
  const bool ctx_empty = is_empty(ctx);
  if (!nullish(ctx) && ctx->t != J_OBJ) unsup("context is not an object");
  if (ctx_empty) flags |= RQ_CTX_EMPTY;
  const JV* subj = get(ctx, "subject");
  if (!nullish(subj) && subj->t != J_OBJ) unsup("context.subject is not an object");
  if (truthy(get(subj, "token"))) unsup("subject token: identity-srv / HR-scope I/O (accessController.ts:110-123)");
  if (ctx_empty || nullish(subj)) flags |= RQ_SUBJ_MISSING;
  const JV* ras_v = get(subj, "role_associations");
  if (truthy(ras_v)) flags |= RQ_RA_TRUTHY;
  if (is_empty(ras_v)) flags |= RQ_RA_EMPTY;
  uint32_t n_ras = 0;
  const JV* ras = truthy(ras_v) ? dict_list(ras_v, n_ras) : nullptr;
  if (n_ras > (uint32_t)RMAX) unsup("too many role associations");
  const JV* hrs = get(subj, "hierarchical_scopes");
  // the subject's forest: its roots and effective-role keys (interned) and owner masks
  SubjectForest forest;
  bool have_forest = false;
  std::vector<uint32_t>& roots = roots_;
  std::vector<uint32_t>& hr_keys = hr_keys_;
  roots.clear();
  hr_keys.clear();
  std::shared_ptr<const HrForest> inl;  // an inline forest (the codec's cache may drop it)
  if (hrs->t == J_RAW) {
    if (hrs->raw == J_ARR) {
      inl = inline_forest(hrs);
      if (inl->why) unsup(inl->why);
      forest.one = inl.get();
      forest.is_array = inl->is_array;
      have_forest = true;
      if (inl->is_array) {
        for (const Scalar& r : inl->roots) roots.push_back(intern(r));
        for (const Scalar& k : inl->keys) hr_keys.push_back(intern(k));
      }
    }
    else if (hrs->raw != J_NULL) unsup("hierarchical_scopes is not an array");
  } else if (hrs->t == J_UNDEF) {
    const JV* key = get(subj, "$hrs");  // the subject's registered forest (createHRScope's cache)
    if (key->t != J_UNDEF) {
      subject_forest(key, forest, roots, hr_keys);
      have_forest = true;
    }
  } else if (hrs->t == J_ARR || hrs->t == J_OBJ) {
    unsup("hierarchical_scopes outside the codec's forest cache");  // (only reached without raw_key)
  } else if (!nullish(hrs)) {
    unsup("hierarchical_scopes is not an array");
  }
  if (have_forest && forest.is_array) flags |= RQ_HRS_ITERABLE;
  SECT(0);

  // ---- resources: kinds, ids, regex columns, suffixes, indexOf masks
  uint8_t kinds[QMAX] = {};
  int n_ent = 0;
  for (uint32_t j = 0; j < nr; ++j) {
    const JV* id = get(&resources[j], "id");
    const JV* v = get(&resources[j], "value");
    uint8_t kind = 0;
    if (eq_urn(id, U_ENT)) {
      kind |= K_ENT;
      ++n_ent;
    }
    if (loose_urn(id, U_ENT)) kind |= K_ENT_LOOSE;
    if (eq_urn(id, U_OP)) kind |= K_OP;
    if (eq_urn(id, U_PROP)) {
      kind |= K_PROP;
      flags |= RQ_ANY_PROP;
    }
    if (loose_urn(id, U_RID)) kind |= K_RID_LOOSE;
    if (v->t == J_STR && v->str().find('#') != std::string_view::npos) kind |= K_HAS_HASH;
    kinds[j] = kind;
  }
  if (n_ent > 1) flags |= RQ_MULTI_ENT;
  {
    int first = -1, cnt = 0;
    for (uint32_t j = 0; j < nr; ++j)
      if (kinds[j] & K_ENT) {
        if (first < 0) first = (int)j;
        ++cnt;
      }
    const uint32_t ent_field = first < 0 ? 0u : (cnt == 1 && first < 6 ? (uint32_t)first + 1 : 7u);
    flags |= ent_field << RQ_ENT_SHIFT;
  }
  const JV* ctx_res = nullptr;
  uint32_t n_ctx = 0;
  if (!ctx_empty) {
    const JV* cr = get(ctx, "resources");
    if (truthy(cr)) {
      if (cr->t != J_ARR) unsup("context.resources is not an array");
      ctx_res = cr->a;
      n_ctx = cr->n;
    }
  }
  std::vector<const JV*>& slot_objs = slot_objs_;
  slot_objs.clear();
  auto slot_of = [&](const JV* obj) -> uint8_t {
    if (!truthy(obj)) return NONE8;
    for (size_t k = 0; k < slot_objs.size(); ++k)
      if (slot_objs[k] == obj) return (uint8_t)k;
    if (slot_objs.size() >= (size_t)MAX_SLOTS) unsup("too many context resources");
    slot_objs.push_back(obj);
    return (uint8_t)(slot_objs.size() - 1);
  };
  auto resolve_a = [&](const JV* v) -> const JV* {  // hierarchicalScope.ts:106-112 / verifyACL.ts:40-48
    const JV* o = find_by(ctx_res, n_ctx, true, v);
    if (truthy(o)) return get(o, "instance");
    return find_by(ctx_res, n_ctx, false, v);
  };
  ReqRes rows[QMAX] = {};
  auto& keys_a = keys_a_;  // first slot per interned value
  auto& keys_b = keys_b_;
  keys_a.clear();
  keys_b.clear();
  for (uint32_t j = 0; j < nr; ++j) {
    const JV* v = get(&resources[j], "value");
    const uint8_t kind = kinds[j];
    uint8_t sa = NONE8, sb = NONE8;
    if (kind & (K_RID_LOOSE | K_OP)) sa = slot_of(resolve_a(v));
    if (kind & K_OP) sb = slot_of(find_by(ctx_res, n_ctx, false, v));
    const uint32_t vid = intern(v);
    auto setdefault = [](std::vector<std::pair<uint32_t, uint8_t>>& m, uint32_t k, uint8_t s) {
      for (auto& x : m)
        if (x.first == k) return;
      m.push_back({k, s});
    };
    if (kind & K_RID_LOOSE) setdefault(keys_a, vid, sa);
    if (kind & K_OP) setdefault(keys_b, vid, sb);
    uint32_t hs = ID_UNDEF;
    uint16_t contains = 0;
    if ((kind & K_PROP) && v->t == J_STR) {
      const std::string_view vs = v->str();
      const size_t h = vs.rfind('#');
      hs = intern_sv(h == std::string_view::npos ? vs : vs.substr(h + 1));
      for (uint32_t i2 = 0; i2 < nr; ++i2) {
        if (!(kinds[i2] & K_ENT)) continue;
        const JV* v2 = get(&resources[i2], "value");
        std::string_view name = "undefined";
        if (v2->t == J_STR) {
          const std::string_view s2 = v2->str();
          const size_t c = s2.rfind(':');
          name = c == std::string_view::npos ? s2 : s2.substr(c + 1);
        }
        if (vs.find(name) != std::string_view::npos) contains |= (uint16_t)(1u << i2);
      }
    }
    uint16_t col = 0;
    if (kind & K_ENT_LOOSE) col = (uint16_t)column(v, i * QMAX + j);
    ReqRes& q = rows[j];
    q.value = vid;
    q.hash_sfx = hs;
    q.col = col;
    q.contains = contains;
    q.kind = kind;
    q.slot_a = sa;
    q.slot_b = sb;
  }
  SECT(1);
  for (auto& b : keys_b)  // HR map key shared by a resource id and an operation name
    for (auto& a : keys_a)
      if (a.first == b.first && a.second != b.second) unsup("resource-id / operation key collision in HR owners map");

  // ---- role associations -> roles, (role, se) pairs, (role, se, inst) grants
  uint32_t roles[RMAX] = {};
  std::vector<uint32_t>& rolese = rolese_;
  std::vector<uint32_t>& grants = grants_;
  rolese.clear();
  grants.clear();
  for (uint32_t k = 0; k < n_ras; ++k) {
    const JV* ra = &ras[k];
    const JV* role = get(ra, "role");
    check_scalar(role);
    const uint32_t rid = intern(role);
    roles[k] = rid;
    const JV* attrs = get(ra, "attributes");
    uint32_t n_at = 0;
    const JV* at = truthy(attrs) ? dict_list(attrs, n_at) : nullptr;
    for (uint32_t x = 0; x < n_at; ++x) {
      const JV* rae = &at[x];
      if (!eq_urn(get(rae, "id"), U_RSE)) continue;
      const JV* sev = get(rae, "value");
      check_scalar(sev);
      const uint32_t se = intern(sev);
      rolese.push_back(rid);
      rolese.push_back(se);
      const JV* insts = get(rae, "attributes");
      uint32_t n_in = 0;
      const JV* in = truthy(insts) ? dict_list(insts, n_in) : nullptr;
      for (uint32_t y = 0; y < n_in; ++y)
        if (eq_urn(get(&in[y], "id"), U_RSI)) {
          const JV* iv = get(&in[y], "value");
          check_scalar(iv);
          grants.push_back(rid);
          grants.push_back(se);
          grants.push_back(intern(iv));
        }
    }
  }
  if (grants.size() / 3 > 255 || rolese.size() / 2 > 255) unsup("too many role scoping grants");
  SECT(2);

  // ---- hierarchical_scopes: owner masks from the subject's forest (roots / keys above)
  auto masks_of = [&](const JV* v) -> uint64_t {
    if (!have_forest || v->t != J_STR) return 0;
    return forest.mask(v->str());
  };

  // ---- verifyACL request loop (verifyACL.ts:37-88)
  uint32_t acl_state = ACL_CONTINUE;
  std::vector<std::pair<uint32_t, std::vector<const JV*>>> tse;
  for (uint32_t j = 0; j < nr && acl_state == ACL_CONTINUE; ++j) {
    const JV* aid = get(&resources[j], "id");
    if (!(loose_urn(aid, U_RID) || eq_urn(aid, U_OP))) continue;
    const JV* obj = resolve_a(get(&resources[j], "value"));
    const JV* acls = &kUndef;
    if (truthy(obj)) {
      const JV* al = get(get(obj, "meta"), "acls");
      if (al->t == J_ARR && al->n > 0) acls = al;
      else if (truthy(al) && al->t != J_ARR) unsup("meta.acls is not an array");
    }
    if (is_empty(acls)) {
      acl_state = ACL_RET_TRUE;
      break;
    }
    uint32_t n_acl = 0;
    const JV* al = dict_list(acls, n_acl);
    for (uint32_t x = 0; x < n_acl && acl_state == ACL_CONTINUE; ++x) {
      const JV* acl = &al[x];
      if (!eq_urn(get(acl, "id"), U_ACLIE)) {
        acl_state = ACL_RET_FALSE;
        break;
      }
      const JV* sev = get(acl, "value");
      check_scalar(sev);
      const uint32_t se = intern(sev);
      size_t e = 0;
      while (e < tse.size() && tse[e].first != se) ++e;
      if (e == tse.size()) tse.push_back({se, {}});
      const JV* attrs = get(acl, "attributes");
      if (!truthy(attrs) || (attrs->t == J_ARR && attrs->n == 0)) {
        acl_state = ACL_RET_FALSE;
        break;
      }
      uint32_t n_at = 0;
      const JV* at = dict_list(attrs, n_at);
      for (uint32_t y = 0; y < n_at; ++y) {
        if (eq_urn(get(&at[y], "id"), U_ACLI)) {
          const JV* iv = get(&at[y], "value");
          check_scalar(iv);
          tse[e].second.push_back(iv);
        } else {
          acl_state = ACL_RET_FALSE;
          break;
        }
      }
    }
  }
  flags |= acl_state << RQ_ACL_SHIFT;
  SECT(3);
  if (na > 0) {
    const JV* a0 = &actions[0];
    if (eq_urn(get(a0, "id"), U_ACTID)) {
      const JV* v0 = get(a0, "value");
      if (eq_urn(v0, U_CREATE)) flags |= RQ_ACT_CREATE;
      else if (eq_urn(v0, U_READ) || eq_urn(v0, U_MODIFY) || eq_urn(v0, U_DELETE)) flags |= RQ_ACT_RMD;
    }
  }

  // ---- arena
  std::vector<uint32_t>& w = w_;
  w.assign(2, 0u);
  w.insert(w.end(), grants.begin(), grants.end());
  w.insert(w.end(), rolese.begin(), rolese.end());
  w.insert(w.end(), roots.begin(), roots.end());
  w.insert(w.end(), hr_keys.begin(), hr_keys.end());
  const size_t slot_base = w.size();
  w.resize(w.size() + slot_objs.size(), 0);
  const size_t tse_base = w.size();
  w.resize(w.size() + 3 * tse.size(), 0);
  for (size_t s = 0; s < slot_objs.size(); ++s) {
    w[slot_base + s] = (uint32_t)w.size();
    const JV* obj = slot_objs[s];
    const JV* meta = obj->t == J_OBJ ? get(obj, "meta") : &kUndef;
    const JV* owners = get(meta, "owners");
    const bool empty = is_empty(meta) || is_empty(owners);
    uint32_t n_o = 0;
    const JV* ol = empty ? nullptr : dict_list(owners, n_o);
    w.push_back(empty ? 1u : 0u);
    w.push_back(n_o);
    for (uint32_t k = 0; k < n_o; ++k) {
      const JV* o = &ol[k];
      const JV* attrs = get(o, "attributes");
      uint32_t n_at = 0;
      const JV* at = nullish(attrs) ? nullptr : dict_list(attrs, n_at);
      const uint32_t is_oe = eq_urn(get(o, "id"), U_OE) ? 1u : 0u;
      const JV* ov = get(o, "value");
      check_scalar(ov);
      w.push_back(is_oe | (n_at << 8));
      w.push_back(intern(ov));
      for (uint32_t x = 0; x < n_at; ++x) {
        const JV* av = get(&at[x], "value");
        check_scalar(av);
        w.push_back(intern(av));
        w.push_back(eq_urn(get(&at[x], "id"), U_OI) ? (uint32_t)K_OI : 0u);
        w.push_back((uint32_t)masks_of(av));
      }
    }
  }
  for (size_t e = 0; e < tse.size(); ++e) {
    const auto& insts = tse[e].second;
    if (insts.size() > 32) unsup("too many ACL instances for one scoping entity");
    w[tse_base + 3 * e] = tse[e].first;
    w[tse_base + 3 * e + 1] = (uint32_t)insts.size();
    w[tse_base + 3 * e + 2] = (uint32_t)w.size();
    for (const JV* v : insts) {
      w.push_back(intern(v));
      w.push_back((uint32_t)(masks_of(v) >> 32));
    }
  }
  if (tse.size() > 255) unsup("too many ACL scoping entities");
  SECT(4);
  w[0] = (uint32_t)(grants.size() / 3) | (uint32_t)(rolese.size() / 2) << 8 | (uint32_t)slot_objs.size() << 16 |
         (uint32_t)roots.size() << 24;
  w[1] = (uint32_t)tse.size() | (uint32_t)hr_keys.size() << 8;

  const JV* sid = get(subj, "id");
  check_scalar(sid);
  // ACL_NONE (acs_layout.h): verifyACL false for every rule, rule-independently and without an
  // error (encoder._acl_none)
  if (acl_state == ACL_CONTINUE && !(flags & RQ_SUBJ_MISSING) && ((flags & RQ_RA_EMPTY) || (flags & RQ_HRS_ITERABLE))) {
    bool none;
    if ((flags & RQ_RA_EMPTY) || !(flags & (RQ_ACT_CREATE | RQ_ACT_RMD))) {
      none = true;
    } else if (tse.empty()) {
      none = false;
    } else if (flags & RQ_ACT_CREATE) {
      none = false;
      for (const auto& e : tse) {
        if (e.first == C.urn[U_USER]) continue;
        bool scoped = false;
        for (size_t k = 0; k + 1 < rolese.size() && !scoped; k += 2) scoped = rolese[k + 1] == e.first;
        if (!scoped) none = true;
      }
    } else {  // read / modify / delete
      none = true;
      const uint32_t sid_id = intern(sid);
      for (const auto& e : tse) {
        for (const JV* v : e.second) {
          const uint32_t x = intern(v);
          if (e.first == C.urn[U_USER] && x == sid_id) none = false;
          for (size_t g = 0; g + 2 < grants.size() && none; g += 3)
            if (grants[g + 1] == e.first && grants[g + 2] == x) none = false;
        }
      }
    }
    if (none) {
      flags = (flags & ~(3u << RQ_ACL_SHIFT)) | ACL_NONE << RQ_ACL_SHIFT;
      hints |= HINT_ACL_NONE;
    }
  }
  SECT(5);
  ReqHdr h{};
  h.flags = flags;
  h.nres = (uint8_t)nr;
  h.nsubj = (uint8_t)ns;
  h.nact = (uint8_t)na;
  h.nroles = (uint8_t)n_ras;
  h.subject_id = intern(sid);
  Pair sp[SMAX] = {}, ap[AMAX] = {};
  for (uint32_t k = 0; k < ns; ++k) sp[k] = Pair{intern(get(&subjects[k], "id")), intern(get(&subjects[k], "value"))};
  for (uint32_t k = 0; k < na; ++k) ap[k] = Pair{intern(get(&actions[k], "id")), intern(get(&actions[k], "value"))};
  // commit (nothing above wrote the batch: an Unsupported leaves no partial request): the
  // request line, then the rows past it as this thread's extension record (offsets are
  // thread-local until the batch is assembled)
  h.arena_off = (uint32_t)arena.size();
  arena.insert(arena.end(), w.begin(), w.end());
  ReqLine& L = B.lines[i];
  L = ReqLine{};
  L.h = h;
  for (uint32_t j = 0; j < nr && j < (uint32_t)LINE_RES; ++j) L.res[j] = rows[j];
  L.s0 = sp[0];
  L.s1 = sp[1];
  L.a0 = ap[0];
  L.r0 = roles[0];
  L.r1 = roles[1];
  if (!(flags & RQ_NO_TARGET)) {
    L.ar0 = w[0];
    L.ar1 = w[1];
  }
  const ExtGeom g = ext_geom(nr, ns, na, n_ras);
  if (g.words) {
    L.ext = 1u + (uint32_t)(ext.size() / 4);
    const size_t x = ext.size();
    ext.resize(x + g.words, 0u);
    uint32_t* d = ext.data() + x;
    for (uint32_t j = LINE_RES; j < nr; ++j) memcpy(d + 4 * (j - LINE_RES), &rows[j], 16);
    for (uint32_t j = LINE_SUBJ; j < ns; ++j) memcpy(d + g.subj + 2 * (j - LINE_SUBJ), &sp[j], 8);
    for (uint32_t j = LINE_ACT; j < na; ++j) memcpy(d + g.act + 2 * (j - LINE_ACT), &ap[j], 8);
    for (uint32_t j = LINE_ROLES; j < n_ras; ++j) d[g.roles + (j - LINE_ROLES)] = roles[j];
  }
  SECT(6);
}

}  // namespace

// ------------------------------------------------------------------ candidate classes
namespace {

using Row = std::vector<uint32_t>;

struct Classes {
  acs_codec& C;
  acs_codec_batch& B;
  int threads;
  Row valid;  // real node bits of the W-word layout
  std::vector<std::string> col_keys;  // per regex-matrix column: its value key ('' = padding)
  Classes(acs_codec& c, acs_codec_batch& b, int t) : C(c), B(b), threads(t) {
    valid.assign(C.W, 0);
    auto fill = [&](uint32_t off, uint32_t n) {
      for (uint32_t k = 0; k < n; ++k) valid[off + (k >> 5)] |= 1u << (k & 31);
    };
    fill(0, C.S);
    fill(C.ws, C.P);
    fill(C.ws + C.wp, C.R);
  }
  void set_node(Row& r, uint32_t g) const { r[C.node_word(g)] |= C.node_bit(g); }

  // entity_candidates: nodes whose target can hit the column's value (or always candidates)
  std::shared_ptr<const Row> entity_row(const std::string& key, const std::vector<uint8_t>& cells) {
    {
      std::lock_guard<std::mutex> lock(C.col_mu);
      auto it = C.ent_rows.find(key);
      if (it != C.ent_rows.end()) return it->second;
    }
    auto row = std::make_shared<Row>(C.always_bits);
    uint32_t exact = NONE32;
    if (key[0] == 'm') exact = ID_UNDEF;
    else if (key[0] == 'n') exact = ID_NULL;
    else exact = C.lookup(std::string_view(key).substr(1));
    uint32_t exact_row = NONE32;
    if (exact != NONE32) {
      auto r = C.row_of_id.find(exact);
      if (r != C.row_of_id.end()) exact_row = r->second;
    }
    for (uint32_t r = 0; r < (uint32_t)C.rx_pat.size(); ++r) {
      if (!((cells[r] & HIT_LIKE) || r == exact_row)) continue;
      for (uint32_t k = C.row_ptr[r]; k < C.row_ptr[r + 1]; ++k) set_node(*row, C.row_nodes[k]);
    }
    std::lock_guard<std::mutex> lock(C.col_mu);
    if (C.ent_rows.size() > 65536) C.ent_rows.clear();
    C.ent_rows.emplace(key, row);
    return row;
  }

  // action_candidates row 2 + k: nodes whose target actions all loosely equal the pair
  std::shared_ptr<const Row> action_row(uint32_t id, uint32_t value) {
    const uint64_t key = (uint64_t)id << 32 | value;
    const bool cacheable = id < C.n_dict && value < C.n_dict;
    if (cacheable) {
      std::lock_guard<std::mutex> lock(C.col_mu);
      auto it = C.act_rows.find(key);
      if (it != C.act_rows.end()) return it->second;
    }
    auto row = std::make_shared<Row>(no_action_row());  // nodes listing no action, then:
    auto leq = [](uint32_t a, uint32_t b) { return a == b || (a <= ID_NULL && b <= ID_NULL); };
    for (uint32_t g : C.need_act_nodes) {
      const NodeRec& N = C.nodes[g];
      bool ok = true;
      for (uint32_t k = 0; k < N.act_n && ok; ++k) {
        const Pair& pr = C.pairs[N.act_off + k];
        ok = leq(pr.id, id) && leq(pr.value, value);
      }
      if (ok) set_node(*row, g);
    }
    if (cacheable) {
      std::lock_guard<std::mutex> lock(C.col_mu);
      if (C.act_rows.size() > 4096) C.act_rows.clear();
      C.act_rows.emplace(key, row);
    }
    return row;
  }

  Row no_action_row() const {  // row 0: a request without action attributes
    Row r(C.W, 0u);
    for (uint32_t w = 0; w < C.W; ++w) r[w] = valid[w] & ~C.need_act_bits[w];
    return r;
  }

  Row role_filter_fn(const int32_t* rows, int nrows) const {
    Row r(C.norole_bits);
    for (int k = 0; k < nrows; ++k)
      for (uint32_t g : C.role_node_list[rows[k]]) r[C.node_word(g)] |= C.node_bit(g);
    return r;
  }

  // set section: keep a set only if one of its policies is kept and it has policies
  void sets_need_policies(Row& r) const {
    each_bit(r, 0, C.S, [&](uint32_t s) {
      const NodeRec& N = C.nodes[s];
      if (!range_any(r, C.ws, N.child_begin, N.child_end)) r[s >> 5] &= ~(1u << (s & 31));
    });
  }

  static bool bit(const Row& r, uint32_t off, uint32_t i) { return (r[off + (i >> 5)] >> (i & 31)) & 1u; }

  // any bit of [b, e) set in the section at word `off`
  static bool range_any(const Row& r, uint32_t off, uint32_t b, uint32_t e) {
    if (b >= e) return false;
    const uint32_t wb = b >> 5, we = (e - 1) >> 5;
    const uint32_t mb = ~0u << (b & 31), me = ~0u >> (31 - ((e - 1) & 31));
    if (wb == we) return (r[off + wb] & mb & me) != 0;
    if (r[off + wb] & mb) return true;
    for (uint32_t w = wb + 1; w < we; ++w)
      if (r[off + w]) return true;
    return (r[off + we] & me) != 0;
  }

  // f(i) for each set bit i of the n-bit section at word `off` (ascending)
  template <class F>
  static void each_bit(const Row& r, uint32_t off, uint32_t n, F f) {
    for (uint32_t w = 0; w < (n + 31) / 32; ++w)
      for (uint32_t x = r[off + w]; x; x &= x - 1) f(w * 32 + (uint32_t)__builtin_ctz(x));
  }

  // [S | P | R] row -> [S | P | useful S | useful P | R] (candidates._useful / _assemble);
  // thr: the column's throwing policies (P bits), or nullptr
  // candidates.resource_verdicts for one column: exact true / false, RegExp true / false of
  // an empty or entity-only target, per policy (P bits) and rule (R bits)
  struct ResV {
    Row p[4], r[4];
  };
  std::vector<std::unique_ptr<ResV>> resv;  // per column + the no-entity column

  // resv[c] for column c (c == ncols: the no-entity column); resv sized ncols + 1 beforehand
  void build_resv_column(uint32_t c, uint32_t ncols) {
    auto v = std::make_unique<ResV>();
    const bool none = c == ncols, real = none || !col_keys[c].empty();
    // an empty resources list: exact and RegExp match known true
    v->p[0] = v->p[2] = C.res_empty_p;
    v->r[0] = v->r[2] = C.res_empty_r;
    // an entity-only list (real columns): known false unless it lists the value's exact row or
    // a RegExp row whose cell the value touched — those nodes are redone below
    if (real) {
      v->p[1] = v->p[3] = C.ent_only_p;
      v->r[1] = v->r[3] = C.ent_only_r;
    } else {
      v->p[1].assign(C.res_empty_p.size(), 0u);
      v->p[3] = v->p[1];
      v->r[1].assign(C.res_empty_r.size(), 0u);
      v->r[3] = v->r[1];
    }
    if (!none && real) {
      const std::string& key = col_keys[c];
      uint32_t exact_row = NONE32;
      uint32_t id = key[0] == 'm' ? ID_UNDEF : key[0] == 'n' ? ID_NULL : C.lookup(std::string_view(key).substr(1));
      if (id != NONE32) {
        auto it = C.row_of_id.find(id);
        if (it != C.row_of_id.end()) exact_row = it->second;
      }
      const uint8_t* cells = B.rx.data() + (size_t)c * B.rx_rows;
      const uint32_t nrx = (uint32_t)C.rx_pat.size();
      for (uint32_t rrow = 0; rrow < nrx; ++rrow) {
        if (!cells[rrow] && rrow != exact_row) continue;
        for (uint32_t k = C.row_ptr[rrow]; k < C.row_ptr[rrow + 1]; ++k) {
          const uint32_t g = C.row_nodes[k];
          if (g < C.S) continue;
          const uint16_t tf = (uint16_t)C.nodes[g].tflags;
          if ((tf & TF_RES_EMPTY) || !(tf & TF_RES_ENT_ONLY)) continue;
          const bool pol = g < C.S + C.P;
          const uint32_t l = pol ? g - C.S : g - C.S - C.P;
          Row* out = pol ? v->p : v->r;
          bool xt = false, em = false, thrown = false;
          for (uint32_t q = C.spec_ptr[g]; q < C.spec_ptr[g + 1]; ++q) {
            const uint32_t row = C.spec_idx[q];
            if (row == exact_row) xt = true;
            const uint8_t cell = row < nrx ? cells[row] : 0;
            if (cell & (C_RX_THROW_TYPE | C_RX_THROW_SYNTAX | C_RX_HOST)) thrown = true;
            if (cell & C_RX_HIT) em = true;
            else if (cell & C_RX_RESET) em = false;
          }
          const uint32_t b = 1u << (l & 31), w = l >> 5;
          for (int s = 0; s < 4; ++s) out[s][w] &= ~b;
          out[xt ? 0 : 1][w] |= b;
          if (!thrown) out[em ? 2 : 3][w] |= b;
        }
      }
    }
    resv[c] = std::move(v);
  }

  // the verdict sections of one class (candidates._verdicts): pc column, a action key,
  // roles / nroles the class's sorted role rows.  Word-parallel over the policy and rule
  // sections: per node, subjects known true (empty list, or a required role the class holds) /
  // false (a required role it lacks), actions known true (none listed, or the class's single
  // pair matches) / false, and the column's resource verdicts
  void verdicts(Row& out, uint32_t pc, uint32_t a, const int32_t* roles, int nroles, bool role_filter,
                bool action_filter, const std::vector<std::shared_ptr<const Row>>& arow) const {
    const ResV& rv = *resv[pc];
    const Row& A = *arow[action_filter ? a : 1u];
    const bool fixed = action_filter && a != 1;
    Row in;  // nodes whose required role the class holds (| role-free nodes, masked off below)
    if (role_filter) in = role_filter_fn(roles, nroles);
    for (int sec = 0; sec < 2; ++sec) {
      const bool pol = sec == 0;
      const uint32_t base = pol ? C.ws : C.ws + C.wp, nw = pol ? C.wp : C.wr;
      const Row* res = pol ? rv.p : rv.r;
      for (uint32_t j = 0; j < nw; ++j) {
        const uint32_t w = base + j, tg = C.tgt_bits[w];
        if (!tg) continue;
        const uint32_t sr = C.subj_role_bits[w], inw = role_filter ? in[w] & sr : 0u;
        const uint32_t subj_t = C.subj_empty_bits[w] | inw, subj_f = role_filter ? sr & ~inw : 0u;
        const uint32_t need = C.need_act_bits[w];
        const uint32_t act_t = ~need | (fixed ? A[w] : 0u), act_f = fixed ? need & ~A[w] : 0u;
        const uint32_t both_t = subj_t & act_t, any_f = subj_f | act_f;
        const uint32_t xt = both_t & res[0][j], xf = any_f | res[1][j], rt = both_t & res[2][j],
                       rf = any_f | res[3][j];
        if (pol) {
          out[C.WV + j] |= xt & tg;
          out[C.WV + C.wp + j] |= xf & tg;
          out[C.WV + 2 * C.wp + j] |= rt & tg;
          out[C.WV + 3 * C.wp + j] |= rf & tg;
        } else {
          out[C.WV + 4 * C.wp + j] |= (xt | (xf & rt)) & tg;
        }
      }
    }
  }

  // policies whose target reads a throwing (or host) RegExp cell of column c
  // (candidates.throw_policies); nullptr when none
  std::unique_ptr<Row> throw_row(uint32_t c) const {
    if (col_keys[c].empty()) return nullptr;
    std::unique_ptr<Row> out;
    const uint8_t* cells = B.rx.data() + (size_t)c * B.rx_rows;
    for (uint32_t r = 0; r < (uint32_t)C.rx_pat.size(); ++r) {
      if (!(cells[r] & (C_RX_THROW_TYPE | C_RX_THROW_SYNTAX | C_RX_HOST))) continue;
      for (uint32_t k = C.row_ptr[r]; k < C.row_ptr[r + 1]; ++k) {
        const uint32_t g = C.row_nodes[k];
        if (g < C.S || g >= C.S + C.P) continue;
        if (!out) out = std::make_unique<Row>(C.wp ? C.wp : 1, 0u);
        (*out)[(g - C.S) >> 5] |= 1u << ((g - C.S) & 31);
      }
    }
    return out;
  }

  Row assemble(const Row& r, const Row* thr) const {
    Row out(C.W2, 0u);
    std::copy(r.begin(), r.begin() + C.ws + C.wp, out.begin());
    std::copy(r.begin() + C.ws + C.wp, r.end(), out.begin() + 2 * C.ws + 2 * C.wp);
    const uint32_t wsu = C.ws + C.wp, wpu = 2 * C.ws + C.wp, rr = C.ws + C.wp;
    each_bit(r, C.ws, C.P, [&](uint32_t q) {
      const NodeRec& N = C.nodes[C.S + q];
      if (C.pol_static[q] || (thr && bit(*thr, 0, q)) || range_any(r, rr, N.child_begin, N.child_end))
        out[wpu + (q >> 5)] |= 1u << (q & 31);
    });
    each_bit(r, 0, C.S, [&](uint32_t s) {
      const NodeRec& N = C.nodes[s];
      if (C.set_null[s] || range_any(out, wpu, N.child_begin, N.child_end)) out[wsu + (s >> 5)] |= 1u << (s & 31);
    });
    return out;
  }

  Row class_row(uint32_t pc, uint32_t a, const int32_t* roles, int nroles, bool role_filter,
                const std::vector<std::shared_ptr<const Row>>& ent,
                const std::vector<std::shared_ptr<const Row>>& arow) const {
    Row r(*ent[pc]);
    const Row& A = *arow[a];
    for (uint32_t w = 0; w < C.W; ++w) r[w] &= A[w] & valid[w];
    if (role_filter) {
      const Row f = role_filter_fn(roles, nroles);
      for (uint32_t w = 0; w < C.W; ++w) r[w] &= f[w];
    }
    sets_need_policies(r);
    return r;
  }

  // Composed-level row (candidates.py "composed", _useful_relaxed): candidate policies and rules
  // with the roles' test, candidate sets and the useful sections role-relaxed so that the OR of
  // two rows covers the joint key's.  [S | P | useful S | useful P | R] like assemble.
  Row composed_row(uint32_t pc, uint32_t a, const int32_t* roles, int nroles, const Row* thr,
                   const std::vector<std::shared_ptr<const Row>>& ent,
                   const std::vector<std::shared_ptr<const Row>>& arow) const {
    Row base(*ent[pc]);  // role-free: entity & action
    const Row& A = *arow[a];
    for (uint32_t w = 0; w < C.W; ++w) base[w] &= A[w] & valid[w];
    Row r(base);
    const Row f = role_filter_fn(roles, nroles);
    for (uint32_t w = 0; w < C.W; ++w) r[w] &= f[w];
    sets_need_policies(base);  // role-free sets holding a role-free candidate policy
    Row out(C.W2, 0u);
    std::copy(base.begin(), base.begin() + C.ws, out.begin());
    std::copy(r.begin() + C.ws, r.begin() + C.ws + C.wp, out.begin() + C.ws);
    std::copy(r.begin() + C.ws + C.wp, r.end(), out.begin() + 2 * C.ws + 2 * C.wp);
    const uint32_t wsu = C.ws + C.wp, wpu = 2 * C.ws + C.wp, rr = C.ws + C.wp;
    each_bit(base, C.ws, C.P, [&](uint32_t q) {  // r's policies are base's with the roles' test
      const NodeRec& N = C.nodes[C.S + q];
      const bool use = (bit(r, C.ws, q) && (C.pol_static[q] || (thr && bit(*thr, 0, q)))) ||
                       range_any(r, rr, N.child_begin, N.child_end);
      if (use) out[wpu + (q >> 5)] |= 1u << (q & 31);
    });
    each_bit(base, 0, C.S, [&](uint32_t s) {
      const NodeRec& N = C.nodes[s];
      if (C.set_null[s] || range_any(out, wpu, N.child_begin, N.child_end)) out[wsu + (s >> 5)] |= 1u << (s & 31);
    });
    return out;
  }

  void run();
};

uint64_t row_hash(const uint32_t* r, size_t n) { return hash_bytes((const char*)r, n * 4); }

// Run f(t, lo, hi) over [0, n) cut into `threads` contiguous ranges (t = 0 on this thread).
template <class F>
void parallel_ranges(int threads, size_t n, F f) {
  int T = threads < 1 ? 1 : threads;
  if ((size_t)T > n / 4096 + 1) T = (int)(n / 4096 + 1);
  acs_pool::run(T, [&](int t) { f(t, n * t / T, n * (t + 1) / T); });
}

// Open-addressing u64 -> u32 map (linear probing; key ~0 is reserved).
class U64Map {
 public:
  explicit U64Map(size_t expect = 64) {
    size_t cap = 64;
    while (cap < 2 * expect) cap <<= 1;
    k_.assign(cap, ~0ull);
    v_.resize(cap);
  }
  // the value for key (inserting `fresh` if absent); *inserted: whether it was absent
  uint32_t get_or_put(uint64_t key, uint32_t fresh, bool* inserted) {
    if (2 * (n_ + 1) > k_.size()) grow();
    size_t m = k_.size() - 1, x = (size_t)(mix(key) & m);
    for (;; x = (x + 1) & m) {
      if (k_[x] == key) {
        *inserted = false;
        return v_[x];
      }
      if (k_[x] == ~0ull) {
        k_[x] = key;
        v_[x] = fresh;
        ++n_;
        *inserted = true;
        return fresh;
      }
    }
  }

 private:
  static uint64_t mix(uint64_t h) {
    h ^= h >> 33;
    h *= 0xFF51AFD7ED558CCDull;
    h ^= h >> 33;
    return h;
  }

 public:
  static uint64_t mixed(uint64_t h) { return mix(h); }

 private:
  void grow() {
    std::vector<uint64_t> k(std::move(k_));
    std::vector<uint32_t> v(std::move(v_));
    k_.assign(k.size() * 2, ~0ull);
    v_.resize(k.size() * 2);
    n_ = 0;
    bool ins;
    for (size_t x = 0; x < k.size(); ++x)
      if (k[x] != ~0ull) get_or_put(k[x], v[x], &ins);
  }
  std::vector<uint64_t> k_;
  std::vector<uint32_t> v_;
  size_t n_ = 0;
};

#if defined(ACS_CODEC_TIMING)
std::atomic<uint64_t> g_cls_ns[8];
#define CLS_T(k)                                                                          \
  do {                                                                                    \
    const auto t_ = std::chrono::steady_clock::now();                                     \
    g_cls_ns[k] += (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(t_ - cls_t0_).count(); \
    cls_t0_ = t_;                                                                         \
  } while (0)
#else
#define CLS_T(k) \
  do {           \
  } while (0)
#endif
void Classes::run() {
#if defined(ACS_CODEC_TIMING)
  auto cls_t0_ = std::chrono::steady_clock::now();
#endif
  const uint32_t n = B.n, W = C.W2;  // output rows: [S | P | useful S | useful P | R]
  const uint32_t ncols = B.rx_cols;
  B.cand_words = W;
  B.cand_wp = C.ws;
  B.cand_wsu = C.ws + C.wp;
  B.cand_wpu = 2 * C.ws + C.wp;
  B.cand_wr = 2 * C.ws + 2 * C.wp;
  B.cand_wv = C.WV;
  // per request: primary column (candidates.primary_columns), action key, sorted role rows
  const bool have_roles = !C.role_ids.empty();
  const int RW = RMAX;
  std::vector<uint32_t> pcol(n, ncols);
  std::vector<uint8_t> active(n, 0);
  std::vector<int32_t> rs((size_t)n * RW, -1);
  std::vector<uint8_t> nrs(n, 0);
  std::atomic<bool> any_active{false};
  parallel_ranges(threads, n, [&](int, size_t lo, size_t hi) {
    bool any = false;
    for (uint32_t i = (uint32_t)lo; i < hi; ++i) {
      const ReqHdr& hd = B.h(i);
      bool seen = false;
      for (uint32_t j = 0; j < hd.nres; ++j) {
        const ReqRes q = B.res_at(i, j);
        if (!(q.kind & K_ENT)) continue;
        if (!seen) pcol[i] = q.col;
        else if (pcol[i] != q.col) pcol[i] = PCOL_ALL;
        seen = true;
      }
      active[i] = pcol[i] != PCOL_ALL && !(hd.flags & (RQ_HOST | RQ_NO_TARGET));
      any = any || active[i];
      if (!have_roles || !(hd.flags & RQ_RA_TRUTHY)) continue;
      int32_t* r = &rs[(size_t)i * RW];
      int m = 0;
      for (uint32_t k = 0; k < hd.nroles; ++k) {
        const uint32_t v = B.role_at(i, k);
        auto it = std::lower_bound(C.role_ids.begin(), C.role_ids.end(), v);
        if (it != C.role_ids.end() && *it == v) r[m++] = (int32_t)(it - C.role_ids.begin());
      }
      std::sort(r, r + m);
      m = (int)(std::unique(r, r + m) - r);
      nrs[i] = (uint8_t)m;
    }
    if (any) any_active = true;
  });
  CLS_T(0);
  auto finish = [&](const std::vector<uint32_t>& cls) {
    parallel_ranges(threads, n, [&](int, size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i) {
        uint32_t& f = B.lines[i].h.flags;
        f = (f & 0xFFFFu) | cls[i] << RQ_PCOL_SHIFT;
      }
    });
  };
  auto set_rows = [&](size_t rows) {
    B.cand_b = C.pool->acquire(rows * W * sizeof(uint32_t));
    B.cand = (uint32_t*)B.cand_b.p;
    B.cand_rows = (uint32_t)rows;
  };
  if (!any_active) {
    set_rows(1);
    memset(B.cand, 0, (size_t)W * 4);
    finish(std::vector<uint32_t>(n, PCOL_ALL));
    return;
  }
  // action keys (candidates.action_keys): 0 none, 1 several / unfiltered, 2 + k a single pair
  std::vector<uint32_t> ak(n, 0);
  std::vector<uint64_t> pairs_k;
  {
    // per-thread counts of the single-action pairs (few distinct), merged
    std::vector<std::unordered_map<uint64_t, uint32_t>> local(threads < 1 ? 1 : threads);
    parallel_ranges(threads, n, [&](int t, size_t lo, size_t hi) {
      auto& m = local[t];
      for (size_t i = lo; i < hi; ++i)
        if (B.h((uint32_t)i).nact == 1) ++m[(uint64_t)B.lines[i].a0.id << 32 | B.lines[i].a0.value];
    });
    std::unordered_map<uint64_t, uint32_t> cnt;
    for (const auto& m : local)
      for (const auto& kv : m) cnt[kv.first] += kv.second;
    std::vector<std::pair<uint64_t, uint32_t>> v(cnt.begin(), cnt.end());
    std::sort(v.begin(), v.end());
    if (v.size() > 62) {
      std::stable_sort(v.begin(), v.end(), [](auto& a, auto& b) { return a.second > b.second; });
      v.resize(62);
      std::sort(v.begin(), v.end());
    }
    std::unordered_map<uint64_t, uint32_t> idx;
    for (uint32_t k = 0; k < v.size(); ++k) {
      idx[v[k].first] = k;
      pairs_k.push_back(v[k].first);
    }
    parallel_ranges(threads, n, [&](int, size_t lo, size_t hi) {  // idx: read only here
      for (size_t i = lo; i < hi; ++i) {
        const uint32_t na = B.h((uint32_t)i).nact;
        if (na == 0) ak[i] = 0;
        else if (na > 1) ak[i] = 1;
        else {
          auto it = idx.find((uint64_t)B.lines[i].a0.id << 32 | B.lines[i].a0.value);
          ak[i] = it == idx.end() ? 1 : 2 + it->second;
        }
      }
    });
  }
  CLS_T(1);
  // per-batch inputs of a row computation, built only when some key misses the cache
  std::vector<std::shared_ptr<const Row>> ent, arow;
  std::vector<std::unique_ptr<Row>> thr;
  bool prepared = false;
  auto prepare = [&] {
    if (prepared) return;
    prepared = true;
    ent.assign(ncols + 1, nullptr);
    resv.clear();
    resv.resize(ncols + 1);
    thr.clear();
    thr.resize(ncols + 1);
    arow.assign(2 + pairs_k.size(), nullptr);
    // per column (entity row, resource verdicts, throwing policies) and per action key, over
    // the threads: each item writes only its own slot (entity / action rows: the codec's
    // caches, under their lock)
    const size_t ncol_items = (size_t)ncols + 1, items = ncol_items + arow.size();
    std::atomic<size_t> next{0};
    auto work = [&] {
      for (;;) {
        const size_t x = next.fetch_add(1);
        if (x >= items) return;
        if (x >= ncol_items) {
          const size_t k = x - ncol_items;
          if (k == 0) arow[0] = std::make_shared<Row>(no_action_row());
          else if (k == 1) arow[1] = std::make_shared<Row>(valid);
          else arow[k] = action_row((uint32_t)(pairs_k[k - 2] >> 32), (uint32_t)pairs_k[k - 2]);
          continue;
        }
        const uint32_t c = (uint32_t)x;
        build_resv_column(c, ncols);
        if (c == ncols || col_keys[c].empty()) {
          ent[c] = std::make_shared<Row>(C.always_bits);
          continue;
        }
        std::vector<uint8_t> cells(B.rx.begin() + (size_t)c * B.rx_rows,
                                   B.rx.begin() + (size_t)c * B.rx_rows + C.rx_pat.size());
        ent[c] = entity_row(col_keys[c], cells);
        thr[c] = throw_row(c);
      }
    };
    acs_pool::run((int)std::min<size_t>((size_t)std::max(threads, 1), std::max<size_t>(items, 1)),
                  [&](int) { work(); });
  };
  // the column part of a cache key: the entity value (a padding column: never a key)
  auto col_key = [&](uint32_t c) -> std::string {
    if (c >= ncols) return std::string("\x01", 1);  // no entity attribute
    return "\x02" + col_keys[c];
  };
  const size_t KEY_ROW_BYTES = size_t(512) << 20, ROLE_ROW_BYTES = size_t(256) << 20;
  const uint32_t MAX_CLASSES = PCOL_ALL;
  // key levels (candidates.LEVELS): 0 entity+roles+action, 1 composed (per-role rows the kernel
  // ORs, two required roles), 2 entity+action (+ role factor), 3 entity; tests pin one
  // (candidates.FORCE_LEVEL) through acs_internal_codec_force_level
  const int force = C.force_level;
  const int first_level = force >= 0 && force <= 3 ? force : (n <= C.level0_given_up.load() ? 1 : 0);
  const int last_level = force >= 0 && force <= 3 ? first_level + 1 : 4;
  const bool packable = C.role_ids.size() < 512;
  // requests with exactly two required roles (the composed level's second keys)
  std::vector<uint32_t> two;
  for (uint32_t i = 0; i < n; ++i)
    if (active[i] && nrs[i] == 2) two.push_back(i);
  for (int lv = first_level; lv < last_level; ++lv) {
    const int level = lv == 1 && !have_roles ? 0 : lv;  // no target requires a role: role-free keys
    const bool composed = level == 1;
    const bool role_filter = level <= 1 && have_roles;
    const bool action_filter = level < 3;
    // key items: item t < n is request t's (primary) key, item n + j the second key of two[j]
    // (composed level); each names its request and its role rows
    const size_t N = composed ? (size_t)n + two.size() : (size_t)n;
    auto req_of = [&](size_t t) -> uint32_t { return t < n ? (uint32_t)t : two[t - n]; };
    auto item_active = [&](size_t t) -> bool { return t >= n || active[t]; };
    // role rows of item t: level 0 all (ascending); composed: the largest (all past two) for a
    // primary, the second largest for a secondary
    auto roles_of = [&](size_t t, int* m) -> const int32_t* {
      const uint32_t i = req_of(t);
      const int32_t* r = &rs[(size_t)i * RW];
      const int k = nrs[i];
      if (!role_filter) {
        *m = 0;
        return r;
      }
      if (!composed || k > 2) {
        *m = k;
        return r;
      }
      if (k == 0) {
        *m = 0;
        return r;
      }
      *m = 1;
      return t < n ? r + (k - 1) : r + (k - 2);
    };
    bool pack_ok = packable;
    if (role_filter)
      for (uint32_t i = 0; i < n && pack_ok; ++i) pack_ok = nrs[i] <= 4;
    auto kv = [&](size_t t) -> uint64_t {  // pcol 16 | ak 6 | nrs 3 | 4 x 9-bit role rows
      const uint32_t i = req_of(t);
      uint64_t k = (uint64_t)(pcol[i] & 0xFFFF) << 48 | (uint64_t)(action_filter ? ak[i] : 0) << 42;
      int m;
      const int32_t* r = roles_of(t, &m);
      k |= (uint64_t)m << 36;
      for (int j = 0; j < m; ++j) k |= (uint64_t)r[j] << (9 * j);
      return k;
    };
    auto ks = [&](size_t t) -> std::string {
      const uint32_t i = req_of(t);
      std::string kb((const char*)&pcol[i], 4);
      if (action_filter) kb.append((const char*)&ak[i], 4);
      int m;
      const int32_t* r = roles_of(t, &m);
      kb.append((const char*)r, 4 * (size_t)m);
      return kb;
    };
    std::vector<uint32_t> key_of(N, NONE32), key_first;  // key_first: first item of each key
    // the level is given up (below) past this many keys: the merge stops there
    const size_t key_limit = level >= 3 ? ~size_t(0)
                             : std::min(W ? KEY_ROW_BYTES / ((size_t)W * 4) : ~size_t(0),
                                        level == 0 && force < 0 ? (size_t)n / 4 : ~size_t(0));
    bool over_limit = false;
    {
      int T = threads < 1 ? 1 : threads;
      if ((size_t)T > N / 4096 + 1) T = (int)(N / 4096 + 1);
      std::vector<std::vector<uint32_t>> firsts(T);
      parallel_ranges(T, N, [&](int t, size_t lo, size_t hi) {
        if (pack_ok) {
          U64Map m(1024);
          bool ins;
          for (size_t x = lo; x < hi; ++x) {
            if (!item_active(x)) continue;
            key_of[x] = m.get_or_put(kv(x), (uint32_t)firsts[t].size(), &ins);
            if (ins) firsts[t].push_back((uint32_t)x);
          }
        } else {
          std::unordered_map<std::string, uint32_t> m;
          for (size_t x = lo; x < hi; ++x) {
            if (!item_active(x)) continue;
            auto it = m.emplace(ks(x), (uint32_t)firsts[t].size());
            if (it.second) firsts[t].push_back((uint32_t)x);
            key_of[x] = it.first->second;
          }
        }
      });
      // merge: thread-local key index -> global key index, global keys in order of first
      // appearance (the first thread's range first: every thread's keys are in item order)
      std::vector<std::vector<uint32_t>> remap(T);
      if (pack_ok && T > 1) {
        // over the threads: keys split into T partitions by hash; partition p merges its keys
        // thread after thread, recording each new key's first item; the global order is the
        // sort by first item — the serial merge's order exactly
        const int Pn = T;
        auto part = [&](uint64_t k) { return (int)((U64Map::mixed(k) >> 32) % (uint64_t)Pn); };
        std::vector<std::vector<std::vector<uint32_t>>> fb(T, std::vector<std::vector<uint32_t>>(Pn));
        acs_pool::run(T, [&](int t) {
          for (uint32_t k = 0; k < firsts[t].size(); ++k) fb[t][part(kv(firsts[t][k]))].push_back(k);
        });
        std::vector<U64Map> pm;
        for (int q = 0; q < Pn; ++q) pm.emplace_back(1024);
        std::vector<std::vector<uint32_t>> pfirst(Pn);  // partition key j -> its first item
        acs_pool::run(Pn, [&](int q) {
          bool ins;
          for (int t = 0; t < T; ++t)
            for (const uint32_t k : fb[t][q]) {
              const uint32_t x = firsts[t][k];
              pm[q].get_or_put(kv(x), (uint32_t)pfirst[q].size(), &ins);
              if (ins) pfirst[q].push_back(x);
            }
        });
        size_t total = 0;
        for (const auto& v : pfirst) total += v.size();
        over_limit = total > key_limit;
        if (!over_limit) {
          std::vector<std::pair<uint32_t, uint32_t>> ord;  // (first item, partition << 24 | j)
          ord.reserve(total);
          for (int q = 0; q < Pn; ++q)
            for (uint32_t j = 0; j < pfirst[q].size(); ++j) ord.push_back({pfirst[q][j], (uint32_t)q << 24 | j});
          std::sort(ord.begin(), ord.end());
          std::vector<std::vector<uint32_t>> gid(Pn);
          for (int q = 0; q < Pn; ++q) gid[q].resize(pfirst[q].size());
          key_first.resize(total);
          for (uint32_t g = 0; g < total; ++g) {
            key_first[g] = ord[g].first;
            gid[ord[g].second >> 24][ord[g].second & 0xFFFFFFu] = g;
          }
          acs_pool::run(T, [&](int t) {
            bool ins;
            remap[t].resize(firsts[t].size());
            for (uint32_t k = 0; k < firsts[t].size(); ++k) {
              const uint64_t key = kv(firsts[t][k]);
              const int q = part(key);
              remap[t][k] = gid[q][pm[q].get_or_put(key, 0u, &ins)];
            }
          });
        }
      }
      U64Map gm(4096);
      std::unordered_map<std::string, uint32_t> gs;
      for (int t = 0; t < T && !over_limit && !(pack_ok && T > 1); ++t) {
        remap[t].resize(firsts[t].size());
        for (size_t k = 0; k < firsts[t].size() && !over_limit; ++k) {
          const uint32_t x = firsts[t][k];
          uint32_t g;
          bool ins;
          if (pack_ok) {
            g = gm.get_or_put(kv(x), (uint32_t)key_first.size(), &ins);
          } else {
            auto it = gs.emplace(ks(x), (uint32_t)key_first.size());
            g = it.first->second;
            ins = it.second;
          }
          if (ins) key_first.push_back(x);
          remap[t][k] = g;
          over_limit = key_first.size() > key_limit;
        }
      }
      if (!over_limit)
        parallel_ranges(T, N, [&](int t, size_t lo, size_t hi) {
        for (size_t x = lo; x < hi; ++x)
          if (key_of[x] != NONE32) key_of[x] = remap[t][key_of[x]];
      });
    }
    const size_t nk = key_first.size();
    CLS_T(2);
#if defined(ACS_CODEC_TIMING)
    if (getenv("ACS_CLS_DEBUG")) fprintf(stderr, "level %d: n %u N %zu keys %zu over %d\n", level, n, N, nk, (int)over_limit);
#endif
    // over the row budget; or joint keys covering fewer than 4 requests each (candidates.classes:
    // waves could not share them, and the rows would outweigh the requests)
    auto give_up = [&] {  // (level 0 as the first choice: remember the batch size)
      if (lv == 0 && force < 0) {
        uint32_t v = C.level0_given_up.load();
        while (v < n && !C.level0_given_up.compare_exchange_weak(v, n)) {
        }
      }
    };
    if (over_limit || (level < 3 && (nk * W * 4 > KEY_ROW_BYTES || (level == 0 && force < 0 && 4 * nk > (size_t)n)))) {
      give_up();
      continue;
    }
    // cache lookup by (level, entity value, action, roles); compute the misses in parallel
    std::vector<std::string> gkey(nk);
    std::vector<std::shared_ptr<const ClassEntry>> entry(nk);
    std::vector<uint32_t> miss;
    parallel_ranges(threads, nk, [&](int, size_t lo, size_t hi) {
    for (size_t k = lo; k < hi; ++k) {
      const uint32_t x = key_first[k], i = req_of(x);
      std::string g(1, (char)('0' + level));
      g += col_key(pcol[i]);
      g.push_back('\0');
      if (action_filter) {
        const uint32_t a = ak[i];
        if (a < 2) g.push_back((char)a);
        else g.append((const char*)&pairs_k[a - 2], 8);
      }
      g.push_back('|');
      int m;
      const int32_t* r = roles_of(x, &m);
      g.append((const char*)r, 4 * (size_t)m);
      gkey[k] = std::move(g);
    }
    });
    {  // lookups over the threads (shared lock: concurrent readers), misses in key order
      std::vector<uint8_t> hit(nk, 0);
      parallel_ranges(threads, nk, [&](int, size_t lo, size_t hi) {
        std::shared_lock<std::shared_mutex> lock(C.classes.mu);
        for (size_t k = lo; k < hi; ++k) {
          auto it = C.classes.by_key.find(gkey[k]);
          if (it != C.classes.by_key.end()) {
            entry[k] = it->second;
            hit[k] = 1;
          }
        }
      });
      for (size_t k = 0; k < nk; ++k)
        if (!hit[k]) miss.push_back((uint32_t)k);
    }
    B.classes_new += (uint32_t)miss.size();
    CLS_T(3);
    if (!miss.empty()) {
      prepare();
      std::vector<Row> rows(miss.size());
      std::atomic<size_t> next{0};
      auto work = [&] {
        for (;;) {
          const size_t m = next.fetch_add(1);
          if (m >= miss.size()) return;
          const uint32_t x = key_first[miss[m]], i = req_of(x);
          const uint32_t a = action_filter ? ak[i] : 1u;
          int nr;
          const int32_t* r = roles_of(x, &nr);
          const Row* tr = pcol[i] < ncols ? thr[pcol[i]].get() : nullptr;
          rows[m] = composed ? composed_row(pcol[i], a, r, nr, tr, ent, arow)
                             : assemble(class_row(pcol[i], a, r, nr, role_filter, ent, arow), tr);
          verdicts(rows[m], pcol[i], a, r, nr, role_filter, action_filter, arow);
        }
      };
      acs_pool::run((int)std::min<size_t>((size_t)std::max(threads, 1), std::max<size_t>(miss.size(), 1)),
                    [&](int) { work(); });
      std::unique_lock<std::shared_mutex> lock(C.classes.mu);
      ClassCache& K = C.classes;
      if (K.bytes > ClassCache::MAX_BYTES) K.clear_locked();  // this batch holds its own references
      for (size_t m = 0; m < miss.size(); ++m) {
        const uint64_t h = row_hash(rows[m].data(), W);
        std::shared_ptr<const ClassEntry> e;
        for (const auto& x : K.by_row[h])
          if (x->row == rows[m]) {
            e = x;
            break;
          }
        if (!e) {
          auto ne = std::make_shared<ClassEntry>();
          uint32_t c = 0;
          for (uint32_t w = 0; w < C.WV; ++w) c += (uint32_t)__builtin_popcount(rows[m][w]);  // filter sections
          ne->cost = c;
          ne->row = std::move(rows[m]);
          K.bytes += (size_t)W * 4 + 64;
          K.by_row[h].push_back(ne);
          e = ne;
        }
        K.by_key.emplace(gkey[miss[m]], e);
        K.bytes += gkey[miss[m]].size() + 64;
        entry[miss[m]] = e;
      }
    }
    // the batch's classes: its distinct rows, heaviest first (candidate nodes in the filter
    // sections; ties in order of first appearance), so the longest waves are dispatched first
    std::unordered_map<const ClassEntry*, uint32_t> uidx;
    std::vector<const ClassEntry*> uent;
    std::vector<uint32_t> cls_of_key(nk);
    for (size_t k = 0; k < nk; ++k) {
      auto it = uidx.emplace(entry[k].get(), (uint32_t)uent.size());
      if (it.second) uent.push_back(entry[k].get());
      cls_of_key[k] = it.first->second;
    }
    if (uent.size() > MAX_CLASSES && level < 3) {
      give_up();
      continue;
    }
    if (uent.size() > MAX_CLASSES) {
      acs_internal_set_error("acs_codec_encode: too many request classes");
      throw Unsup{"too many request classes"};
    }
    CLS_T(4);
    std::vector<uint32_t> order(uent.size()), rank(uent.size());
    for (size_t u = 0; u < uent.size(); ++u) order[u] = (uint32_t)u;
    std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return uent[a]->cost > uent[b]->cost; });
    for (size_t k = 0; k < order.size(); ++k) rank[order[k]] = (uint32_t)k;
    set_rows(uent.size());
    parallel_ranges(threads, uent.size() * (size_t)W / 1024 + 1, [&](int, size_t lo, size_t hi) {
      // rows split by bytes: chunk c covers classes [c * U / C, (c + 1) * U / C)
      const size_t U = uent.size(), Cn = uent.size() * (size_t)W / 1024 + 1;
      for (size_t u = U * lo / Cn; u < U * hi / Cn; ++u)
        memcpy(B.cand + (size_t)rank[u] * W, uent[u]->row.data(), (size_t)W * 4);
    });
    std::vector<uint32_t> cls(n, PCOL_ALL);
    parallel_ranges(threads, n, [&](int, size_t lo, size_t hi) {
      for (size_t i = lo; i < hi; ++i)
        if (active[i]) cls[i] = rank[cls_of_key[key_of[i]]];
    });
    if (composed) {
      // the second class of each two-role request: the heavier class first (the coherence
      // order groups by it), the same row once
      parallel_ranges(threads, two.size(), [&](int, size_t lo, size_t hi) {
        for (size_t j = lo; j < hi; ++j) {
          const uint32_t i = two[j], a = cls[i], b = rank[cls_of_key[key_of[n + j]]];
          cls[i] = a < b ? a : b;
          B.lines[i].cls2 = a == b ? 0u : (a < b ? b : a) + 1u;
        }
      });
    }
    finish(cls);
    CLS_T(5);
    if (role_filter || !have_roles) return;
    // role factor (candidates._role_factor): role-relaxed rows like the composed level's, one per
    // required role (and one for "no required role"; a request with more than two roles: one
    // of its whole role set), cached by (roles, the batch's may-throw policies).  role_key:
    // row | (1 + second row) << 16 for a request with two required roles
    std::unordered_map<std::string, uint32_t> sidx;
    std::vector<std::pair<uint32_t, int>> key_roles;  // (request, 0 all / 1 largest / 2 second)
    std::vector<uint32_t> rkey(n, 0xFFFFu);
    std::string kb;
    auto role_span = [&](uint32_t i, int which, int* m) -> const int32_t* {
      const int32_t* r = &rs[(size_t)i * RW];
      const int k = nrs[i];
      if (which == 0 || k > 2) {
        *m = k;
        return r;
      }
      if (k == 0) {
        *m = 0;
        return r;
      }
      *m = 1;
      return which == 1 ? r + (k - 1) : r + (k - 2);
    };
    auto key_id = [&](uint32_t i, int which) -> uint32_t {
      int m;
      const int32_t* r = role_span(i, which, &m);
      kb.assign((const char*)r, 4 * (size_t)m);
      auto it = sidx.find(kb);
      if (it == sidx.end()) {
        it = sidx.emplace(kb, (uint32_t)key_roles.size()).first;
        key_roles.emplace_back(i, which);
      }
      return it->second;
    };
    for (uint32_t i = 0; i < n; ++i) {
      if (!active[i]) continue;
      const uint32_t a = key_id(i, nrs[i] > 2 ? 0 : 1);
      rkey[i] = a;
      if (nrs[i] == 2) {
        const uint32_t b = key_id(i, 2);
        const uint32_t lo = a < b ? a : b, hi = a < b ? b : a;
        rkey[i] = lo | (lo == hi ? 0u : (hi + 1u) << 16);
      }
    }
    const size_t nkr = key_roles.size();
    if (nkr == 0 || nkr * W * 4 > ROLE_ROW_BYTES || nkr >= 0xFFFF) return;
    // the role side's useful sections keep every policy that may throw for some column
    Row thr_any(C.wp ? C.wp : 1, 0u);
    for (uint32_t c = 0; c < ncols; ++c) {
      std::unique_ptr<Row> t = prepared ? nullptr : throw_row(c);
      const Row* tr = prepared ? thr[c].get() : t.get();
      if (tr)
        for (uint32_t w = 0; w < thr_any.size(); ++w) thr_any[w] |= (*tr)[w];
    }
    const std::string thr_key((const char*)thr_any.data(), thr_any.size() * 4);
    B.role_bits.assign(nkr * W, 0u);
    std::vector<std::shared_ptr<const std::vector<uint32_t>>> rrow(nkr);
    std::vector<uint32_t> rmiss;
    std::vector<std::string> rkeys(nkr);
    {
      std::shared_lock<std::shared_mutex> lock(C.classes.mu);
      for (size_t k = 0; k < nkr; ++k) {
        int m;
        const int32_t* r = role_span(key_roles[k].first, key_roles[k].second, &m);
        rkeys[k].assign((const char*)r, 4 * (size_t)m);
        rkeys[k] += '|';
        rkeys[k] += thr_key;
        auto it = C.classes.role_rows.find(rkeys[k]);
        if (it != C.classes.role_rows.end()) rrow[k] = it->second;
        else rmiss.push_back((uint32_t)k);
      }
    }
    B.classes_new += (uint32_t)rmiss.size();
    const uint32_t wsu = C.ws + C.wp, wpu = 2 * C.ws + C.wp, rr = C.ws + C.wp;
    for (uint32_t k : rmiss) {
      int m;
      const int32_t* roles = role_span(key_roles[k].first, key_roles[k].second, &m);
      Row r = role_filter_fn(roles, m);
      for (uint32_t w = 0; w < C.W; ++w) r[w] &= valid[w];
      Row o(C.W2, 0u);
      // candidate sets: every set with policies (role-free, _role_factor's s_free)
      for (uint32_t s = 0; s < C.S; ++s)
        if (C.nodes[s].child_end > C.nodes[s].child_begin) o[s >> 5] |= 1u << (s & 31);
      std::copy(r.begin() + C.ws, r.begin() + C.ws + C.wp, o.begin() + C.ws);
      std::copy(r.begin() + C.ws + C.wp, r.end(), o.begin() + 2 * C.ws + 2 * C.wp);
      // role-relaxed useful sections (_useful_relaxed with every policy role-free)
      for (uint32_t q = 0; q < C.P; ++q) {  // every policy role-free
        const NodeRec& N = C.nodes[C.S + q];
        const bool use = (bit(r, C.ws, q) && (C.pol_static[q] || bit(thr_any, 0, q))) ||
                         range_any(r, rr, N.child_begin, N.child_end);
        if (use) o[wpu + (q >> 5)] |= 1u << (q & 31);
      }
      each_bit(o, 0, C.S, [&](uint32_t s) {
        const NodeRec& N = C.nodes[s];
        if (C.set_null[s] || range_any(o, wpu, N.child_begin, N.child_end)) o[wsu + (s >> 5)] |= 1u << (s & 31);
      });
      // the verdict sections are the class row's: the role side keeps them (all nodes)
      for (uint32_t q = 0; q < C.P; ++q)
        for (int s = 0; s < 4; ++s) o[C.WV + s * C.wp + (q >> 5)] |= 1u << (q & 31);
      for (uint32_t x = 0; x < C.R; ++x) o[C.WV + 4 * C.wp + (x >> 5)] |= 1u << (x & 31);
      rrow[k] = std::make_shared<const std::vector<uint32_t>>(std::move(o));
    }
    if (!rmiss.empty()) {
      std::unique_lock<std::shared_mutex> lock(C.classes.mu);
      for (uint32_t k : rmiss) {
        C.classes.role_rows.emplace(rkeys[k], rrow[k]);
        C.classes.bytes += (size_t)W * 4 + rkeys[k].size() + 64;
      }
    }
    for (size_t k = 0; k < nkr; ++k)
      std::copy(rrow[k]->begin(), rrow[k]->end(), B.role_bits.begin() + k * W);
    B.role_key = std::move(rkey);
    B.role_rows = (uint32_t)nkr;
    return;
  }
}

}  // namespace

// ------------------------------------------------------------------ batch driver + C ABI
namespace {

std::vector<std::pair<const char*, const char*>> array_items(const char* p, const char* e) {
  auto ws = [&] {
    while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  };
  std::vector<std::pair<const char*, const char*>> out;
  ws();
  if (p >= e || *p != '[') throw ParseError{"requests: expected a JSON array"};
  ++p;
  ws();
  if (p < e && *p == ']') {
    ++p;
  } else {
    for (;;) {
      ws();
      const char* b = p;
      p = skip_value(p, e);
      out.push_back({b, p});
      ws();
      if (p < e && *p == ',') {
        ++p;
        continue;
      }
      if (p < e && *p == ']') {
        ++p;
        break;
      }
      throw ParseError{"requests: expected ',' or ']'"};
    }
  }
  ws();
  if (p != e) throw ParseError{"requests: trailing text"};
  return out;
}

inline bool is_ws(char c) { return c == ' ' || c == '\n' || c == '\r' || c == '\t'; }

#ifndef ACS_AB_SERIAL_SPLIT  // A/B builds only: delimit the request array on one thread
#define ACS_AB_SERIAL_SPLIT 0
#endif

// 64-byte block masks (SSE2): bit i set where block[i] == c.
inline uint64_t block_eq(const __m128i v[4], char c) {
  const __m128i k = _mm_set1_epi8(c);
  uint64_t m = 0;
  for (int x = 0; x < 4; ++x) m |= (uint64_t)(uint16_t)_mm_movemask_epi8(_mm_cmpeq_epi8(v[x], k)) << (16 * x);
  return m;
}
inline uint64_t prefix_xor(uint64_t x) {
  x ^= x << 1;
  x ^= x << 2;
  x ^= x << 4;
  x ^= x << 8;
  x ^= x << 16;
  x ^= x << 32;
  return x;
}

// Byte-serial string / nesting scan of [q, e) from state (in_str, trailing backslash-run parity
// bs_odd): calls on(ptr, ch) for every '{' '[' '}' ']' ',' outside strings, returns the state.
template <class On>
inline void scan_serial(const char* q, const char* e, bool& in_str, bool& bs_odd, uint64_t& quotes, On&& on) {
  for (; q < e; ++q) {
    const char ch = *q;
    if (ch == '\\') {
      bs_odd = !bs_odd;
      continue;
    }
    const bool esc = bs_odd;
    bs_odd = false;
    if (ch == '"') {
      if (!esc) {
        in_str = !in_str;
        ++quotes;
      }
    } else if (!in_str && (ch == '{' || ch == '[' || ch == '}' || ch == ']' || ch == ',')) {
      on(q, ch);
    }
  }
}

// Scan [q, e) 64 bytes at a time: blocks without a backslash (and not following an odd
// backslash run) take the masks — quotes, the in-string bytes by prefix XOR, the structural
// bytes outside strings — the rest the serial scan.
template <class On>
inline void scan_chunk(const char* q, const char* e, bool& in_str, bool& bs_odd, uint64_t& quotes, On&& on) {
  while (e - q >= 64) {
    __m128i v[4];
    for (int x = 0; x < 4; ++x) v[x] = _mm_loadu_si128((const __m128i*)(q + 16 * x));
    const uint64_t bsl = block_eq(v, '\\');
    if (bsl || bs_odd) {
      scan_serial(q, q + 64, in_str, bs_odd, quotes, on);
      q += 64;
      continue;
    }
    const uint64_t qm = block_eq(v, '"');
    const uint64_t instr = prefix_xor(qm) ^ (in_str ? ~0ull : 0ull);
    const uint64_t opens = (block_eq(v, '{') | block_eq(v, '[')) & ~instr;
    const uint64_t closes = (block_eq(v, '}') | block_eq(v, ']')) & ~instr;
    const uint64_t commas = block_eq(v, ',') & ~instr;
    if (!on.block(__builtin_popcountll(opens), __builtin_popcountll(closes))) {
      uint64_t st = opens | closes | commas;
      while (st) {
        const int b = __builtin_ctzll(st);
        st &= st - 1;
        on(q + b, q[b]);
      }
    }
    const int nq = __builtin_popcountll(qm);
    quotes += (uint64_t)nq;
    if (nq & 1) in_str = !in_str;
    q += 64;
  }
  scan_serial(q, e, in_str, bs_odd, quotes, on);
}

// The top-level array's items, delimited on `threads` threads in three passes over T equal
// chunks of the array body (no guessing: every byte's string / nesting state is derived):
//   1. per chunk, the unescaped quotes (a quote is escaped by an odd run of backslashes,
//      which may begin in the previous chunk) -> by prefix parity, whether the chunk starts
//      inside a string;
//   2. per chunk, scanning with that state: its net nesting change and the commas outside
//      strings at its lowest nesting level (a comma between top-level items sits at absolute
//      depth 0, the lowest any byte of the body can have, so it is at the chunk's minimum);
//   3. serially, each chunk's starting depth: its minimum-level commas are item separators
//      exactly when that level is absolute depth 0.
// Both passes scan 64-byte blocks with SSE2 masks.  The items' own syntax is checked by the
// encoder's parser.  Serial delimiting ran at ~1-3 GB/s (0.39 s of a 0.77 s pipelined
// 1M-request c3 run).
std::vector<std::pair<const char*, const char*>> split_items(const char* p, const char* e, int threads) {
  const char* b = p;
  while (b < e && is_ws(*b)) ++b;
  const char* z = e;
  while (z > b && is_ws(z[-1])) --z;
  const size_t len = (size_t)(z - b);
  int T = threads < 1 ? 1 : threads;
  if (ACS_AB_SERIAL_SPLIT || len < (size_t(4) << 20) || T == 1 || *b != '[' || z[-1] != ']') return array_items(p, e);
  const char* body = b + 1;
  const char* end = z - 1;  // the closing ']'
  std::vector<const char*> c(T + 1);
  for (int t = 0; t <= T; ++t) c[t] = body + (size_t)(end - body) * t / T;
  std::vector<uint64_t> quotes(T, 0);
  std::vector<int64_t> delta(T, 0), lowest(T, 0);
  std::vector<std::vector<const char*>> commas(T);
  std::vector<char> start_in_str(T, 0), start_bs(T, 0);
  for (int t = 1; t < T; ++t) {  // the parity of the backslash run ending where chunk t starts
    size_t n = 0;
    while (c[t] - 1 - (ptrdiff_t)n >= body && c[t][-1 - (ptrdiff_t)n] == '\\') ++n;
    start_bs[t] = (char)(n & 1);
  }
  struct Quotes {  // pass 1: only the quote count matters
    bool block(int, int) { return true; }
    void operator()(const char*, char) {}
  };
  struct Depth {  // pass 2: nesting change, lowest level, the commas at it
    int64_t d = 0, lo = 0;
    std::vector<const char*> out;
    // a block whose closes cannot reach the lowest level holds no comma at it: counts suffice
    bool block(int opens, int closes) {
      if (d - closes > lo) {
        d += opens - closes;
        return true;
      }
      return false;
    }
    void operator()(const char* q, char ch) {
      if (ch == '{' || ch == '[') {
        ++d;
      } else if (ch == ',') {
        if (d == lo) out.push_back(q);
      } else if (--d < lo) {
        lo = d;
        out.clear();
      }
    }
  };
  auto pass1 = [&](int t) {
    bool in_str = false, bs = start_bs[t] != 0;
    uint64_t n = 0;
    Quotes on;
    scan_chunk(c[t], c[t + 1], in_str, bs, n, on);
    quotes[t] = n;
  };
  auto pass2 = [&](int t) {
    bool in_str = start_in_str[t] != 0, bs = start_bs[t] != 0;
    uint64_t n = 0;
    Depth on;
    scan_chunk(c[t], c[t + 1], in_str, bs, n, on);
    delta[t] = on.d;
    lowest[t] = on.lo;
    commas[t] = std::move(on.out);  // (a thread-local vector: no shared cache line per push)
  };
  auto run = [&](auto&& f) { acs_pool::run(T, [&](int t) { f(t); }); };
  run(pass1);
  uint64_t parity = 0;
  for (int t = 0; t < T; ++t) {
    start_in_str[t] = (char)(parity & 1);
    parity += quotes[t];
  }
  run(pass2);
  std::vector<const char*> seps;
  int64_t depth = 0;  // absolute depth at the chunk's start (0: between top-level items)
  for (int t = 0; t < T; ++t) {
    if (depth + lowest[t] < 0) return array_items(p, e);  // unbalanced: the serial path reports it
    if (depth + lowest[t] == 0) seps.insert(seps.end(), commas[t].begin(), commas[t].end());
    depth += delta[t];
  }
  if (depth != 0 || (parity & 1)) return array_items(p, e);
  std::vector<std::pair<const char*, const char*>> out;
  out.reserve(seps.size() + 1);
  const char* from = body;
  auto emit = [&](const char* x, const char* y, bool last) {
    while (x < y && is_ws(*x)) ++x;
    while (y > x && is_ws(y[-1])) --y;
    if (x == y) return last && seps.empty();  // "[ ]": no item; any other empty item is an error
    out.push_back({x, y});
    return true;
  };
  for (const char* sep : seps) {
    if (!emit(from, sep, false)) return array_items(p, e);  // the serial path says where
    from = sep + 1;
  }
  if (!emit(from, end, true)) return array_items(p, e);
  return out;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// acs_req_batch.perm (candidates.coherence_order): request indices grouped by [bucket | second
// class] (bucket = 1 + class; 0: an unfiltered request) or, with a role factor, role-major
// [role key | bucket]; stable (index order within a key).  Runs of equal buckets start on
// 64-lane wave boundaries (holes 0xFFFFFFFF) when the classes average 32 to 256 requests, or
// at least 32 and no request has a second class, and there is no role factor.  A parallel LSD radix sort of 32-bit (role-major: 48-bit) keys,
// 8-bit digits, a digit whose value every key shares skipped.
void coherence_order(acs_codec_batch& B, int threads) {
  const size_t n = B.n;
  const bool rmaj = !B.role_key.empty();
  std::vector<uint64_t> key(n), key2(n);
  std::vector<uint32_t> idx(n), idx2(n);
  int T = threads < 1 ? 1 : threads;
  if ((size_t)T > n / 65536 + 1) T = (int)(n / 65536 + 1);
  std::atomic<bool> any_cls2{false};
  parallel_ranges(T, n, [&](int, size_t lo, size_t hi) {
    uint32_t c2 = 0;
    for (size_t i = lo; i < hi; ++i) c2 |= B.lines[i].cls2;
    if (c2) any_cls2 = true;
    for (size_t i = lo; i < hi; ++i) {
      const uint32_t c = B.lines[i].h.flags >> RQ_PCOL_SHIFT;
      const uint32_t bucket = c < B.cand_rows ? c + 1u : 0u;
      if (rmaj) {  // [role row | 1 + second role row | bucket]
        const uint64_t rk = B.role_key[i];
        key[i] = (rk & 0xFFFFu) << 32 | (rk >> 16) << 16 | bucket;
      } else {
        key[i] = bucket << 16 | B.lines[i].cls2;
      }
      idx[i] = (uint32_t)i;
    }
  });
  std::vector<std::array<size_t, 256>> cnt(T);
  for (int sh = 0; sh < (rmaj ? 48 : 32); sh += 8) {
    auto range = [&](int t, size_t& lo, size_t& hi) {
      lo = n * t / T;
      hi = n * (t + 1) / T;
    };
    auto hist = [&](int t) {
      size_t lo, hi;
      range(t, lo, hi);
      cnt[t].fill(0);
      for (size_t x = lo; x < hi; ++x) ++cnt[t][(key[x] >> sh) & 255u];
    };
    acs_pool::run(T, hist);
    size_t total = 0;
    bool constant = false;
    for (uint32_t d = 0; d < 256 && !constant; ++d) {
      size_t c = 0;
      for (int t = 0; t < T; ++t) c += cnt[t][d];
      constant = c == n;
    }
    if (constant) continue;
    for (uint32_t d = 0; d < 256; ++d)  // per (digit, thread) exclusive offsets
      for (int t = 0; t < T; ++t) {
        const size_t c = cnt[t][d];
        cnt[t][d] = total;
        total += c;
      }
    auto scatter = [&](int t) {
      size_t lo, hi;
      range(t, lo, hi);
      std::array<size_t, 256>& o = cnt[t];
      for (size_t x = lo; x < hi; ++x) {
        const size_t at = o[(key[x] >> sh) & 255u]++;
        key2[at] = key[x];
        idx2[at] = idx[x];
      }
    };
    acs_pool::run(T, scatter);
    key.swap(key2);
    idx.swap(idx2);
  }
  const bool pad = !rmaj && n >= 32ull * B.cand_rows && (n < 256ull * B.cand_rows || !any_cls2);
  const int rs = 16;  // runs of equal buckets (key >> 16)
  size_t lanes = n;
  if (pad) {
    lanes = 0;
    for (size_t x = 0; x < n;) {
      size_t y = x + 1;
      while (y < n && (key[y] >> rs) == (key[x] >> rs)) ++y;
      lanes += (y - x + 63) & ~size_t(63);
      x = y;
    }
  }
  B.perm_b = B.pool->acquire(lanes * sizeof(uint32_t));
  B.perm = (uint32_t*)B.perm_b.p;
  B.perm_lanes = lanes;
  if (!pad) {
    memcpy(B.perm, idx.data(), n * sizeof(uint32_t));
    return;
  }
  size_t at = 0;
  for (size_t x = 0; x < n;) {
    size_t y = x + 1;
    while (y < n && (key[y] >> rs) == (key[x] >> rs)) ++y;
    memcpy(B.perm + at, idx.data() + x, (y - x) * sizeof(uint32_t));
    const size_t run = (y - x + 63) & ~size_t(63);
    for (size_t k = y - x; k < run; ++k) B.perm[at + k] = 0xFFFFFFFFu;
    at += run;
    x = y;
  }
}


using Items = std::vector<std::pair<const char*, const char*>>;

acs_codec_batch* encode_items(acs_codec* c, const std::pair<const char*, const char*>* items, size_t count,
                              int threads, double t0);

acs_codec_batch* encode_batch(acs_codec* c, const char* json, size_t len, int threads) {
  const double t0 = now_s();
  const int T = threads < 1 ? 1 : (threads > 64 ? 64 : threads);
  const Items items = split_items(json, json + len, T);
  return encode_items(c, items.data(), items.size(), T, t0);
}

// Encode the requests items[0..count) (delimited JSON values) into one batch.
acs_codec_batch* encode_items(acs_codec* c, const std::pair<const char*, const char*>* items, size_t count,
                              int threads, double t0) {
  auto B = std::make_unique<acs_codec_batch>();
  B->codec = c;
  B->pool = c->pool;
  int T = threads < 1 ? 1 : (threads > 64 ? 64 : threads);
  const uint32_t n = (uint32_t)count;
  if (count > 0xFFFFFFFull) throw ParseError{"requests: batch too large"};
  B->n = n;
  B->lines_b = c->pool->acquire((size_t)n * sizeof(ReqLine));
  B->lines = (ReqLine*)B->lines_b.p;
  B->reason.assign(n, nullptr);
  if ((uint32_t)T > n / 64 + 1) T = (int)(n / 64 + 1);
  B->strings.resize(T);
  for (int t = 0; t < T; ++t) B->strings[t].base = c->n_dict + ((uint32_t)t << LOCAL_BITS);
  Shared sh;
  std::vector<std::vector<uint32_t>> arenas(T), exts(T);
  std::vector<std::string> errs(T);
  std::atomic<uint64_t> hits{0}, misses{0};
  std::atomic<uint32_t> hints{0};
  auto range = [&](int t, uint32_t& lo, uint32_t& hi) {
    lo = (uint32_t)((uint64_t)n * t / T);
    hi = (uint32_t)((uint64_t)n * (t + 1) / T);
  };
  auto work = [&](int t) {
    uint32_t lo, hi;
    range(t, lo, hi);
    try {
      Encoder enc(*c, *B, sh, (uint32_t)t);
      for (uint32_t i = lo; i < hi; ++i) enc.encode(i, items[i].first, items[i].second);
      arenas[t] = std::move(enc.arena);
      exts[t] = std::move(enc.ext);
      hits += enc.hits;
      misses += enc.misses;
      hints |= enc.hints;
    } catch (const ParseError& e) {
      errs[t] = std::string("requests: ") + e.what;
    } catch (const std::exception& e) {
      errs[t] = e.what();
    }
  };
  acs_pool::run(T, work);
  for (auto& e : errs)
    if (!e.empty()) throw std::runtime_error(e);
  B->hr_hits = hits;
  B->hr_misses = misses;
  B->hints = hints;
  const double t1 = now_s();
  // regex-matrix columns in first-use order (request, attribute), as encoder.py numbers them
  std::vector<uint32_t> order(sh.cols.size()), remap(sh.cols.size());
  for (size_t k = 0; k < order.size(); ++k) order[k] = (uint32_t)k;
  std::sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return sh.cols[a].first < sh.cols[b].first; });
  for (size_t k = 0; k < order.size(); ++k) remap[order[k]] = (uint32_t)k;
  // regex matrix: one cached column of cells per distinct entity value
  const uint32_t n_rx = (uint32_t)c->rx_pat.size();
  B->rx_cols = order.empty() ? 1u : (uint32_t)order.size();
  B->rx_rows = n_rx ? n_rx : 1u;
  B->rx.assign((size_t)B->rx_cols * B->rx_rows, 0);
  std::vector<std::string> keys(B->rx_cols);
  for (size_t k = 0; k < order.size(); ++k) keys[k] = sh.cols[order[k]].key;
  {
    std::atomic<size_t> next{0};
    auto cells = [&] {
      for (;;) {
        const size_t k = next.fetch_add(1);
        if (k >= order.size()) return;
        std::shared_ptr<const std::vector<uint8_t>> col;
        {
          std::lock_guard<std::mutex> lock(c->col_mu);
          auto it = c->rx_cols.find(keys[k]);
          if (it != c->rx_cols.end()) col = it->second;
        }
        if (!col) {
          auto v = std::make_shared<std::vector<uint8_t>>(n_rx);
          const bool nul = keys[k][0] != 's';
          const std::string_view q = nul ? std::string_view() : std::string_view(keys[k]).substr(1);
          for (uint32_t r = 0; r < n_rx; ++r) (*v)[r] = rx_cell(c->rx_pat[r], nul, q);
          std::lock_guard<std::mutex> lock(c->col_mu);
          if (c->rx_cols.size() > 65536) c->rx_cols.clear();
          c->rx_cols.emplace(keys[k], v);
          col = v;
        }
        std::copy(col->begin(), col->end(), B->rx.begin() + k * B->rx_rows);
      }
    };
    acs_pool::run((int)std::min<size_t>((size_t)T, std::max<size_t>(order.size(), 1)), [&](int) { cells(); });
  }
  // RES_RX_SAFE on every entity attribute whose column holds no throwing / host cell (K1 may
  // then cut a combining loop short once its result is final: encoder.mark_rx_safe)
  std::vector<uint8_t> safe(B->rx_cols, 1);
  for (uint32_t k = 0; k < B->rx_cols; ++k)
    for (uint32_t r = 0; r < B->rx_rows; ++r)
      if (B->rx[(size_t)k * B->rx_rows + r] & (C_RX_THROW_TYPE | C_RX_THROW_SYNTAX | C_RX_HOST)) safe[k] = 0;
  // one arena and one extension-record array: each thread copies its part into place and
  // rebases its requests' offsets; column ids in first-use order; RES_RX_SAFE
  std::vector<size_t> abase(T + 1, 0), ebase(T + 1, 0);
  for (int t = 0; t < T; ++t) {
    abase[t + 1] = abase[t] + arenas[t].size();
    ebase[t + 1] = ebase[t] + exts[t].size();
  }
  if (abase[T] > 0xFFFFFFFFull || ebase[T] / 4 >= 0xFFFFFFFFull) throw std::runtime_error("batch arena too large");
  B->arena_b = c->pool->acquire(abase[T] * 4);
  B->arena = (uint32_t*)B->arena_b.p;
  B->arena_words = abase[T];
  B->ext_b = c->pool->acquire(ebase[T] * 4);
  B->ext = (uint32_t*)B->ext_b.p;
  B->ext_words = ebase[T];
  {
    auto fix = [&](int t) {
      if (!arenas[t].empty()) memcpy(B->arena + abase[t], arenas[t].data(), arenas[t].size() * 4);
      if (!exts[t].empty()) memcpy(B->ext + ebase[t], exts[t].data(), exts[t].size() * 4);
      uint32_t lo, hi;
      range(t, lo, hi);
      for (uint32_t i = lo; i < hi; ++i) {
        ReqLine& L = B->lines[i];
        L.h.arena_off += (uint32_t)abase[t];
        if (L.ext) L.ext += (uint32_t)(ebase[t] / 4);
        for (uint32_t j = 0; j < L.h.nres; ++j) {
          ReqRes* q = B->res_ptr(i, j);
          if (!(q->kind & K_ENT_LOOSE)) continue;
          q->col = (uint16_t)remap[q->col];
          if (q->col < B->rx_cols && safe[q->col]) q->pad |= RES_RX_SAFE;
        }
      }
    };
    acs_pool::run(T, fix);
  }
  const double t2 = now_s();
  Classes cl(*c, *B, T);
  cl.col_keys = keys;  // padding column: ''
  cl.run();
  coherence_order(*B, T);  // the kernels' order: the classes are known here (no device sort)
  const double t3 = now_s();
  B->seconds[0] = t1 - t0;
  B->seconds[1] = t2 - t1;
  B->seconds[2] = t3 - t2;
  B->seconds[3] = t3 - t0;
  return B.release();
}

// SoA rows of a compact batch (acs_codec_batch_expand): tests and the CPU build of the core.
void expand_soa(acs_codec_batch& B) {
  if (B.expanded) return;
  const uint32_t n = B.n;
  B.hdr.assign(n, ReqHdr{});
  B.res.assign((size_t)QMAX * n, ReqRes{});
  B.subj.assign((size_t)SMAX * n, Pair{});
  B.act.assign((size_t)AMAX * n, Pair{});
  B.roles.assign((size_t)RMAX * n, 0u);
  for (uint32_t i = 0; i < n; ++i) {
    const ReqLine& L = B.lines[i];
    const ReqHdr& h = L.h;
    B.hdr[i] = h;
    for (uint32_t j = 0; j < h.nres; ++j) B.res[(size_t)j * n + i] = B.res_at(i, j);
    const ExtGeom g = ext_geom(h.nres, h.nsubj, h.nact, h.nroles);
    const uint32_t* x = L.ext ? B.ext + (size_t)(L.ext - 1) * 4 : nullptr;
    for (uint32_t j = 0; j < h.nsubj; ++j)
      B.subj[(size_t)j * n + i] = j == 0 ? L.s0 : j == 1 ? L.s1 : Pair{x[g.subj + 2 * (j - 2)], x[g.subj + 2 * (j - 2) + 1]};
    for (uint32_t j = 0; j < h.nact; ++j)
      B.act[(size_t)j * n + i] = j == 0 ? L.a0 : Pair{x[g.act + 2 * (j - 1)], x[g.act + 2 * (j - 1) + 1]};
    for (uint32_t j = 0; j < h.nroles; ++j) B.roles[(size_t)j * n + i] = B.role_at(i, j);
  }
  B.expanded = true;
}

thread_local std::string g_codec_err;

}  // namespace

extern "C" {

acs_codec* acs_codec_create(const void* blob, size_t n_bytes) {
  auto c = std::make_unique<acs_codec>();
  std::string err;
  try {
    if (!codec_load(c.get(), blob, n_bytes, err)) {
      g_codec_err = "acs_codec_create: " + err;
      acs_internal_set_error(g_codec_err.c_str());
      return nullptr;
    }
  } catch (const std::exception& e) {
    g_codec_err = std::string("acs_codec_create: ") + e.what();
    acs_internal_set_error(g_codec_err.c_str());
    return nullptr;
  }
  return c.release();
}

void acs_codec_free(acs_codec* c) { delete c; }

int acs_codec_set_subject_scopes(acs_codec* c, const char* key, size_t key_len, const char* json, size_t len) {
  if (!c || !key || (!json && len)) {
    acs_internal_set_error("acs_codec_set_subject_scopes: null argument");
    return -1;
  }
  auto F = std::make_shared<HrForest>();
  try {
    Arena ar;
    Parser p(ar);
    const JV* v = p.parse(json, json + len);
    build_forest(*F, v);
  } catch (const ParseError& e) {
    g_codec_err = std::string("acs_codec_set_subject_scopes: ") + e.what;
    acs_internal_set_error(g_codec_err.c_str());
    return -1;
  }
  std::unique_lock<std::shared_mutex> lock(c->hr_mu);
  c->hr_subject[std::string(key, key_len)] = F;
  return 0;
}

#if defined(ACS_CODEC_TIMING)
int acs_internal_codec_cycles(uint64_t* parse, uint64_t* encode) {
  *parse = g_cyc_parse.exchange(0);
  *encode = g_cyc_encode.exchange(0);
  for (int k = 0; k < 7; ++k) encode[1 + k] = g_cyc_sect[k].exchange(0);
  for (int k = 0; k < 6; ++k) encode[8 + k] = g_cls_ns[k].exchange(0);
  return 0;
}
#endif

// Pipeline support (acs_kernels.hip acs_pipeline_*, not in include/acs_mi355x.h): delimit the
// request array once, then encode it chunk by chunk.
struct acs_internal_items {
  std::vector<std::pair<const char*, const char*>> v;
};
acs_internal_items* acs_internal_split(const char* json, size_t len, int threads, size_t* n) {
  try {
    auto it = std::make_unique<acs_internal_items>();
    it->v = split_items(json, json + len, threads < 1 ? 1 : (threads > 64 ? 64 : threads));
    *n = it->v.size();
    return it.release();
  } catch (const ParseError& e) {
    g_codec_err = std::string("acs_codec_encode: ") + e.what;
  } catch (const std::exception& e) {
    g_codec_err = std::string("acs_codec_encode: ") + e.what();
  }
  acs_internal_set_error(g_codec_err.c_str());
  return nullptr;
}
void acs_internal_items_free(acs_internal_items* it) { delete it; }
acs_codec_batch* acs_internal_encode_range(acs_codec* c, const acs_internal_items* it, size_t lo, size_t hi,
                                           int threads) {
  try {
    return encode_items(c, it->v.data() + lo, hi - lo, threads, now_s());
  } catch (const ParseError& e) {
    g_codec_err = std::string("acs_codec_encode: ") + e.what;
  } catch (const Unsup& u) {
    g_codec_err = std::string("acs_codec_encode: ") + u.why;
  } catch (const std::exception& e) {
    g_codec_err = std::string("acs_codec_encode: ") + e.what();
  }
  acs_internal_set_error(g_codec_err.c_str());
  return nullptr;
}

// Test hook (not in include/acs_mi355x.h): pin the candidate-class key level of every later
// encode (0 entity+roles+action, 1 composed, 2 entity+action, 3 entity; -1 automatic).
int acs_internal_codec_force_level(acs_codec* c, int level) {
  if (!c) return -1;
  c->force_level = level;
  return 0;
}

int acs_codec_evict_subject(acs_codec* c, const char* key, size_t key_len) {
  if (!c || !key) {
    acs_internal_set_error("acs_codec_evict_subject: null argument");
    return -1;
  }
  std::unique_lock<std::shared_mutex> lock(c->hr_mu);
  return c->hr_subject.erase(std::string(key, key_len)) ? 1 : 0;
}

acs_codec_batch* acs_codec_encode(acs_codec* c, const char* json, size_t len, int threads) {
  if (!c || (!json && len)) {
    acs_internal_set_error("acs_codec_encode: null argument");
    return nullptr;
  }
  try {
    return encode_batch(c, json, len, threads);
  } catch (const ParseError& e) {
    g_codec_err = std::string("acs_codec_encode: ") + e.what;
  } catch (const Unsup& u) {
    g_codec_err = std::string("acs_codec_encode: ") + u.why;
  } catch (const std::exception& e) {
    g_codec_err = std::string("acs_codec_encode: ") + e.what();
  }
  acs_internal_set_error(g_codec_err.c_str());
  return nullptr;
}

void acs_codec_batch_free(acs_codec_batch* b) { delete b; }

int acs_codec_batch_view(const acs_codec_batch* b, acs_req_batch* out) {
  if (!b || !out) {
    acs_internal_set_error("acs_codec_batch_view: null argument");
    return -1;
  }
  acs_req_batch v{};
  v.n = b->n;
  if (b->expanded) {
    v.hdr = b->hdr.data();
    v.res = b->res.data();
    v.subj = b->subj.data();
    v.act = b->act.data();
    v.roles = b->roles.data();
  }
  v.lines = b->n ? b->lines : nullptr;
  v.ext = b->ext_words ? b->ext : nullptr;
  v.ext_words = b->ext_words;
  v.arena = b->arena;
  v.arena_words = b->arena_words;
  v.rx = b->rx.data();
  v.rx_cols = b->rx_cols;
  v.rx_rows = b->rx_rows;
  v.cand = b->cand;
  v.cand_words = b->cand_words;
  v.cand_wp = b->cand_wp;
  v.cand_wr = b->cand_wr;
  v.cand_wsu = b->cand_wsu;
  v.cand_wpu = b->cand_wpu;
  v.cand_wv = b->cand_wv;
  v.cand_rows = b->cand_rows;
  if (!b->role_key.empty()) {
    v.role_key = b->role_key.data();
    v.role_rows_bits = b->role_bits.data();
    v.role_rows = b->role_rows;
  }
  v.perm = b->n ? b->perm : nullptr;
  v.perm_lanes = b->n ? b->perm_lanes : 0;
  v.hints = b->hints;
  *out = v;
  return 0;
}

int acs_codec_batch_expand(acs_codec_batch* b) {
  if (!b) {
    acs_internal_set_error("acs_codec_batch_expand: null argument");
    return -1;
  }
  try {
    expand_soa(*b);
  } catch (const std::exception& e) {
    g_codec_err = std::string("acs_codec_batch_expand: ") + e.what();
    acs_internal_set_error(g_codec_err.c_str());
    return -1;
  }
  return 0;
}

const char* acs_codec_batch_reason(const acs_codec_batch* b, uint32_t i) {
  return b && i < b->n ? b->reason[i] : nullptr;
}

int acs_codec_string(const acs_codec_batch* b, uint32_t id, const char** s, size_t* len) {
  if (!b || !s || !len) return -1;
  *s = nullptr;
  *len = 0;
  if (id == ID_UNDEF) return 0;
  if (id == ID_NULL) return 1;
  const acs_codec* c = b->codec;
  if (id < c->n_dict) {
    const std::string_view v = c->string_of(id);
    *s = v.data();
    *len = v.size();
    return 2;
  }
  const uint32_t t = (id - c->n_dict) >> LOCAL_BITS, k = (id - c->n_dict) & ((1u << LOCAL_BITS) - 1);
  if (t >= b->strings.size() || k >= b->strings[t].strs.size()) return -1;
  *s = b->strings[t].strs[k].data();
  *len = b->strings[t].strs[k].size();  // (views into the thread's StrPool, alive with the batch)
  return 2;
}

int acs_codec_ec_values(const acs_codec* c, const char** json, size_t* len) {
  if (!c || !json || !len) return -1;
  *json = c->ec_json.data();
  *len = c->ec_json.size();
  return 0;
}

int acs_codec_batch_stats(const acs_codec_batch* b, double* out, int n) {
  if (!b || !out) return -1;
  const double v[8] = {b->seconds[0], b->seconds[1], b->seconds[2], b->seconds[3], (double)b->hr_hits,
                       (double)b->hr_misses, (double)b->classes_new, (double)b->cand_rows};
  for (int k = 0; k < n && k < 8; ++k) out[k] = v[k];
  return 8;
}

}  // extern "C"
