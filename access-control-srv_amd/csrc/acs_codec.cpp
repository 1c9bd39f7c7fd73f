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
#include <atomic>
#include <cstring>
#include <memory>
#include <mutex>
#include <regex>
#include <shared_mutex>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "../../include/acs_mi355x.h"
#include "acs_json.h"
#include "acs_layout.h"

extern "C" void acs_internal_set_error(const char* msg);

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

constexpr uint32_t CODEC_MAGIC = 0x43534341u, CODEC_VERSION = 1u;
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
  std::unordered_map<std::string, uint64_t> masks;  // org id -> root bits | key bits << 32
  std::string text;           // inline forests: the exact JSON text they were built from
  size_t bytes() const { return text.size() + masks.size() * 48 + 256; }
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
          if (hid->t == J_STR) F.masks[std::string(hid->s, hid->n)] |= (1ull << r) | (1ull << (32 + val_key[vi]));
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
