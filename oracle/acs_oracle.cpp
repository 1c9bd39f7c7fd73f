// acs_oracle.cpp — CPU oracle for the access-control decision path, C++17.
// TEST INFRASTRUCTURE ONLY: only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg load it (through oracle/acs_oracle_c.py), as the checker and as the
// multi-core CPU baseline.  The product (access-control-srv_amd/) never links it.
//
// A scalar, un-interned restatement of the reference PDP of
// restorecommerce/access-control-srv (TypeScript) over JSON-shaped values with explicit
// JS semantics (undefined / null / '' kept apart, == vs ===, truthiness, lodash isEmpty /
// find, Map order).  It follows oracle/acs_oracle.py (the Python restatement pinned by
// the reference's own test vectors, tests/golden/kats.json) function for function; both
// cite the reference lines they restate:
//
//   AccessController.isAllowed            src/core/accessController.ts:88-324
//   checkMultipleEntitiesMatch            src/core/accessController.ts:429-463
//   resourceAttributesMatch               src/core/accessController.ts:465-654
//   targetMatches                         src/core/accessController.ts:661-672
//   attributesMatch                       src/core/accessController.ts:681-699
//   checkSubjectMatches                   src/core/accessController.ts:793-823
//   decide / denyOverrides /
//     permitOverrides / firstApplicable   src/core/accessController.ts:832-893
//   checkHierarchicalScope                src/core/hierarchicalScope.ts:10-259
//   verifyACLList                         src/core/verifyACL.ts:11-251
//   formatTarget                          src/core/utils.ts:35-45
//   populate (store loader of the tests)  test/utils.ts:345-383
//
// Scope: isAllowed and whatIsAllowed (rule sets + maskedProperty pushes,
// accessController.ts:326-427, :592-640).  Inputs the restatement cannot decide exactly
// report "unsupported"
// (rule `condition` — JS eval —, subject `token` I/O, RegExp patterns outside the
// restated subset, non-ASCII case mapping), exactly where oracle/acs_oracle.py raises
// OracleUnsupported.  tests/test_oracle_c.py checks it against the golden vectors and
// against the Python oracle on randomised stores and requests.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <map>
#include <memory>
#include <regex>
#include <set>
#include <stdexcept>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <unordered_set>
#include <utility>
#include <vector>

namespace {

// ------------------------------------------------------------------ JS values
enum class T : uint8_t { Undef, Null, Bool, Num, Str, Arr, Obj };

struct Val {
  T t = T::Undef;
  bool b = false;
  double n = 0;
  std::string s;
  std::vector<const Val*> a;
  std::vector<std::pair<std::string, const Val*>> o;
};
using VP = const Val*;

const Val kUndef{};
const Val kEmptyArr = [] { Val v; v.t = T::Arr; return v; }();
VP UNDEF = &kUndef;

struct JSError {
  int kind;  // 1 TypeError, 2 InvalidCombiningAlgorithm, 3 SyntaxError (csrc/acs_layout.h ErrKind)
};
struct Unsupported {
  const char* why;
};

[[noreturn]] void type_error() { throw JSError{1}; }
[[noreturn]] void unsupported(const char* why) { throw Unsupported{why}; }

// Values are owned by an arena (one per parsed document).
struct Arena {
  std::deque<Val> vals;
  Val* make(T t) {
    vals.emplace_back();
    vals.back().t = t;
    return &vals.back();
  }
};

// ------------------------------------------------------------------ JSON parser
struct Parser {
  const char* p;
  const char* e;
  Arena& ar;
  // Optional table of pre-parsed values: an object {"$shared": k} parses to shared[k]
  // itself (large sub-documents common to many requests — a synthetic batch's HR scope
  // trees — are parsed once; the oracle never mutates request values).
  const std::vector<VP>* shared = nullptr;
  Parser(const char* s, size_t n, Arena& a) : p(s), e(s + n), ar(a) {}
  void ws() {
    while (p < e && (*p == ' ' || *p == '\n' || *p == '\t' || *p == '\r')) ++p;
  }
  [[noreturn]] void bad() { throw std::runtime_error("bad JSON"); }
  static void utf8(std::string& out, uint32_t c) {
    if (c < 0x80) {
      out += (char)c;
    } else if (c < 0x800) {
      out += (char)(0xC0 | (c >> 6));
      out += (char)(0x80 | (c & 0x3F));
    } else if (c < 0x10000) {
      out += (char)(0xE0 | (c >> 12));
      out += (char)(0x80 | ((c >> 6) & 0x3F));
      out += (char)(0x80 | (c & 0x3F));
    } else {
      out += (char)(0xF0 | (c >> 18));
      out += (char)(0x80 | ((c >> 12) & 0x3F));
      out += (char)(0x80 | ((c >> 6) & 0x3F));
      out += (char)(0x80 | (c & 0x3F));
    }
  }
  uint32_t hex4() {
    if (e - p < 4) bad();
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      const char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else bad();
    }
    return v;
  }
  std::string str() {
    if (p >= e || *p != '"') bad();
    ++p;
    std::string out;
    while (p < e && *p != '"') {
      if (*p == '\\') {
        ++p;
        if (p >= e) bad();
        const char c = *p++;
        switch (c) {
          case '"': out += '"'; break;
          case '\\': out += '\\'; break;
          case '/': out += '/'; break;
          case 'b': out += '\b'; break;
          case 'f': out += '\f'; break;
          case 'n': out += '\n'; break;
          case 'r': out += '\r'; break;
          case 't': out += '\t'; break;
          case 'u': {
            uint32_t c1 = hex4();
            if (c1 >= 0xD800 && c1 < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
              p += 2;
              const uint32_t c2 = hex4();
              c1 = 0x10000 + ((c1 - 0xD800) << 10) + (c2 - 0xDC00);
            }
            utf8(out, c1);
            break;
          }
          default: bad();
        }
      } else {
        out += *p++;
      }
    }
    if (p >= e) bad();
    ++p;
    return out;
  }
  VP value() {
    ws();
    if (p >= e) bad();
    const char c = *p;
    if (c == '{') {
      ++p;
      Val* v = ar.make(T::Obj);
      ws();
      if (p < e && *p == '}') {
        ++p;
        return v;
      }
      for (;;) {
        ws();
        std::string k = str();
        ws();
        if (p >= e || *p != ':') bad();
        ++p;
        VP x = value();
        bool dup = false;
        for (auto& kv : v->o)
          if (kv.first == k) {
            kv.second = x;
            dup = true;
          }
        if (!dup) v->o.emplace_back(std::move(k), x);
        ws();
        if (p < e && *p == ',') {
          ++p;
          continue;
        }
        if (p < e && *p == '}') {
          ++p;
          if (shared && v->o.size() == 1 && v->o[0].first == "$shared" && v->o[0].second->t == T::Num) {
            const double k = v->o[0].second->n;
            if (k < 0 || k >= (double)shared->size()) bad();
            return (*shared)[(size_t)k];
          }
          return v;
        }
        bad();
      }
    }
    if (c == '[') {
      ++p;
      Val* v = ar.make(T::Arr);
      ws();
      if (p < e && *p == ']') {
        ++p;
        return v;
      }
      for (;;) {
        v->a.push_back(value());
        ws();
        if (p < e && *p == ',') {
          ++p;
          continue;
        }
        if (p < e && *p == ']') {
          ++p;
          return v;
        }
        bad();
      }
    }
    if (c == '"') {
      Val* v = ar.make(T::Str);
      v->s = str();
      return v;
    }
    if (e - p >= 4 && !strncmp(p, "true", 4)) {
      p += 4;
      Val* v = ar.make(T::Bool);
      v->b = true;
      return v;
    }
    if (e - p >= 5 && !strncmp(p, "false", 5)) {
      p += 5;
      return ar.make(T::Bool);
    }
    if (e - p >= 4 && !strncmp(p, "null", 4)) {
      p += 4;
      return ar.make(T::Null);
    }
    char* end = nullptr;
    const double d = strtod(p, &end);
    if (end == p) bad();
    p = end;
    Val* v = ar.make(T::Num);
    v->n = d;
    return v;
  }
};

// ------------------------------------------------------------------ JS semantics (jsval.py)
bool nullish(VP v) { return v->t == T::Undef || v->t == T::Null; }

bool truthy(VP v) {
  switch (v->t) {
    case T::Undef: case T::Null: return false;
    case T::Bool: return v->b;
    case T::Num: return !(v->n == 0 || std::isnan(v->n));
    case T::Str: return !v->s.empty();
    default: return true;
  }
}

bool is_obj(VP v) { return v->t == T::Arr || v->t == T::Obj; }

bool strict_eq(VP a, VP b) {  // ===
  if (a->t != b->t) return false;
  switch (a->t) {
    case T::Undef: case T::Null: return true;
    case T::Bool: return a->b == b->b;
    case T::Num: return a->n == b->n;
    case T::Str: return a->s == b->s;
    default: return a == b;
  }
}

double to_number(VP v) {
  if (v->t == T::Num) return v->n;
  if (v->t == T::Bool) return v->b ? 1.0 : 0.0;
  if (v->t == T::Str) {
    size_t a = 0, b = v->s.size();
    while (a < b && isspace((unsigned char)v->s[a])) ++a;
    while (b > a && isspace((unsigned char)v->s[b - 1])) --b;
    if (a == b) return 0.0;
    const std::string t = v->s.substr(a, b - a);
    char* end = nullptr;
    double d;
    if (t.size() > 2 && t[0] == '0' && (t[1] == 'x' || t[1] == 'X')) d = (double)strtoll(t.c_str() + 2, &end, 16);
    else d = strtod(t.c_str(), &end);
    if (!end || *end) return NAN;
    return d;
  }
  unsupported("ToNumber on object");
}

bool loose_eq(VP a, VP b) {  // == for the primitive cases the path meets
  if (nullish(a) || nullish(b)) return nullish(a) && nullish(b);
  if (is_obj(a) || is_obj(b)) {
    if (is_obj(a) && is_obj(b)) return a == b;
    unsupported("loose == between object and primitive");
  }
  if (a->t == b->t) return strict_eq(a, b);
  return to_number(a) == to_number(b);
}

bool same_value_zero(VP a, VP b) {
  if (a->t == T::Num && b->t == T::Num && std::isnan(a->n) && std::isnan(b->n)) return true;
  return strict_eq(a, b);
}

bool js_includes(const std::vector<VP>& arr, VP v) {
  for (VP x : arr)
    if (same_value_zero(x, v)) return true;
  return false;
}

VP get(VP obj, const char* key) {  // obj?.key (no "length": see length_of)
  if (obj->t != T::Obj) return UNDEF;
  for (auto& kv : obj->o)
    if (kv.first == key) return kv.second;
  return UNDEF;
}

bool has_key(VP obj, const char* key) {
  if (obj->t != T::Obj) return false;
  for (auto& kv : obj->o)
    if (kv.first == key) return true;
  return false;
}

VP prop(VP obj, const char* key) {  // obj.key
  if (nullish(obj)) type_error();
  return get(obj, key);
}

// x?.length as a number (-1: undefined)
long length_of(VP v) {
  if (v->t == T::Arr) return (long)v->a.size();
  if (v->t == T::Str) return (long)v->s.size();  // UTF-8 bytes: only compared with 0
  return -1;
}

bool length_gt0(VP v) { return length_of(v) > 0; }

const std::vector<VP>& iterate(VP v) {  // for (const x of v)
  if (v->t == T::Arr) return v->a;
  if (v->t == T::Str) unsupported("iterating a string");
  type_error();
}

const std::vector<VP>& or_empty(VP v) {  // (v || []) iterated
  if (!truthy(v)) return kEmptyArr.a;
  return iterate(v);
}

bool lodash_is_empty(VP v) {
  if (nullish(v)) return true;
  if (v->t == T::Arr) return v->a.empty();
  if (v->t == T::Str) return v->s.empty();
  if (v->t == T::Obj) return v->o.empty();
  return true;
}

VP get_path(VP obj, const char* path) {  // lodash get along a dotted path
  VP cur = obj;
  std::string k;
  for (const char* c = path;; ++c) {
    if (*c == '.' || *c == 0) {
      if (nullish(cur)) return UNDEF;
      cur = get(cur, k.c_str());
      k.clear();
      if (!*c) break;
    } else {
      k += *c;
    }
  }
  return cur;
}

bool has_in_path(VP obj, const char* path) {
  VP cur = obj;
  std::string k;
  for (const char* c = path;; ++c) {
    if (*c == '.' || *c == 0) {
      if (nullish(cur) || cur->t != T::Obj || !has_key(cur, k.c_str())) return false;
      cur = get(cur, k.c_str());
      k.clear();
      if (!*c) break;
    } else {
      k += *c;
    }
  }
  return true;
}

bool base_is_equal(VP a, VP b) {
  if (a->t == T::Num && b->t == T::Num && std::isnan(a->n) && std::isnan(b->n)) return true;
  if (a->t == T::Obj && b->t == T::Obj) {
    if (a->o.size() != b->o.size()) return false;
    for (auto& kv : a->o) {
      if (!has_key(b, kv.first.c_str())) return false;
      if (!base_is_equal(kv.second, get(b, kv.first.c_str()))) return false;
    }
    return true;
  }
  if (a->t == T::Arr && b->t == T::Arr) {
    if (a->a.size() != b->a.size()) return false;
    for (size_t i = 0; i < a->a.size(); ++i)
      if (!base_is_equal(a->a[i], b->a[i])) return false;
    return true;
  }
  return strict_eq(a, b);
}

VP lodash_find(VP coll, const char* path, VP src) {  // _.find(coll, [path, src])
  std::vector<VP> items;
  if (coll->t == T::Arr) items = coll->a;
  else if (coll->t == T::Obj)
    for (auto& kv : coll->o) items.push_back(kv.second);
  for (VP obj : items) {
    VP ov = get_path(obj, path);
    if (ov->t == T::Undef && src->t == T::Undef) {
      if (has_in_path(obj, path)) return obj;
      continue;
    }
    if (base_is_equal(src, ov)) return obj;
  }
  return UNDEF;
}

// ---- String.prototype helpers (ASCII case mapping only)
std::string upper(const std::string& s) {
  std::string o = s;
  for (char& c : o) {
    if ((unsigned char)c >= 0x80) unsupported("non-ASCII toUpperCase");
    c = (char)toupper((unsigned char)c);
  }
  return o;
}

std::string substring(const std::string& s, long a, long b) {
  const long n = (long)s.size();
  a = std::min(std::max(a, 0L), n);
  b = std::min(std::max(b, 0L), n);
  if (a > b) std::swap(a, b);
  return s.substr(a, b - a);
}

long last_index_of(const std::string& s, char c) {
  const size_t k = s.rfind(c);
  return k == std::string::npos ? -1 : (long)k;
}

std::vector<std::string> split(const std::string& s, char c) {
  std::vector<std::string> out;
  size_t a = 0;
  for (;;) {
    const size_t k = s.find(c, a);
    if (k == std::string::npos) {
      out.push_back(s.substr(a));
      return out;
    }
    out.push_back(s.substr(a, k - a));
    a = k + 1;
  }
}

const std::string& str_of(VP v) {  // receiver of a string method (?. already handled)
  if (v->t != T::Str) unsupported("string method on non-string");
  return v->s;
}

bool all_in(const std::string& s, const char* allowed_extra, bool alnum) {
  for (char c : s) {
    const unsigned char u = (unsigned char)c;
    if (alnum && (isalnum(u) || c == '_' || c == '-')) continue;
    if (strchr(allowed_extra, c) && c) continue;
    return false;
  }
  return true;
}

// subject.match(new RegExp(pattern)) != null for the restated subset (jsval.js_regex_search)
bool js_regex_search(const std::string& pattern, const std::string& subject) {
  if (all_in(pattern, " \t\n\r\f\v#@%&=,;'\"<>~`!", true)) return subject.find(pattern) != std::string::npos;
  if (!all_in(pattern, "*+?|()[]^$", true) || pattern.find("(?") != std::string::npos ||
      pattern.find("[]") != std::string::npos || pattern.find("[^]") != std::string::npos)
    unsupported("regex pattern outside the restated subset");
  // V8 rejects a quantifier that follows a quantifier ("Nothing to repeat": a**, a*+, a???);
  // libstdc++'s ECMAScript grammar accepts them, so the check is explicit (pinned by
  // tests/golden/regex_cells.json).  A '?' right after a quantifier is its lazy marker.
  {
    bool in_class = false;
    int quant = 0;  // 0: previous token not a quantifier, 1: a quantifier, 2: quantifier + lazy '?'
    for (char c : pattern) {
      if (in_class) {
        in_class = c != ']';
        continue;
      }
      if (c == '*' || c == '+' || c == '?') {
        if (quant == 1 && c == '?') quant = 2;
        else if (quant) throw JSError{3};
        else quant = 1;
        continue;
      }
      quant = 0;
      if (c == '[') in_class = true;
    }
  }
  try {
    std::regex rx(pattern, std::regex::ECMAScript);
    return std::regex_search(subject, rx);
  } catch (const std::regex_error&) {
    throw JSError{3};
  }
}

// ------------------------------------------------------------------ Map keys (SameValueZero)
std::string map_key(VP v) {
  switch (v->t) {
    case T::Undef: return "u";
    case T::Null: return "n";
    case T::Bool: return v->b ? "bt" : "bf";
    case T::Num: {
      char buf[64];
      snprintf(buf, sizeof buf, "d%.17g", v->n == 0 ? 0.0 : v->n);
      return buf;
    }
    case T::Str: return "s" + v->s;
    default: {
      char buf[32];
      snprintf(buf, sizeof buf, "o%p", (const void*)v);
      return buf;
    }
  }
}

template <class X>
struct OrderedMap {  // JS Map: insertion order, re-set keeps the position
  std::vector<std::pair<std::string, X>> items;
  std::unordered_map<std::string, size_t> index;
  X& set(const std::string& k, X x) {
    auto it = index.find(k);
    if (it != index.end()) {
      items[it->second].second = std::move(x);
      return items[it->second].second;
    }
    index.emplace(k, items.size());
    items.emplace_back(k, std::move(x));
    return items.back().second;
  }
  size_t size() const { return items.size(); }
};

// ------------------------------------------------------------------ store (test/utils.ts populate)
struct Target {
  bool present = false;  // formatTarget(null) -> null
  VP subjects = &kEmptyArr, resources = &kEmptyArr, actions = &kEmptyArr;
  // checkSubjectMatches' rule side (accessController.ts:797-806), a pure function of the
  // immutable store: subjects empty, and ruleRole (the last role-URN subject value); set by
  // Oracle::load once the URN config is known
  bool subj_empty = true;
  VP rule_role = nullptr;
};

Target format_target(VP t) {  // utils.ts:35-45
  Target f;
  if (!truthy(t)) return f;
  f.present = true;
  VP s = get(t, "subjects"), r = get(t, "resources"), a = get(t, "actions");
  if (truthy(s)) f.subjects = s;
  if (truthy(r)) f.resources = r;
  if (truthy(a)) f.actions = a;
  return f;
}

struct Rule {
  VP raw;
  Target target;
};
struct Policy {
  VP raw;
  Target target;
  OrderedMap<Rule> rules;
  bool null = false;  // a null Map entry (resourceManager re-reads, accessController.ts:138): {"id", "$null": true}
};
struct PolicySet {
  VP raw;
  Target target;
  OrderedMap<Policy> policies;
};

// ------------------------------------------------------------------ the oracle
struct Outcome {
  int32_t kind = 0;      // 0 OK, 1 the reference rejects (err = JS error kind), 2 unsupported
  int32_t decision = 0;  // DecisionCode (2 PERMIT .. 6 UNRECOGNIZED)
  int32_t ec = 0;        // 0 undefined, 1 null, 2 false, 3 true, 4 other value
  int32_t code = 0;      // status code (200 / 400) or the error kind
};

struct Effect {
  VP effect = UNDEF;
  VP ec = UNDEF;
};

enum UrnName {U_roleScopingEntity, U_roleScopingInstance, U_hierarchicalRoleScoping, U_ownerEntity, U_ownerInstance, U_resourceID, U_entity, U_role, U_operation, U_aclIndicatoryEntity, U_aclInstance, U_actionID, U_create, U_modify, U_read, U_delete, U_user, U_skipACL, U_property, U_maskedProperty, U_COUNT};
const char* const kUrnNames[U_COUNT] = {"roleScopingEntity", "roleScopingInstance", "hierarchicalRoleScoping", "ownerEntity", "ownerInstance", "resourceID", "entity", "role", "operation", "aclIndicatoryEntity", "aclInstance", "actionID", "create", "modify", "read", "delete", "user", "skipACL", "property", "maskedProperty"};

enum Method { M_DENY, M_PERMIT, M_FIRST };

struct Oracle {
  Arena arena;
  std::map<std::string, std::string> urns;
  std::unordered_map<std::string, Method> cas;
  OrderedMap<PolicySet> sets;
  // URN values as JS values (UNDEF when the config lacks them), indexed by UrnName: an
  // array read per lookup (the matchers run it per rule and request attribute)
  VP U[U_COUNT];
  VP S_PERMIT, S_DENY, S_TRUE;

  VP str_val(const std::string& s) {
    Val* v = arena.make(T::Str);
    v->s = s;
    return v;
  }

  VP u(UrnName k) const { return U[k]; }
  VP S_EMPTY = nullptr;  // ''


  void init_urns(VP cfg) {
    for (int k = 0; k < U_COUNT; ++k) U[k] = get(cfg, kUrnNames[k]);
    S_PERMIT = str_val("PERMIT");
    S_DENY = str_val("DENY");
    S_TRUE = str_val("true");
    S_EMPTY = str_val("");
  }

  void init_cas(VP list) {  // accessController.ts:51-62
    for (VP ca : iterate(list)) {
      VP m = get(ca, "method");
      if (m->t != T::Str) throw std::runtime_error("bad combining algorithm method");
      Method k;
      if (m->s == "denyOverrides") k = M_DENY;
      else if (m->s == "permitOverrides") k = M_PERMIT;
      else if (m->s == "firstApplicable") k = M_FIRST;
      else throw std::runtime_error("bad combining algorithm method");
      cas[map_key(get(ca, "urn"))] = k;
    }
  }

  void load(VP doc) {  // test/utils.ts:345-383
    for (VP ps : iterate(prop(doc, "policy_sets"))) {
      PolicySet s;
      s.raw = ps;
      s.target = format_target(get(ps, "target"));
      prepare_target(s.target);
      for (VP py : iterate(prop(ps, "policies"))) {
        Policy p;
        p.raw = py;
        if (truthy(get(py, "$null"))) {  // the fixture form of a null entry under this id
          p.null = true;
          s.policies.set(map_key(get(py, "id")), std::move(p));
          continue;
        }
        p.target = format_target(get(py, "target"));
        prepare_target(p.target);
        VP rules = get(py, "rules");
        for (VP ry : or_empty(rules)) {
          Rule r;
          r.raw = ry;
          r.target = format_target(get(ry, "target"));
          prepare_target(r.target);
          p.rules.set(map_key(get(ry, "id")), r);
        }
        s.policies.set(map_key(get(py, "id")), std::move(p));
      }
      sets.set(map_key(get(ps, "id")), std::move(s));
    }
  }

  // ---------------------------------------------------------------- combining (:832-893)
  Effect decide(VP ca, const std::vector<Effect>& effects) const {
    auto it = cas.find(map_key(ca));
    if (it == cas.end()) throw JSError{2};
    if (it->second == M_FIRST) return effects[0];
    VP want = it->second == M_DENY ? S_DENY : S_PERMIT;
    Effect chosen;
    for (const Effect& e : effects) {
      chosen = e;
      if (strict_eq(e.effect, want)) break;
    }
    return chosen;
  }

  // ---------------------------------------------------------------- matchers
  bool attributes_match(VP rule_attrs, VP req_attrs) const {  // :681-699 (loose ==)
    for (VP a : or_empty(rule_attrs)) {
      VP aid = get(a, "id"), av = get(a, "value");
      bool found = false;
      if (!nullish(req_attrs))
        for (VP ra : iterate(req_attrs))
          if (loose_eq(get(ra, "id"), aid) && loose_eq(get(ra, "value"), av)) {
            found = true;
            break;
          }
      if (!found) return false;
    }
    return true;
  }

  bool subject_matches(VP rule_subs, VP req_subs, VP request) const {  // :793-823
    VP ctx = get(request, "context");
    VP role_urn = u(U_role);
    if (nullish(rule_subs) || length_of(rule_subs) == 0) return true;
    VP rule_role = UNDEF;
    for (VP s : iterate(rule_subs))
      if (strict_eq(get(s, "id"), role_urn)) rule_role = get(s, "value");
    if (!truthy(rule_role)) return attributes_match(rule_subs, req_subs);
    VP ras = get(get(ctx, "subject"), "role_associations");
    if (!truthy(ras)) return false;
    for (VP r : iterate(ras))
      if (strict_eq(get(r, "role"), rule_role)) return true;
    return false;
  }

  // The request side of checkSubjectMatches, per request (the request is not mutated on the
  // supported paths): whether context.subject.role_associations is truthy and the string
  // `role` values it holds (any non-string role: the general path above).
  struct RoleSet {
    VP request = nullptr;
    bool truthy_ras = false, strings_only = true;
    std::unordered_set<std::string_view> roles;
  };
  static RoleSet& role_set_slot() {
    thread_local RoleSet rs;
    return rs;
  }
  // called at the start of every request evaluation (a later request may reuse an address)
  static void role_set_reset() { role_set_slot().request = nullptr; }
  static RoleSet& role_set(VP request) {
    RoleSet& rs = role_set_slot();
    if (rs.request == request) return rs;
    rs.request = request;
    rs.roles.clear();
    rs.strings_only = true;
    VP ras = get(get(get(request, "context"), "subject"), "role_associations");
    rs.truthy_ras = truthy(ras);
    if (rs.truthy_ras) {
      if (ras->t != T::Arr) {
        rs.strings_only = false;
      } else {
        for (VP r : ras->a) {
          VP role = get(r, "role");
          if (role->t == T::Str) rs.roles.insert(std::string_view(role->s));
          else if (role->t != T::Undef && role->t != T::Null) rs.strings_only = false;
        }
      }
    }
    return rs;
  }

  // checkSubjectMatches with the rule side precomputed (Target::rule_role): the same result
  // as subject_matches(t.subjects, ...), one hash probe for a role-scoped target
  bool target_subject_matches(const Target& t, VP req_subs, VP request) const {
    if (t.subj_empty) return true;
    if (!t.rule_role || !truthy(t.rule_role)) return subject_matches(t.subjects, req_subs, request);
    const RoleSet& rs = role_set(request);
    if (!rs.truthy_ras) return false;
    if (!rs.strings_only || t.rule_role->t != T::Str) return subject_matches(t.subjects, req_subs, request);
    return rs.roles.count(std::string_view(t.rule_role->s)) > 0;
  }

  void prepare_target(Target& t) const {  // the rule side of :797-806
    t.subj_empty = nullish(t.subjects) || length_of(t.subjects) == 0;
    if (t.subj_empty) return;
    VP rule_role = UNDEF;
    for (VP s : iterate(t.subjects))
      if (strict_eq(get(s, "id"), u(U_role))) rule_role = get(s, "value");
    t.rule_role = rule_role;
  }

  // namespace / RegExp entity test (:528-566, hierarchicalScope.ts:64-101) -> (reset, hit).
  // A pure function of the two strings: memoised per thread by their contents (a 1M-rule
  // store asks for the same (rule value, request value) pairs again and again).
  std::pair<bool, bool> regex_entity(VP rule_value, VP req_value) const {
    if (rule_value->t != T::Str || req_value->t != T::Str) return regex_entity_eval(rule_value, req_value);
    thread_local std::unordered_map<std::string, int> memo;  // 0..3: reset<<1 | hit; 4: unsupported
    std::string key;
    key.reserve(rule_value->s.size() + req_value->s.size() + 1);
    key += rule_value->s;
    key += '\0';
    key += req_value->s;
    auto it = memo.find(key);
    if (it == memo.end()) {
      int code;
      try {
        const auto rh = regex_entity_eval(rule_value, req_value);
        code = (rh.first ? 2 : 0) | (rh.second ? 1 : 0);
      } catch (const Unsupported&) {
        code = 4;
      }
      if (memo.size() > (1u << 20)) memo.clear();
      it = memo.emplace(std::move(key), code).first;
    }
    if (it->second == 4) unsupported("RegExp pattern outside the restated subset");
    return {(it->second & 2) != 0, (it->second & 1) != 0};
  }

  std::pair<bool, bool> regex_entity_eval(VP rule_value, VP req_value) const {
    if (nullish(rule_value)) type_error();  // nsEntityArray[0] of undefined
    const std::string& rv = str_of(rule_value);
    const std::string pattern = rv.substr(last_index_of(rv, ':') + 1);
    const std::vector<std::string> ns_arr = split(pattern, '.');
    const std::string& ns_or_entity = ns_arr[0];
    const std::string& entity_rx = ns_arr.back();
    std::string rule_ns;
    bool has_rule_ns = false;
    if (upper(ns_or_entity) != upper(entity_rx)) {
      rule_ns = upper(ns_or_entity);
      has_rule_ns = !rule_ns.empty();
    }
    const std::string rule_prefix = substring(rv, 0, last_index_of(rv, ':'));
    if (nullish(req_value)) type_error();  // reqNSEntityArray[0] of undefined
    const std::string& qv = str_of(req_value);
    const std::string req_prefix = substring(qv, 0, last_index_of(qv, ':'));
    const bool reset = req_prefix != rule_prefix;
    const std::string req_pattern = qv.substr(last_index_of(qv, ':') + 1);
    const std::vector<std::string> req_arr = split(req_pattern, '.');
    std::string req_ns;
    bool has_req_ns = false;
    if (upper(req_arr[0]) != upper(req_arr.back())) {
      req_ns = upper(req_arr[0]);
      has_req_ns = !req_ns.empty();
    }
    bool hit = false;
    if ((has_req_ns && has_rule_ns && req_ns == rule_ns) || (!has_req_ns && !has_rule_ns))
      hit = js_regex_search(entity_rx, req_arr.back());
    return {reset, hit};
  }

  // whatIsAllowed's maskedProperty pushes, in evaluation order: (requestEntityURN, maskProperty)
  // per push (:599-613, 624-638); the obligations list groups them by entity value.
  using Pushes = std::vector<std::pair<VP, VP>>;

  // :597-614 / :622-639: returns true where the reference `continue`s (no push)
  bool push_mask(Pushes* masks, VP qa, bool req_props, VP req_entity_urn, VP rule_prop_value) const {
    VP qval = get(qa, "value");
    VP mask = UNDEF;
    if (req_props && truthy(qval)) mask = qval;
    else if (!req_props) mask = rule_prop_value;
    if (!nullish(mask) && str_of(mask).find('#') == std::string::npos) return true;  // indexOf('#') <= -1
    masks->push_back({req_entity_urn ? req_entity_urn : S_EMPTY, mask});
    return false;
  }

  bool resource_attrs_match(VP rule_attrs, const std::vector<VP>& req_list, VP effect, bool regex,
                            Pushes* masks = nullptr) const {
    // :465-654; masks != nullptr: operation 'whatIsAllowed' (pushes into *masks)
    const bool wia = masks != nullptr;
    VP ent = u(U_entity), prop_urn = u(U_property), op_urn = u(U_operation);
    bool entity_match = false, property_match = false, rule_props = false, req_props = false;
    bool operation_match = false, skip_deny = true;
    VP req_entity_urn = nullptr;  // '' initially
    VP rule_prop_value = S_EMPTY;  // rulePropertyValue = ''
    if (lodash_is_empty(rule_attrs)) return true;
    for (VP ra : req_list)
      if (strict_eq(prop(ra, "id"), prop_urn)) req_props = true;
    const bool eff_permit = strict_eq(effect, S_PERMIT), eff_deny = strict_eq(effect, S_DENY);
    for (VP qa : req_list) {
      property_match = false;
      for (VP r : or_empty(rule_attrs)) {
        VP rid = get(r, "id"), rval = get(r, "value");
        VP qid = get(qa, "id"), qval = get(qa, "value");
        if (strict_eq(prop(r, "id"), prop_urn)) {
          rule_props = true;
          rule_prop_value = prop(r, "value");
        }
        if (!regex) {
          if (strict_eq(qid, ent) && strict_eq(rid, ent) && strict_eq(qval, rval)) {
            entity_match = true;
            req_entity_urn = prop(qa, "value");
          } else if (strict_eq(qid, op_urn) && strict_eq(rid, op_urn) && strict_eq(qval, rval)) {
            operation_match = true;
          } else if (entity_match && strict_eq(qid, prop_urn) && strict_eq(rid, prop_urn)) {
            // entityName = requestEntityURN?.substring(lastIndexOf(':') + 1); qval?.indexOf(entityName)
            std::string entity_name = "undefined";
            if (req_entity_urn && !nullish(req_entity_urn)) {
              const std::string& s = str_of(req_entity_urn);
              entity_name = s.substr(last_index_of(s, ':') + 1);
            } else if (req_entity_urn == nullptr) {
              entity_name = "";  // ''.substring(...) of the initial ''
            }
            bool idx_ok = false, idx_undef = nullish(qval);
            if (!idx_undef) idx_ok = str_of(qval).find(entity_name) != std::string::npos;
            if (!idx_undef && idx_ok) {
              if (strict_eq(rval, qval)) property_match = true;
            } else if (eff_permit) {
              property_match = true;
            }
          }
        } else {
          if (strict_eq(qid, ent) && strict_eq(rid, ent)) {
            const auto rh = regex_entity(rval, qval);
            req_entity_urn = qval;
            if (rh.first) entity_match = false;
            if (rh.second) entity_match = true;
          } else if (entity_match && strict_eq(qid, prop_urn) && strict_eq(rid, prop_urn)) {
            bool rps_undef = nullish(rval), qps_undef = nullish(qval);
            std::string rps, qps;
            if (!rps_undef) rps = str_of(rval).substr(last_index_of(str_of(rval), '#') + 1);
            if (!qps_undef) qps = str_of(qval).substr(last_index_of(str_of(qval), '#') + 1);
            if (rps_undef == qps_undef && (rps_undef || rps == qps)) property_match = true;
          }
        }
      }
      VP qid = get(qa, "id");
      const bool scope = strict_eq(qid, prop_urn) || !req_props;
      if (!wia) {
        if (eff_deny && scope && entity_match && rule_props && property_match) skip_deny = false;
        if (eff_permit && scope && entity_match && rule_props && !property_match) return false;
        continue;
      }
      if (eff_permit && scope && entity_match && rule_props && !property_match) {  // :592-614
        if (!req_props) return false;
        if (push_mask(masks, qa, req_props, req_entity_urn, rule_prop_value)) continue;
      }
      if (eff_deny && scope && entity_match && rule_props && (property_match || !req_props)) {  // :619-639
        if (push_mask(masks, qa, req_props, req_entity_urn, rule_prop_value)) continue;
      }
    }
    if (!wia && skip_deny && rule_props && req_props && eff_deny && !property_match) return false;
    if (!entity_match && !operation_match) return false;
    return true;
  }

  bool target_matches(const Target& t, VP request, VP effect, bool regex, Pushes* masks = nullptr) const {
    // :661-672 (masks: operation 'whatIsAllowed')
    if (effect->t == T::Undef) effect = S_PERMIT;
    VP req_target = prop(request, "target");
    if (!target_subject_matches(t, prop(req_target, "subjects"), request)) return false;
    if (!attributes_match(t.actions, prop(req_target, "actions"))) return false;
    VP res = prop(req_target, "resources");
    return resource_attrs_match(t.resources, or_empty(res), effect, regex, masks);
  }

  bool multiple_entities_match(const PolicySet& ps, VP request) const {  // :429-463
    VP ent = u(U_entity);
    for (VP qa : or_empty(get(get(request, "target"), "resources"))) {
      if (!strict_eq(prop(qa, "id"), ent)) continue;
      bool multi = false;
      for (auto& kv : ps.policies.items) {
        const Policy& pol = kv.second;
        if (pol.null) throw JSError{1};  // policy.effect of null (:439)
        VP pe = UNDEF;
        if (truthy(prop(pol.raw, "effect"))) pe = get(pol.raw, "effect");
        if (pol.target.present && length_gt0(pol.target.resources)) {
          const std::vector<VP> one{qa};
          if (resource_attrs_match(pol.target.resources, one, pe, false)) multi = true;
        }
      }
      if (!multi) return false;
    }
    return true;
  }

  // ---------------------------------------------------------------- HR scope
  // The flattened HR ids of one (hierarchical_scopes, rule role): views into the request's
  // own strings, plus the id sets of children arrays taken from the call's shared-value
  // table (computed once per thread for every request that names them; a pure function of
  // immutable input, so memoising it changes no result).
  using IdSet = std::unordered_set<std::string_view>;
  struct Flat {
    IdSet own;
    std::vector<const IdSet*> shared;
    bool count(std::string_view v) const {
      if (own.count(v)) return true;
      for (const IdSet* s : shared)
        if (s->count(v)) return true;
      return false;
    }
  };
  struct SharedIds {  // per worker thread, for one acs_oracle_is_allowed_shared call
    const std::unordered_set<VP>* shared_values = nullptr;
    std::unordered_map<VP, IdSet> ids;
  };
  struct Memo {
    std::map<std::pair<VP, std::string>, Flat> flat;
    SharedIds* cache = nullptr;
  };

  static void collect_ids(VP h, IdSet& out, std::vector<VP>& stack) {
    stack.push_back(h);
    while (!stack.empty()) {
      VP x = stack.back();
      stack.pop_back();
      VP hid = get(x, "id");
      if (truthy(hid)) {
        if (is_obj(hid)) unsupported("object-valued HR id");
        if (hid->t == T::Str) out.insert(std::string_view(hid->s));
      }
      VP ch = get(x, "children");
      if (length_gt0(ch)) {
        const std::vector<VP>& kids = iterate(ch);
        for (auto k = kids.rbegin(); k != kids.rend(); ++k) stack.push_back(*k);
      }
    }
  }

  const Flat& flat_hr(VP scopes, VP rule_role, Memo& memo) const {  // hierarchicalScope.ts:207-220
    if (nullish(scopes)) type_error();
    const auto key = std::make_pair(scopes, map_key(rule_role));
    auto it = memo.flat.find(key);
    if (it != memo.flat.end()) return it->second;
    Flat out;
    std::vector<VP> stack;
    for (VP r : iterate(scopes)) {
      if (!strict_eq(get(r, "role"), rule_role)) continue;
      VP ch = get(r, "children");
      if (memo.cache && memo.cache->shared_values && memo.cache->shared_values->count(ch) && length_gt0(ch)) {
        VP hid = get(r, "id");
        if (truthy(hid)) {
          if (is_obj(hid)) unsupported("object-valued HR id");
          if (hid->t == T::Str) out.own.insert(std::string_view(hid->s));
        }
        auto c = memo.cache->ids.find(ch);
        if (c == memo.cache->ids.end()) {
          IdSet ids;
          for (VP k : iterate(ch)) collect_ids(k, ids, stack);
          c = memo.cache->ids.emplace(ch, std::move(ids)).first;
        }
        out.shared.push_back(&c->second);
      } else {
        collect_ids(r, out.own, stack);
      }
    }
    return memo.flat.emplace(key, std::move(out)).first->second;
  }

  bool check_hierarchical_scope(const Target& t, VP request, Memo& memo) const {  // hierarchicalScope.ts:10-259
    OrderedMap<VP> owners_map;
    VP subs = t.subjects;
    if (length_of(subs) == 0) return true;
    VP hr_check = S_TRUE;
    VP rule_role = UNDEF, scoping_entity = UNDEF;
    VP role_urn = u(U_role);
    for (VP s : or_empty(subs)) {
      VP sid = get(s, "id");
      if (strict_eq(sid, role_urn)) rule_role = get(s, "value");
      else if (strict_eq(sid, u(U_hierarchicalRoleScoping))) hr_check = prop(s, "value");
      else if (strict_eq(sid, u(U_roleScopingEntity))) scoping_entity = prop(s, "value");
    }
    if (!truthy(scoping_entity)) return true;
    VP ctx = get(request, "context");
    if (lodash_is_empty(ctx)) return false;
    VP ctx_resources_v = get(ctx, "resources");
    VP ctx_resources = truthy(ctx_resources_v) ? ctx_resources_v : &kEmptyArr;
    VP req_target = get(request, "target");
    for (VP attr : or_empty(t.resources)) {
      if (loose_eq(get(attr, "id"), u(U_entity))) {
        VP eoo = get(attr, "value");
        bool entities_match = false;
        for (VP qa : or_empty(prop(req_target, "resources"))) {
          if (loose_eq(get(qa, "id"), get(attr, "id")) && loose_eq(get(qa, "value"), eoo)) {
            entities_match = true;
          } else if (loose_eq(get(qa, "id"), get(attr, "id"))) {
            const auto rh = regex_entity(eoo, get(qa, "value"));
            if (rh.first) entities_match = false;
            if (rh.second) entities_match = true;
          } else if (loose_eq(get(qa, "id"), u(U_resourceID)) && entities_match) {
            VP inst_id = get(qa, "value");
            VP res = lodash_find(ctx_resources, "instance.id", inst_id);
            if (truthy(res)) res = get(res, "instance");
            else res = lodash_find(ctx_resources, "id", inst_id);
            if (truthy(res)) {
              VP meta = get(res, "meta");
              if (lodash_is_empty(meta) || lodash_is_empty(get(meta, "owners"))) return false;
              owners_map.set(map_key(inst_id), get(meta, "owners"));
            } else {
              return false;
            }
          }
        }
      } else if (strict_eq(get(attr, "id"), u(U_operation))) {
        VP eoo = get(attr, "value");
        for (VP qa : or_empty(prop(req_target, "resources"))) {
          if (strict_eq(get(qa, "id"), get(attr, "id")) && strict_eq(get(qa, "value"), get(attr, "value"))) {
            VP res = lodash_find(ctx_resources, "id", eoo);
            if (truthy(res)) {
              VP meta = get(res, "meta");
              if (lodash_is_empty(meta) || lodash_is_empty(get(meta, "owners"))) return false;
              owners_map.set(map_key(eoo), get(meta, "owners"));
            } else {
              return false;
            }
          }
        }
      }
    }
    VP ras = get(get(ctx, "subject"), "role_associations");
    if (lodash_is_empty(ras)) return false;
    std::vector<VP> reduced;
    for (VP r : iterate(ras))
      if (strict_eq(prop(r, "role"), rule_role)) reduced.push_back(r);
    VP rse = u(U_roleScopingEntity), oe = u(U_ownerEntity), rsi = u(U_roleScopingInstance);
    auto direct = [&](VP owner) -> bool {
      for (VP ra : reduced) {
        VP attrs = get(ra, "attributes");
        if (nullish(attrs)) continue;
        for (VP rae : or_empty(attrs)) {
          if (strict_eq(get(rae, "id"), rse) && strict_eq(get(owner, "id"), oe) &&
              strict_eq(prop(owner, "value"), scoping_entity) && strict_eq(prop(owner, "value"), get(rae, "value"))) {
            VP insts = get(rae, "attributes");
            if (nullish(insts)) continue;
            for (VP inst : iterate(insts)) {
              if (!strict_eq(get(inst, "id"), rsi)) continue;
              VP oattrs = get(owner, "attributes");
              if (nullish(oattrs)) continue;
              for (VP oa : iterate(oattrs))
                if (strict_eq(get(oa, "value"), get(inst, "value"))) {
                  if (truthy(oa)) return true;
                  break;
                }
            }
          }
        }
      }
      return false;
    };
    std::vector<VP> remaining;  // owners lists still unmatched (Map order)
    for (auto& kv : owners_map.items) {
      bool any = false;
      for (VP o : iterate(kv.second))
        if (direct(o)) {
          any = true;
          break;
        }
      if (!any) remaining.push_back(kv.second);
    }
    if (remaining.empty()) return true;
    if (strict_eq(hr_check, S_TRUE)) {
      VP subj = get(ctx, "subject");
      if (truthy(get(subj, "token")) && lodash_is_empty(get(subj, "hierarchical_scopes")))
        unsupported("createHRScope I/O (token)");
      const Flat& flat = flat_hr(get(subj, "hierarchical_scopes"), rule_role, memo);
      auto owner_ok = [&](VP owner) -> bool {
        for (VP ra : reduced) {
          VP attrs = get(ra, "attributes");
          if (nullish(attrs)) continue;
          for (VP rae : or_empty(attrs))
            if (strict_eq(get(rae, "id"), rse) && strict_eq(get(owner, "id"), oe) &&
                strict_eq(get(owner, "value"), scoping_entity) && strict_eq(get(owner, "value"), get(rae, "value")))
              return true;
        }
        return false;
      };
      std::vector<VP> still;
      for (VP owners : remaining) {
        bool hit = false;
        for (VP owner : iterate(owners)) {
          if (!owner_ok(owner)) continue;
          VP oattrs = get(owner, "attributes");
          if (nullish(oattrs)) continue;
          for (VP a : iterate(oattrs))
            if (strict_eq(get(a, "id"), u(U_ownerInstance))) {
              VP v = get(a, "value");
              if (v->t == T::Str && flat.count(std::string_view(v->s))) hit = true;
            }
        }
        if (!hit) still.push_back(owners);
      }
      remaining.swap(still);
    }
    return remaining.empty();
  }

  // ---------------------------------------------------------------- ACL
  bool verify_acl(const Target& t, VP request) const {  // verifyACL.ts:11-251
    std::vector<VP> scoped_roles;
    for (VP a : or_empty(t.subjects)) {
      if (strict_eq(prop(a, "id"), u(U_role))) {
        scoped_roles.push_back(get(a, "value"));
      } else if (strict_eq(prop(a, "id"), u(U_skipACL))) {
        return true;
      }
    }
    VP ctx = get(request, "context");
    static const Val kEmptyObj = [] { Val v; v.t = T::Obj; return v; }();
    if (lodash_is_empty(ctx)) ctx = &kEmptyObj;
    VP ctx_resources = &kEmptyArr;
    {
      VP cr = prop(ctx, "resources");
      if (truthy(cr)) ctx_resources = cr;
    }
    VP req_target = get(request, "target");
    OrderedMap<std::vector<VP>> tmap;  // scopingEntity -> instances
    std::vector<VP> t_entities;
    for (VP qa : or_empty(prop(req_target, "resources"))) {
      if (!(loose_eq(prop(qa, "id"), u(U_resourceID)) || strict_eq(prop(qa, "id"), u(U_operation)))) continue;
      VP inst_id = prop(qa, "value");
      VP res = lodash_find(ctx_resources, "instance.id", inst_id);
      VP acl_list = UNDEF;
      if (truthy(res)) res = prop(res, "instance");
      else res = lodash_find(ctx_resources, "id", inst_id);
      if (truthy(res)) {
        VP meta = prop(res, "meta");
        if (length_gt0(get(meta, "acls"))) acl_list = get(meta, "acls");
      }
      if (lodash_is_empty(acl_list)) return true;
      for (VP acl : iterate(acl_list)) {
        if (!strict_eq(get(acl, "id"), u(U_aclIndicatoryEntity))) return false;
        VP se = prop(acl, "value");
        const std::string k = map_key(se);
        if (!tmap.index.count(k)) {
          tmap.set(k, {});
          t_entities.push_back(se);
        }
        VP attrs = prop(acl, "attributes");
        if (!truthy(attrs) || length_of(attrs) == 0) return false;
        for (VP at : iterate(attrs)) {
          if (!strict_eq(prop(at, "id"), u(U_aclInstance))) return false;
          tmap.items[tmap.index[k]].second.push_back(prop(at, "value"));
        }
      }
    }
    VP subj = prop(ctx, "subject");
    if (truthy(get(subj, "token")) && lodash_is_empty(get(subj, "hierarchical_scopes")))
      unsupported("createHRScope I/O (token)");
    VP ras = prop(subj, "role_associations");
    if (lodash_is_empty(ras)) return false;
    OrderedMap<std::vector<VP>> smap;
    for (VP ra : iterate(ras)) {
      VP role = get(ra, "role");
      if (!js_includes(scoped_roles, role)) continue;
      for (VP rattr : or_empty(get(ra, "attributes"))) {
        if (strict_eq(get(rattr, "id"), u(U_roleScopingEntity)) && js_includes(t_entities, get(rattr, "value"))) {
          VP rse_v = get(rattr, "value");
          const std::string k = map_key(rse_v);
          if (!smap.index.count(k)) smap.set(k, {});  // !subjectScopedInstancesMap.get(k) -> []
          if (length_gt0(get(rattr, "attributes")))
            for (VP ri : iterate(get(rattr, "attributes")))
              if (strict_eq(get(ri, "id"), u(U_roleScopingInstance)))
                smap.items[smap.index[k]].second.push_back(get(ri, "value"));
        }
      }
    }
    VP actions = get(req_target, "actions");
    // roleWithOrgScopesMap: effective role -> org ids (verifyACL.ts:129-145)
    OrderedMap<std::vector<VP>> role_orgs;
    std::vector<VP> role_keys;
    std::function<void(VP, VP)> walk = [&](VP nodes, VP role) {
      for (VP h : iterate(nodes)) {
        VP hr = prop(h, "role");
        VP key = nullish(hr) ? role : hr;
        if (truthy(get(h, "id"))) {
          const std::string k = map_key(key);
          if (!role_orgs.index.count(k)) {
            role_orgs.set(k, {});
            role_keys.push_back(key);
          }
          role_orgs.items[role_orgs.index[k]].second.push_back(get(h, "id"));
        }
        if (length_gt0(get(h, "children"))) walk(get(h, "children"), key);
      }
    };
    walk(get(subj, "hierarchical_scopes"), UNDEF);
    VP a0 = truthy(actions) && actions->t == T::Arr && !actions->a.empty() ? actions->a[0] : UNDEF;
    const bool is_action = truthy(actions) && truthy(a0) && strict_eq(prop(a0, "id"), u(U_actionID));
    if (is_action && strict_eq(prop(a0, "value"), u(U_create))) {
      bool valid = false;
      if (t_entities.empty()) return true;
      for (VP se : t_entities) {
        if (strict_eq(se, u(U_user))) {
          valid = true;
          continue;
        }
        const std::vector<VP>& t_inst = tmap.items[tmap.index[map_key(se)]].second;
        if (!smap.index.count(map_key(se))) return false;
        std::vector<VP> validated;
        for (size_t k = 0; k < role_orgs.items.size(); ++k) {
          if (!js_includes(scoped_roles, role_keys[k])) continue;
          const std::vector<VP>& orgs = role_orgs.items[k].second;
          for (VP ti : t_inst) {
            if (js_includes(orgs, ti)) {
              valid = true;
              validated.push_back(ti);
              continue;
            } else if (!js_includes(validated, ti)) {
              valid = false;
              break;
            }
          }
        }
        if (!valid) return false;
      }
      if (valid) return true;
    }
    if (is_action && (strict_eq(prop(a0, "value"), u(U_read)) || strict_eq(prop(a0, "value"), u(U_modify)) ||
                      strict_eq(prop(a0, "value"), u(U_delete)))) {
      if (t_entities.empty()) return true;
      for (VP se : t_entities) {
        const std::vector<VP>& t_inst = tmap.items[tmap.index[map_key(se)]].second;
        if (strict_eq(se, u(U_user)))
          if (js_includes(t_inst, get(subj, "id"))) return true;
        auto it = smap.index.find(map_key(se));
        if (it != smap.index.end())
          for (VP si : smap.items[it->second].second)
            if (js_includes(t_inst, si)) return true;
      }
      return false;
    }
    return false;
  }

  // ---------------------------------------------------------------- isAllowed (:88-324)
  static int32_t ec_code(VP v) {
    if (v->t == T::Undef) return 0;
    if (v->t == T::Null) return 1;
    if (v->t == T::Bool) return v->b ? 3 : 2;
    return 4;
  }

  static int32_t decision_code(VP e) {
    if (e->t != T::Str) return 5;
    if (e->s == "PERMIT") return 2;
    if (e->s == "DENY") return 3;
    if (e->s == "NOT_APPLICABLE") return 4;
    if (e->s == "INDETERMINATE") return 5;
    if (e->s == "UNRECOGNIZED") return 6;
    return 5;
  }

  Outcome is_allowed(VP request, SharedIds* cache = nullptr) const {
    role_set_reset();
    Outcome out;
    if (!truthy(get(request, "target"))) {  // :91-102
      out.decision = 3;
      out.ec = 2;
      out.code = 400;
      return out;
    }
    Memo memo;
    memo.cache = cache;
    VP ctx = get(request, "context");
    if (truthy(get(get(ctx, "subject"), "token"))) unsupported("subject token (identity-srv / Redis I/O)");
    bool have_effect = false;
    Effect effect;
    for (auto& skv : sets.items) {
      const PolicySet& pset = skv.second;
      std::vector<Effect> policy_effects;
      if (pset.target.present && !target_matches(pset.target, request, UNDEF, false)) continue;
      bool exact = false;
      VP pe = UNDEF;
      for (auto& pkv : pset.policies.items) {  // loop 2a (:136-157)
        const Policy& pol = pkv.second;
        if (pol.null) throw JSError{1};  // policy.effect of null (:138)
        VP eff = prop(pol.raw, "effect");
        if (truthy(eff)) pe = eff;
        if (pol.target.present && target_matches(pol.target, request, pe, false)) {
          exact = true;
          break;
        }
      }
      if (exact) {
        long n_ent = 0;
        for (VP a : or_empty(get(get(request, "target"), "resources")))
          if (strict_eq(get(a, "id"), u(U_entity))) ++n_ent;
        if (n_ent > 1) exact = multiple_entities_match(pset, request);
      }
      for (auto& pkv : pset.policies.items) {  // loop 2b (:167-290)
        const Policy& pol = pkv.second;
        if (pol.null) continue;  // if (!policy) continue
        std::vector<Effect> rule_effects;
        const bool gate = !pol.target.present || (exact && target_matches(pol.target, request, pe, false)) ||
                          (!exact && target_matches(pol.target, request, pe, true));
        if (!gate) continue;
        const bool psm = length_gt0(pol.target.present ? pol.target.subjects : UNDEF)
                             ? check_hierarchical_scope(pol.target, request, memo)
                             : true;
        if (pol.rules.size() == 0 && truthy(get(pol.raw, "effect"))) {
          policy_effects.push_back({get(pol.raw, "effect"), get(pol.raw, "evaluation_cacheable")});
          continue;
        }
        bool ec_rule = true;
        for (auto& rkv : pol.rules.items) {
          const Rule& rule = rkv.second;
          VP ec = get(rule.raw, "evaluation_cacheable");
          if (!truthy(ec)) ec_rule = false;
          bool m = !rule.target.present || target_matches(rule.target, request, get(rule.raw, "effect"), false);
          if (!m) m = target_matches(rule.target, request, get(rule.raw, "effect"), true);
          if (!m) continue;
          if (rule.target.present) m = check_hierarchical_scope(rule.target, request, memo);
          if (m && length_gt0(get(rule.raw, "condition"))) unsupported("rule condition (JS eval)");
          if (m && rule.target.present) m = verify_acl(rule.target, request);
          if (m && psm) {
            static const Val kFalse = [] { Val v; v.t = T::Bool; return v; }();
            rule_effects.push_back({get(rule.raw, "effect"), ec_rule ? ec : &kFalse});
          }
        }
        if (!rule_effects.empty()) policy_effects.push_back(decide(get(pol.raw, "combining_algorithm"), rule_effects));
      }
      if (!policy_effects.empty()) {
        effect = decide(get(pset.raw, "combining_algorithm"), policy_effects);
        have_effect = true;
      }
    }
    out.code = 200;
    if (!have_effect) {
      out.decision = 5;
      out.ec = 0;
      return out;
    }
    out.decision = decision_code(effect.effect);
    out.ec = ec_code(effect.ec);
    return out;
  }

  // ---------------------------------------------------------------- whatIsAllowed (:326-427)
  // The included sets / policies / rules as global node indices (sets in Map order, then every
  // set's policies in order, then every policy's rules in order; null entries keep their
  // slot: the numbering of the product's compiled image) and the maskedProperty push log.
  struct ReverseQuery {
    std::vector<uint32_t> sets, pols, rules;
    Pushes pushes;
  };

  ReverseQuery what_is_allowed(VP request) const {
    role_set_reset();
    ReverseQuery rq;
    VP ctx = get(request, "context");
    if (truthy(get(get(ctx, "subject"), "token"))) unsupported("subject token (identity-srv / Redis I/O)");
    Pushes* masks = &rq.pushes;
    uint32_t si = 0, pbase = 0, rbase = 0;
    for (auto& skv : sets.items) {
      const PolicySet& pset = skv.second;
      const uint32_t p0 = pbase;
      uint32_t rcount = 0;  // rules of this set's policies (null policies hold none)
      std::vector<uint32_t> rule_base(pset.policies.items.size());
      for (size_t q = 0; q < pset.policies.items.size(); ++q) {
        rule_base[q] = rbase + rcount;
        rcount += (uint32_t)pset.policies.items[q].second.rules.size();
      }
      pbase += (uint32_t)pset.policies.items.size();
      rbase += rcount;
      const uint32_t s_idx = si++;
      // set gate: _.isEmpty(target) || targetMatches(target, request, 'whatIsAllowed') (:344-347)
      if (pset.target.present && !target_matches(pset.target, request, UNDEF, false, masks)) continue;
      bool exact = false;
      VP pe = UNDEF;
      for (auto& pkv : pset.policies.items) {  // :353-368 (the CA branch never fires, as in isAllowed)
        const Policy& pol = pkv.second;
        if (pol.null) throw JSError{1};  // policy.effect of null
        VP eff = prop(pol.raw, "effect");
        if (truthy(eff)) pe = eff;
        if (pol.target.present && target_matches(pol.target, request, pe, false, masks)) {
          exact = true;
          break;
        }
      }
      if (exact) {  // :373-376
        long n_ent = 0;
        for (VP a : or_empty(get(get(request, "target"), "resources")))
          if (strict_eq(get(a, "id"), u(U_entity))) ++n_ent;
        if (n_ent > 1) exact = multiple_entities_match(pset, request);
      }
      std::vector<uint32_t> pols, rules;
      for (size_t q = 0; q < pset.policies.items.size(); ++q) {  // :378-414
        const Policy& pol = pset.policies.items[q].second;
        if (pol.null || !truthy(pol.raw)) continue;
        const bool gate = !pol.target.present || (exact && target_matches(pol.target, request, pe, false, masks)) ||
                          (!exact && target_matches(pol.target, request, pe, true, masks));
        if (!gate) continue;
        std::vector<uint32_t> prules;
        for (size_t r = 0; r < pol.rules.items.size(); ++r) {
          const Rule& rule = pol.rules.items[r].second;
          if (!truthy(rule.raw)) continue;
          VP re = get(rule.raw, "effect");
          bool m = !rule.target.present || target_matches(rule.target, request, re, false, masks);
          if (!m) m = target_matches(rule.target, request, re, true, masks);
          if (!rule.target.present || m) prules.push_back(rule_base[q] + (uint32_t)r);
        }
        if (truthy(get(pol.raw, "effect")) || !prules.empty()) {  // :411-413
          pols.push_back(p0 + (uint32_t)q);
          rules.insert(rules.end(), prules.begin(), prules.end());
        }
      }
      if (!pols.empty()) {  // :416-418
        rq.sets.push_back(s_idx);
        rq.pols.insert(rq.pols.end(), pols.begin(), pols.end());
        rq.rules.insert(rq.rules.end(), rules.begin(), rules.end());
      }
    }
    return rq;
  }
};

void json_string(std::string& o, const std::string& s) {
  o += '"';
  for (unsigned char c : s) {
    if (c == '"' || c == '\\') {
      o += '\\';
      o += (char)c;
    } else if (c < 0x20) {
      char b[8];
      snprintf(b, sizeof b, "\\u%04x", c);
      o += b;
    } else {
      o += (char)c;
    }
  }
  o += '"';
}

// A JS value of the push log as JSON: strings as strings, null as null, undefined as
// {"$undef":1}, anything else as {"$other":1} (never compared: the product sends such values
// to the host).
void json_value(std::string& o, VP v) {
  if (v->t == T::Str) json_string(o, v->s);
  else if (v->t == T::Null) o += "null";
  else if (v->t == T::Undef) o += "{\"$undef\":1}";
  else o += "{\"$other\":1}";
}

template <class V>
void json_ints(std::string& o, const V& v) {
  o += '[';
  for (size_t k = 0; k < v.size(); ++k) {
    if (k) o += ',';
    o += std::to_string(v[k]);
  }
  o += ']';
}

thread_local std::string g_err;

}  // namespace

extern "C" {

const char* acs_oracle_last_error(void) { return g_err.c_str(); }

// urns / cas / doc: JSON texts (policies.options.urns, .combiningAlgorithms, {policy_sets}).
void* acs_oracle_create(const char* urns, const char* cas, const char* doc) {
  auto* o = new Oracle();
  try {
    Parser pu(urns, strlen(urns), o->arena), pc(cas, strlen(cas), o->arena), pd(doc, strlen(doc), o->arena);
    o->init_urns(pu.value());
    o->init_cas(pc.value());
    o->load(pd.value());
  } catch (const std::exception& e) {
    g_err = e.what();
    delete o;
    return nullptr;
  } catch (const JSError&) {
    g_err = "JS error while loading the store";
    delete o;
    return nullptr;
  } catch (const Unsupported& u) {
    g_err = u.why;
    delete o;
    return nullptr;
  }
  return o;
}

void acs_oracle_free(void* h) { delete (Oracle*)h; }

// One step of the entity namespace / RegExp test (regex_entity) for two string values
// (NULL = JSON null): 1 HIT | 2 RESET, 4 TypeError, 8 SyntaxError, -1 outside the restated
// subset.  tests/test_regex_v8.py checks it against V8 (tests/golden/regex_cells.json).
int acs_oracle_regex_cell(const char* rule, const char* req) {
  static const Oracle kNoStore{};
  Val rv, qv;
  if (rule) { rv.t = T::Str; rv.s = rule; } else { rv.t = T::Null; }
  if (req) { qv.t = T::Str; qv.s = req; } else { qv.t = T::Null; }
  try {
    const auto rh = kNoStore.regex_entity(&rv, &qv);
    return (rh.first ? 2 : 0) | (rh.second ? 1 : 0);
  } catch (const JSError& e) {
    return e.kind == 1 ? 4 : 8;
  } catch (const Unsupported&) {
    return -1;
  }
}

// requests: a JSON array of n requests.  out: 4 int32 per request (Outcome).  Evaluation
// (not parsing) is timed and spread over `threads` std::threads; *seconds gets its wall time.
int acs_oracle_is_allowed_shared(void* h, const char* shared_json, const char* requests, size_t n, int threads,
                                 int32_t* out, double* seconds);

int acs_oracle_is_allowed(void* h, const char* requests, size_t n, int threads, int32_t* out, double* seconds) {
  return acs_oracle_is_allowed_shared(h, nullptr, requests, n, threads, out, seconds);
}

// shared_json: NULL, or a JSON array whose k-th element replaces every {"$shared": k} object
// of the requests (parsed once, shared read-only by the requests that name it).
int acs_oracle_is_allowed_shared(void* h, const char* shared_json, const char* requests, size_t n, int threads,
                                 int32_t* out, double* seconds) {
  auto* o = (Oracle*)h;
  Arena arena;
  VP arr;
  std::vector<VP> shared;
  try {
    if (shared_json) {
      Parser ps(shared_json, strlen(shared_json), arena);
      VP sv = ps.value();
      if (sv->t != T::Arr) throw std::runtime_error("shared: expected a JSON array");
      shared = sv->a;
    }
    Parser p(requests, strlen(requests), arena);
    if (shared_json) p.shared = &shared;
    arr = p.value();
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
  if (arr->t != T::Arr || arr->a.size() != n) {
    g_err = "requests: expected a JSON array of n requests";
    return -1;
  }
  if (threads < 1) threads = 1;
  std::atomic<size_t> next{0};
  // requests per grab: 64 for large calls, down to 1 so that every thread has work in a small one
  const size_t grain = std::max<size_t>(1, std::min<size_t>(64, n / (4 * (size_t)threads)));
  const std::unordered_set<VP> shared_set(shared.begin(), shared.end());
  auto work = [&] {
    Oracle::SharedIds cache;
    cache.shared_values = &shared_set;
    for (;;) {
      const size_t i = next.fetch_add(grain);
      if (i >= n) return;
      const size_t e = std::min(n, i + grain);
      for (size_t k = i; k < e; ++k) {
        Outcome r;
        try {
          r = o->is_allowed(arr->a[k], &cache);
        } catch (const JSError& err) {
          r.kind = 1;
          r.code = err.kind;
        } catch (const Unsupported&) {
          r.kind = 2;
        }
        out[4 * k] = r.kind;
        out[4 * k + 1] = r.decision;
        out[4 * k + 2] = r.ec;
        out[4 * k + 3] = r.code;
      }
    }
  };
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return 0;
}

// whatIsAllowed (accessController.ts:326-427) of n requests (a JSON array; shared_json as in
// acs_oracle_is_allowed_shared), evaluated on `threads` std::threads.  *out_json (free with
// acs_oracle_free_text): a JSON array with one element per request:
//   {"k":0,"s":[set idx],"p":[policy idx],"r":[rule idx],"o":[[entity, mask], ...]}  (global
//   node indices in the compiled image's numbering; "o" the maskedProperty pushes in order)
//   {"k":1,"e":kind}  the reference rejects (1 TypeError, 2 InvalidCombiningAlgorithm, 3 SyntaxError)
//   {"k":2}           outside the restatement (token I/O, RegExp outside the subset, ...)
int acs_oracle_what_is_allowed_shared(void* h, const char* shared_json, const char* requests, size_t n, int threads,
                                      char** out_json, double* seconds) {
  auto* o = (Oracle*)h;
  Arena arena;
  VP arr;
  std::vector<VP> shared;
  try {
    if (shared_json) {
      Parser ps(shared_json, strlen(shared_json), arena);
      VP sv = ps.value();
      if (sv->t != T::Arr) throw std::runtime_error("shared: expected a JSON array");
      shared = sv->a;
    }
    Parser p(requests, strlen(requests), arena);
    if (shared_json) p.shared = &shared;
    arr = p.value();
  } catch (const std::exception& e) {
    g_err = e.what();
    return -1;
  }
  if (arr->t != T::Arr || arr->a.size() != n) {
    g_err = "requests: expected a JSON array of n requests";
    return -1;
  }
  if (threads < 1) threads = 1;
  std::vector<std::string> parts(n);
  std::atomic<size_t> next{0};
  // requests per grab: 64 for large calls, down to 1 so that every thread has work in a small one
  const size_t grain = std::max<size_t>(1, std::min<size_t>(64, n / (4 * (size_t)threads)));
  auto work = [&] {
    for (;;) {
      const size_t i = next.fetch_add(grain);
      if (i >= n) return;
      const size_t e = std::min(n, i + grain);
      for (size_t k = i; k < e; ++k) {
        std::string& s = parts[k];
        try {
          const Oracle::ReverseQuery rq = o->what_is_allowed(arr->a[k]);
          s = "{\"k\":0,\"s\":";
          json_ints(s, rq.sets);
          s += ",\"p\":";
          json_ints(s, rq.pols);
          s += ",\"r\":";
          json_ints(s, rq.rules);
          s += ",\"o\":[";
          for (size_t x = 0; x < rq.pushes.size(); ++x) {
            if (x) s += ',';
            s += '[';
            json_value(s, rq.pushes[x].first);
            s += ',';
            json_value(s, rq.pushes[x].second);
            s += ']';
          }
          s += "]}";
        } catch (const JSError& err) {
          s = "{\"k\":1,\"e\":" + std::to_string(err.kind) + "}";
        } catch (const Unsupported&) {
          s = "{\"k\":2}";
        }
      }
    }
  };
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> pool;
  for (int t = 1; t < threads; ++t) pool.emplace_back(work);
  work();
  for (auto& t : pool) t.join();
  if (seconds) *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  size_t total = 2;
  for (auto& x : parts) total += x.size() + 1;
  char* buf = (char*)malloc(total + 1);
  if (!buf) {
    g_err = "out of memory";
    return -1;
  }
  size_t at = 0;
  buf[at++] = '[';
  for (size_t k = 0; k < n; ++k) {
    if (k) buf[at++] = ',';
    memcpy(buf + at, parts[k].data(), parts[k].size());
    at += parts[k].size();
  }
  buf[at++] = ']';
  buf[at] = 0;
  *out_json = buf;
  return 0;
}

void acs_oracle_free_text(char* p) { free(p); }

}  // extern "C"
