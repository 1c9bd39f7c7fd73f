// acs_compiler.cpp — native policy-store compiler (C ABI: acs_store_compile, include/acs_mi355x.h).
//
// The `policySets` Map of AccessController (accessController.ts:32; nested combinables
// Maps, interfaces.ts:12-18) as a JSON snapshot -> the store image acs_compile and
// acs_codec_create take.  It restates acs_mi355x/compiler.py (compile_store + store_blob)
// step for step, interning strings in the same order, so the image is byte-identical to
// the Python compiler's (tests/test_codec.py).  Everything that depends on a rule / policy
// / set alone is evaluated here once:
//
//   target subject scan (role, roleScopingEntity, hierarchicalRoleScoping, skipACL)
//                                  accessController.ts:797-806, hierarchicalScope.ts:25-42, verifyACL.ts:13-25
//   policyEffect prefix (pe_at)    accessController.ts:136-148
//   evaluation_cacheable prefix    accessController.ts:202-211
//   effect / CA codes              accessController.ts:299-312, 832-838
//   candidate specs                acs_mi355x/candidates.py
//
// Snapshot format: a JSON array of the Map's values in Map order; a set's `combinables` is
// the array of its policies (Map order, null entries kept), a policy's `combinables` the
// array of its rules — JSON.stringify of Array.from(map.values()) at each level.
#include <sys/mman.h>
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <string_view>
#include <unordered_map>
#include <vector>

#include "../../include/acs_mi355x.h"
#include "acs_json.h"
#include "acs_layout.h"

extern "C" void acs_internal_set_error(const char* msg);

using namespace acs;
using namespace acs_json;

namespace {

// Image blobs: zeroed storage behind a 64-B header (kind, mapping size).  Large images are
// anonymous mappings with 2-MB pages (zero on first touch; the fragments are written in
// parallel, and 4-KB page faults serialised a c5 image's 120 MB); small ones come from calloc.
constexpr uint64_t BLOB_MMAP = 0x6d6d6170u, BLOB_HEAP = 0x68656170u;
void* blob_alloc_zeroed(size_t n) {
  constexpr size_t HDR = 64, HUGE = size_t(2) << 20;
  if (n >= 8 * HUGE) {
    const size_t m = (n + HDR + HUGE - 1) / HUGE * HUGE;
    void* p = mmap(nullptr, m, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
    if (p != MAP_FAILED) {
      madvise(p, m, MADV_HUGEPAGE);
      uint64_t* h = (uint64_t*)p;
      h[0] = BLOB_MMAP;
      h[1] = m;
      return (char*)p + HDR;
    }
  }
  uint64_t* h = (uint64_t*)calloc(n + HDR, 1);
  if (!h) return nullptr;
  h[0] = BLOB_HEAP;
  return (char*)h + HDR;
}
void blob_release(void* blob) {
  if (!blob) return;
  uint64_t* h = (uint64_t*)((char*)blob - 64);
  if (h[0] == BLOB_MMAP) munmap(h, (size_t)h[1]);
  else free(h);
}

}  // namespace

namespace {

struct CompileError {
  std::string why;
};
[[noreturn]] void fail(const std::string& why) { throw CompileError{why}; }

const char* const kCodecUrns[] = {"entity", "property", "operation", "resourceID", "actionID", "role",
                                  "roleScopingEntity", "roleScopingInstance", "hierarchicalRoleScoping",
                                  "ownerEntity", "ownerInstance", "aclIndicatoryEntity", "aclInstance", "create",
                                  "read", "modify", "delete", "user", "skipACL", "maskedProperty"};
constexpr int N_CODEC_URNS = 20;

// Object.prototype members: an effect string naming one resolves to a function in
// Response_Decision[effect] (accessController.ts:312) — not restated, refused.
const char* const kProtoKeys[] = {"constructor", "__proto__", "toString", "toLocaleString", "valueOf",
                                  "hasOwnProperty", "isPrototypeOf", "propertyIsEnumerable", "__defineGetter__",
                                  "__defineSetter__", "__lookupGetter__", "__lookupSetter__"};

void json_write(std::string& o, const JV* v);

struct Builder {
  // dictionary (compiler.Dictionary: 0 undefined, 1 null, 2 '')
  std::vector<std::string> strings{"", "", ""};
  std::unordered_map<std::string, uint32_t> ids{{"", ID_EMPTY}};
  // URN config
  std::vector<std::pair<std::string, const JV*>> urns;  // config order
  std::unordered_map<std::string, const JV*> urn;
  // combining algorithms: urn key -> code
  std::vector<std::pair<std::string, uint8_t>> ca_map;  // key: 's'+urn / 'm' undefined / 'n' null
  // pools
  std::vector<RuleResAttr> rres;
  std::vector<Pair> pairs;
  std::vector<uint32_t> u32pool;
  std::vector<uint32_t> rx_rows;  // row -> dictionary id of the value (0 undefined, 1 null)
  std::unordered_map<uint32_t, uint32_t> rx_index;
  // evaluation_cacheable values: kind (0 undefined 1 null 2 false 3 true 4 number 5 string 6 object)
  struct Ec {
    int kind;
    double num;
    std::string s;
    bool truthy;
    std::string json;  // the value as JSON text (the codec section; outlives the parsed store)
  };
  std::vector<Ec> ec{{0, 0, "", false}, {1, 0, "", false}, {2, 0, "", false}, {3, 0, "", true}};
  // node tables + candidate specs (kind 0 never, 1 always, 2 rows)
  std::vector<NodeRec> sets, pols, rules;
  // flat per section (sets, policies, rules): kind per node, the node's end in spec_idx, and
  // the regex rows of kind-2 nodes
  std::vector<uint8_t> spec_kind[3];
  std::vector<uint32_t> spec_end[3], spec_idx[3];

  uint32_t intern(const JV* v) {
    if (v->t == J_UNDEF) return ID_UNDEF;
    if (v->t == J_NULL) return ID_NULL;
    if (v->t != J_STR) fail("non-string value");
    return intern_sv(v->str());
  }
  uint32_t intern_sv(std::string_view s) {
    auto it = ids.find(std::string(s));
    if (it != ids.end()) return it->second;
    const uint32_t i = (uint32_t)strings.size();
    strings.emplace_back(s);
    ids.emplace(std::string(s), i);
    return i;
  }
  const JV* U(const char* name) const {
    auto it = urn.find(name);
    return it == urn.end() ? &kUndef : it->second;
  }
  static bool strict_eq(const JV* a, const JV* b) {
    if (a->t == J_UNDEF || b->t == J_UNDEF || a->t == J_NULL || b->t == J_NULL) return a->t == b->t;
    if (a->t == J_STR || b->t == J_STR) return a->t == J_STR && b->t == J_STR && a->str() == b->str();
    if ((a->t == J_TRUE || a->t == J_FALSE) || (b->t == J_TRUE || b->t == J_FALSE)) return a->t == b->t;
    if (a->t == J_NUM && b->t == J_NUM) return a->num == b->num;
    return a == b;
  }
  static void check_scalar(const JV* v) {
    if (!(v->t == J_UNDEF || v->t == J_NULL || v->t == J_STR)) fail("non-string attribute scalar");
  }
  uint8_t ca_code(const JV* urn_v) const {
    std::string key;
    if (urn_v->t == J_UNDEF) key = "m";
    else if (urn_v->t == J_NULL) key = "n";
    else if (urn_v->t == J_STR) key = "s" + std::string(urn_v->str());
    else return CA_INVALID;  // a non-string combining_algorithm matches no configured URN
    for (auto& kv : ca_map)
      if (kv.first == key) return kv.second;
    return CA_INVALID;
  }
  static uint8_t effect_code(const JV* e) {
    if (e->t == J_UNDEF) return EFF_UNDEF;
    if (e->t == J_NULL) return EFF_NULL;
    if (e->t == J_STR) {
      const std::string_view s = e->str();
      for (const char* k : kProtoKeys)
        if (s == k) fail("effect resolves to an Object.prototype member");
      if (s == "PERMIT") return EFF_PERMIT;
      if (s == "DENY") return EFF_DENY;
      if (s == "NOT_APPLICABLE") return EFF_NOT_APPLICABLE;
      if (s == "INDETERMINATE") return EFF_INDETERMINATE;
      if (s == "UNRECOGNIZED") return EFF_UNRECOGNIZED;
    }
    return truthy(e) ? EFF_OTHER_TRUTHY : EFF_OTHER_FALSY;
  }
  uint8_t ec_code(const JV* v) {
    Ec x{6, 0, "", true};
    switch (v->t) {
      case J_UNDEF: return EC_UNDEF;
      case J_NULL: return EC_NULL;
      case J_FALSE: return EC_FALSE;
      case J_TRUE: return EC_TRUE;
      case J_NUM: x = {4, v->num, "", v->num == v->num && v->num != 0}; break;
      case J_STR: x = {5, 0, std::string(v->str()), v->n != 0}; break;
      default: break;  // objects / arrays: each value its own entry (identity)
    }
    if (x.kind != 6)
      for (size_t k = 4; k < ec.size(); ++k)
        if (ec[k].kind == x.kind && (x.kind == 4 ? ec[k].num == x.num : ec[k].s == x.s)) return (uint8_t)k;
    if (ec.size() >= 255) fail("too many distinct evaluation_cacheable values");
    json_write(x.json, v);
    ec.push_back(x);
    return (uint8_t)(ec.size() - 1);
  }
  uint32_t rx_row(const JV* v) {
    const uint32_t id = intern(v);
    auto it = rx_index.find(id);
    if (it != rx_index.end()) return it->second;
    const uint32_t r = (uint32_t)rx_rows.size();
    if (r >= 0xFFFF) fail("too many distinct rule entity values");
    rx_index.emplace(id, r);
    rx_rows.push_back(id);
    return r;
  }
  static const JV* attrs(const JV* v, const char* what) {  // _attrs of `v || []`
    if (!truthy(v)) return nullptr;
    if (v->t != J_ARR) fail(std::string("target ") + what + " is not an array");
    for (uint32_t k = 0; k < v->n; ++k) {
      if (v->a[k].t != J_OBJ) fail(std::string("non-object entry in target ") + what);
      check_scalar(get(&v->a[k], "id"));
      check_scalar(get(&v->a[k], "value"));
    }
    return v;
  }
  uint32_t add_pairs(const JV* lst) {
    const uint32_t off = (uint32_t)pairs.size();
    if (lst)
      for (uint32_t k = 0; k < lst->n; ++k)
        pairs.push_back(Pair{intern(get(&lst->a[k], "id")), intern(get(&lst->a[k], "value"))});
    return off;
  }

  struct Target {
    bool present = false;
    NodeRec rec{};
    int spec_kind = 1;  // 1 always, 2 rows
    std::vector<uint32_t> rows;
  };

  // compiler._Builder.target: inline target fields of a node record
  Target target(const JV* t) {
    Target T;
    if (!truthy(t)) return T;
    if (t->t != J_OBJ) fail("target is not an object");
    T.present = true;
    const JV* subs = attrs(get(t, "subjects"), "subjects");
    const JV* acts = attrs(get(t, "actions"), "actions");
    const JV* res = attrs(get(t, "resources"), "resources");
    const JV* sj = get(t, "subjects");
    if (sj->t != J_UNDEF && sj->t != J_ARR) fail("subjects");
    const uint32_t ns = subs ? subs->n : 0, na = acts ? acts->n : 0, nr = res ? res->n : 0;
    NodeRec& R = T.rec;
    uint32_t flags = 0;
    const JV* role = &kUndef;
    for (uint32_t k = 0; k < ns; ++k)
      if (strict_eq(get(&subs->a[k], "id"), U("role"))) role = get(&subs->a[k], "value");
    if (ns == 0) flags |= TF_SUBJ_EMPTY;
    else if (truthy(role)) flags |= TF_SUBJ_ROLE;
    if (ns > 0) flags |= TF_HAS_SUBJECTS;
    R.role = intern(role);
    R.subj_off = add_pairs(subs);
    R.subj_n = (uint16_t)ns;
    R.act_off = add_pairs(acts);
    R.act_n = (uint16_t)na;
    // checkHierarchicalScope subject scan (if / else-if chain, hierarchicalScope.ts:29-37)
    static const JV kTrue = [] {
      JV v;
      v.t = J_STR;
      v.s = "true";
      v.n = 4;
      return v;
    }();
    const JV* hr_check = &kTrue;
    const JV* se = &kUndef;
    for (uint32_t k = 0; k < ns; ++k) {
      const JV* i = get(&subs->a[k], "id");
      if (strict_eq(i, U("role"))) {
      } else if (strict_eq(i, U("hierarchicalRoleScoping"))) {
        hr_check = get(&subs->a[k], "value");
      } else if (strict_eq(i, U("roleScopingEntity"))) {
        se = get(&subs->a[k], "value");
      }
    }
    if (ns == 0 || !truthy(se)) flags |= TF_HR_TRIVIAL;
    if (hr_check->t == J_STR && hr_check->str() == "true") flags |= TF_HR_CHECK;
    R.se = intern(se);
    // verifyACLList subject scan (verifyACL.ts:17-25)
    std::vector<uint32_t> scoped;
    for (uint32_t k = 0; k < ns; ++k) {
      const JV* i = get(&subs->a[k], "id");
      if (strict_eq(i, U("role"))) {
        scoped.push_back(intern(get(&subs->a[k], "value")));
      } else if (strict_eq(i, U("skipACL"))) {
        flags |= TF_ACL_SKIP;
        break;
      }
    }
    R.acl_roles_off = (uint32_t)u32pool.size();
    R.acl_roles_n = (uint16_t)scoped.size();
    u32pool.insert(u32pool.end(), scoped.begin(), scoped.end());
    // resources
    if (nr == 0) flags |= TF_RES_EMPTY;
    R.res_off = (uint32_t)rres.size();
    R.res_n = (uint16_t)nr;
    const JV* last_prop = &kUndef;
    const JV* uent = U("entity");
    for (uint32_t k = 0; k < nr; ++k) {
      const JV* i = get(&res->a[k], "id");
      const JV* v = get(&res->a[k], "value");
      uint8_t kind = 0;
      if (strict_eq(i, uent)) kind |= K_ENT;
      if ((nullish(i) && nullish(uent)) || strict_eq(i, uent)) kind |= K_ENT_LOOSE;
      if (strict_eq(i, U("operation"))) kind |= K_OP;
      if (strict_eq(i, U("property"))) {
        kind |= K_PROP;
        flags |= TF_RULE_PROPS;
        last_prop = v;
      }
      uint32_t hs = ID_UNDEF;
      if ((kind & K_PROP) && v->t == J_STR) {
        const std::string_view s = v->str();
        const size_t h = s.rfind('#');
        hs = intern_sv(h == std::string_view::npos ? s : s.substr(h + 1));
      }
      const uint32_t row = (kind & K_ENT_LOOSE) ? rx_row(v) : 0;
      RuleResAttr a{};
      a.value = intern(v);
      a.hash_sfx = hs;
      a.row = (uint16_t)row;
      a.kind = kind;
      rres.push_back(a);
    }
    R.last_prop_value = intern(last_prop);
    bool has_op = false, prop_or_op = false;
    for (uint32_t k = 0; k < nr; ++k) {
      const JV* i = get(&res->a[k], "id");
      has_op = has_op || strict_eq(i, U("operation"));
      prop_or_op = prop_or_op || strict_eq(i, U("property")) || strict_eq(i, U("operation"));
    }
    if (nr == 0 || has_op) {
      T.spec_kind = 1;
    } else {
      T.spec_kind = 2;
      for (uint32_t k = 0; k < nr; ++k)
        if (strict_eq(get(&res->a[k], "id"), uent)) T.rows.push_back(rx_row(get(&res->a[k], "value")));
    }
    if (nr > 0 && !prop_or_op) flags |= TF_RES_ENT_ONLY;
    if (last_prop->t == J_STR) {
      flags |= TF_LASTPROP_STR;
      if (last_prop->str().find('#') != std::string_view::npos) flags |= TF_LASTPROP_HASH;
    }
    R.tflags = flags;
    return T;
  }

  void push_spec(int sec, bool has_target, const Target& T, bool null_rule) {
    // a target listing entity rows but none (no entity attribute): never a candidate
    const uint8_t k = has_target ? (uint8_t)(T.spec_kind == 2 && T.rows.empty() ? 0 : T.spec_kind) : (null_rule ? 0 : 1);
    spec_kind[sec].push_back(k);
    if (k == 2) spec_idx[sec].insert(spec_idx[sec].end(), T.rows.begin(), T.rows.end());
    spec_end[sec].push_back((uint32_t)spec_idx[sec].size());
  }

  // compiler._compile_set + _assemble (global offsets from the start)
  void compile_set(const JV* ps) {
    if (ps->t != J_OBJ) fail("null policy set");
    Target st = target(get(ps, "target"));
    NodeRec S = st.rec;
    S.nflags = st.present ? NF_HAS_TARGET : 0;
    S.child_begin = (uint32_t)pols.size();
    const JV* combin = get(ps, "combinables");
    if (combin->t != J_ARR) fail("policy set without combinables");
    uint8_t pe_at = EFF_UNDEF;
    uint8_t set_free = NF_COND_FREE;  // no condition rule and no invalid combining algorithm below
    std::vector<NodeRec> my_pols;  // set record goes first in the Python order of node appends
    for (uint32_t k = 0; k < combin->n; ++k) {
      const JV* pol = &combin->a[k];
      if (pol->t == J_NULL) {
        NodeRec P{};
        P.nflags = NF_NULL;
        P.child_begin = P.child_end = P.fe = (uint32_t)rules.size();
        P.pe_at = pe_at;
        pols.push_back(P);
        push_spec(1, false, Target{}, false);
        continue;
      }
      if (pol->t != J_OBJ) fail("policy is not an object");
      Target pt = target(get(pol, "target"));
      NodeRec P = pt.rec;
      uint8_t nf = pt.present ? NF_HAS_TARGET : 0;
      if (truthy(get(pol, "effect"))) {
        nf |= NF_EFFECT_TRUTHY;
        pe_at = effect_code(get(pol, "effect"));  // accessController.ts:138-140
      }
      P.nflags = nf;
      P.child_begin = (uint32_t)rules.size();
      P.effect = effect_code(get(pol, "effect"));
      P.ec = ec_code(get(pol, "evaluation_cacheable"));
      P.ca = ca_code(get(pol, "combining_algorithm"));
      P.pe_at = pe_at;
      const JV* rcomb = get(pol, "combinables");
      if (rcomb->t != J_ARR) fail("policy without combinables");
      uint32_t fe = NONE32;
      uint8_t pol_free = NF_COND_FREE;
      for (uint32_t r = 0; r < rcomb->n; ++r) {
        const JV* rule = &rcomb->a[r];
        if (rule->t == J_NULL) {
          NodeRec Q{};
          Q.nflags = NF_NULL;
          rules.push_back(Q);
          push_spec(2, false, Target{}, true);
          continue;
        }
        if (rule->t != J_OBJ) fail("rule is not an object");
        Target rt = target(get(rule, "target"));
        NodeRec Q = rt.rec;
        uint8_t rf = rt.present ? NF_HAS_TARGET : 0;
        const JV* cond = get(rule, "condition");
        const JV* clen_v = &kUndef;
        bool clen = false;
        if (cond->t == J_STR || cond->t == J_ARR) clen = cond->n > 0;
        else {
          clen_v = get(cond, "length");
          clen = truthy(clen_v);
        }
        if (clen) {
          rf |= NF_HAS_CONDITION;
          pol_free = 0;
        }
        const uint8_t ec = ec_code(get(rule, "evaluation_cacheable"));
        if (this->ec[ec].truthy) rf |= NF_EC_TRUTHY;
        else if (fe == NONE32) fe = (uint32_t)rules.size();
        Q.nflags = rf;
        Q.effect = effect_code(get(rule, "effect"));
        Q.ec = ec;
        rules.push_back(Q);
        push_spec(2, rt.present, rt, false);
      }
      P.child_end = (uint32_t)rules.size();
      P.map_size = rcomb->n;
      P.fe = fe == NONE32 ? (uint32_t)rules.size() : fe;
      P.nflags |= pol_free;
      if (!pol_free || P.ca == CA_INVALID) set_free = 0;
      pols.push_back(P);
      push_spec(1, pt.present, pt, false);
    }
    S.child_end = (uint32_t)pols.size();
    S.ca = ca_code(get(ps, "combining_algorithm"));
    S.pe_at = pe_at;
    S.nflags |= set_free;
    sets.push_back(S);
    push_spec(0, st.present, st, false);
  }
};


// JSON text as Python's json.dumps(v, ensure_ascii=False, separators=(",", ":")) writes it
void json_write(std::string& o, const JV* v) {
  switch (v->t) {
    case J_NULL: case J_UNDEF: o += "null"; return;
    case J_TRUE: o += "true"; return;
    case J_FALSE: o += "false"; return;
    case J_NUM: {
      char buf[64];
      const double d = v->num;
      if (d == std::floor(d) && std::fabs(d) < 9007199254740992.0) {
        snprintf(buf, sizeof buf, "%lld", (long long)d);
      } else {
        auto r = std::to_chars(buf, buf + sizeof buf, d);
        *r.ptr = 0;
      }
      o += buf;
      return;
    }
    case J_STR: {
      o += '"';
      for (unsigned char c : v->str()) {
        switch (c) {
          case '"': o += "\\\""; break;
          case '\\': o += "\\\\"; break;
          case '\n': o += "\\n"; break;
          case '\r': o += "\\r"; break;
          case '\t': o += "\\t"; break;
          case '\b': o += "\\b"; break;
          case '\f': o += "\\f"; break;
          default:
            if (c < 0x20) {
              char buf[8];
              snprintf(buf, sizeof buf, "\\u%04x", c);
              o += buf;
            } else {
              o += (char)c;
            }
        }
      }
      o += '"';
      return;
    }
    case J_ARR:
      o += '[';
      for (uint32_t k = 0; k < v->n; ++k) {
        if (k) o += ',';
        json_write(o, &v->a[k]);
      }
      o += ']';
      return;
    case J_OBJ:
      o += '{';
      for (uint32_t k = 0; k < v->n; ++k) {
        if (k) o += ',';
        JV key;
        key.t = J_STR;
        key.s = v->o[k].k;
        key.n = v->o[k].kn;
        json_write(o, &key);
        o += ':';
        json_write(o, &v->o[k].v);
      }
      o += '}';
      return;
    default: o += "null"; return;
  }
}

// Combining algorithms (accessController.ts:51-62) and the URN config, URN ids interned first
// in config order (compiler.compile_store).
void configure(Builder& b, const JV* urns, const JV* cas) {
  if (urns->t != J_OBJ) fail("urns: expected a JSON object");
  if (cas->t != J_ARR) fail("combining algorithms: expected a JSON array");
  for (uint32_t k = 0; k < cas->n; ++k) {
    const JV* m = get(&cas->a[k], "method");
    uint8_t code;
    if (m->t == J_STR && m->str() == "denyOverrides") code = CA_DENY_OVERRIDES;
    else if (m->t == J_STR && m->str() == "permitOverrides") code = CA_PERMIT_OVERRIDES;
    else if (m->t == J_STR && m->str() == "firstApplicable") code = CA_FIRST_APPLICABLE;
    else fail("combining algorithm method");
    const JV* u = get(&cas->a[k], "urn");
    std::string key = u->t == J_UNDEF ? "m" : u->t == J_NULL ? "n" : u->t == J_STR ? "s" + std::string(u->str()) : "x";
    bool found = false;
    for (auto& kv : b.ca_map)
      if (kv.first == key) {
        kv.second = code;
        found = true;
      }
    if (!found) b.ca_map.push_back({key, code});
  }
  for (uint32_t k = 0; k < urns->n; ++k) {
    const std::string name(urns->o[k].key());
    const JV* v = &urns->o[k].v;
    if (b.urn.count(name)) {
      b.urn[name] = v;
    } else {
      b.urn.emplace(name, v);
      b.urns.push_back({name, v});
    }
  }
  for (auto& kv : b.urns) b.intern(b.urn[kv.first]);
}

// compiler.mark_clean_below: NF_CLEAN_BELOW on a set when every earlier set is clean
// (NF_COND_FREE, valid combining algorithm, no null policy), NF_CLEAN on a clean set
void mark_clean_below(NodeRec* sets, size_t n_sets, const NodeRec* pols) {
  bool clean_so_far = true;
  for (size_t k = 0; k < n_sets; ++k) {
    NodeRec& S = sets[k];
    if (clean_so_far) S.nflags |= NF_CLEAN_BELOW;
    bool clean = (S.nflags & NF_COND_FREE) && S.ca != CA_INVALID;
    for (uint32_t p = S.child_begin; p < S.child_end && clean; ++p)
      if (pols[p].nflags & NF_NULL) clean = false;
    if (clean) S.nflags |= NF_CLEAN;
    clean_so_far = clean_so_far && clean;
  }
}

// ------------------------------------------------------------------ incremental compile
// One policy set compiled alone: its node records and pools with offsets from 0 (the
// Builder's per-set state while it was compiled), keyed by the set's JSON text.  The
// dictionary, regex rows and evaluation_cacheable table live in the builder and only grow,
// so a fragment's interned ids stay valid across compiles (compiler.IncrementalCompiler).
// A full compile is one fragment holding every set.
struct Fragment {
  uint64_t h1 = 0, h2 = 0;
  size_t len = 0;
  std::vector<NodeRec> sets, pols, rules;
  std::vector<RuleResAttr> rres;
  std::vector<Pair> pairs;
  std::vector<uint32_t> u32pool;
  std::vector<uint8_t> spec_kind[3];
  std::vector<uint32_t> spec_end[3], spec_idx[3];
};

void swap_state(Builder& b, Fragment& f) {
  std::swap(b.sets, f.sets);
  std::swap(b.pols, f.pols);
  std::swap(b.rules, f.rules);
  std::swap(b.rres, f.rres);
  std::swap(b.pairs, f.pairs);
  std::swap(b.u32pool, f.u32pool);
  for (int k = 0; k < 3; ++k) {
    std::swap(b.spec_kind[k], f.spec_kind[k]);
    std::swap(b.spec_end[k], f.spec_end[k]);
    std::swap(b.spec_idx[k], f.spec_idx[k]);
  }
}

// a target's pool offsets (present targets only: an absent one keeps zeros)
void shift_target(NodeRec& R, uint32_t pairs0, uint32_t rres0, uint32_t u320) {
  if (!(R.nflags & NF_HAS_TARGET)) return;
  R.subj_off += pairs0;
  R.act_off += pairs0;
  R.res_off += rres0;
  R.acl_roles_off += u320;
}

size_t a16(size_t x) { return (x + 15) & ~size_t(15); }
size_t a4(size_t x) { return (x + 3) & ~size_t(3); }

// The store image (compiler.store_blob + compiler.codec_section) of the fragments in order,
// written straight into one zeroed allocation: per fragment, its node records with their
// offsets shifted to where they land, its pools and candidate specs (fragments in parallel,
// each at its prefix-sum offsets), then the builder's dictionary / regex rows /
// evaluation_cacheable table.  The caller owns the buffer (acs_blob_free).
void* write_image(Builder& b, const std::vector<const Fragment*>& F, size_t* len_out) {
  const size_t nf = F.size();
  // per-fragment starts (prefix sums), the last entry the total
  struct Off {
    size_t s, p, r, rres, pairs, u32, k[3], i[3];
  };
  std::vector<Off> o(nf + 1);
  o[0] = Off{};
  for (size_t f = 0; f < nf; ++f) {
    const Fragment& x = *F[f];
    Off& n = o[f + 1];
    n = o[f];
    n.s += x.sets.size();
    n.p += x.pols.size();
    n.r += x.rules.size();
    n.rres += x.rres.size();
    n.pairs += x.pairs.size();
    n.u32 += x.u32pool.size();
    for (int q = 0; q < 3; ++q) {
      n.k[q] += x.spec_kind[q].size();
      n.i[q] += x.spec_idx[q].size();
    }
  }
  const Off& T = o[nf];
  if (T.s > UINT32_MAX || T.p > UINT32_MAX || T.r > UINT32_MAX || T.rres > UINT32_MAX || T.pairs > UINT32_MAX ||
      T.u32 > UINT32_MAX)
    fail("store too large");
  // body layout: 64-B header, then 16-B aligned tables and pools
  const size_t o_sets = 64, o_pols = o_sets + a16(T.s * sizeof(NodeRec)), o_rules = o_pols + a16(T.p * sizeof(NodeRec));
  const size_t o_rres = o_rules + a16(T.r * sizeof(NodeRec)), o_pairs = o_rres + a16(T.rres * sizeof(RuleResAttr));
  const size_t o_u32 = o_pairs + a16(T.pairs * sizeof(Pair)), o_sec = o_u32 + a16(T.u32 * 4);
  // codec section: header, urn ids, regex rows, kinds, spec ptr / idx, string offsets + bytes, ec
  std::vector<uint32_t> urn_ids(N_CODEC_URNS);
  for (int k = 0; k < N_CODEC_URNS; ++k) {
    const JV* v = b.U(kCodecUrns[k]);
    urn_ids[k] = v->t == J_STR ? b.intern(v) : ID_UNDEF;
  }
  const JV* user = b.U("user");
  const uint32_t id_user = user->t == J_UNDEF ? ID_UNDEF : b.intern(user);
  const uint32_t n_str2 = (uint32_t)b.strings.size();  // (configure interned every URN value)
  std::vector<uint32_t> offs{0};
  offs.reserve(n_str2 + 1);
  size_t sb = 0;
  for (uint32_t i = 0; i < n_str2; ++i) {
    if (i > ID_EMPTY) sb += b.strings[i].size();
    offs.push_back((uint32_t)sb);
  }
  std::string ecj = "[";
  for (size_t k = 4; k < b.ec.size(); ++k) {
    if (k > 4) ecj += ',';
    ecj += b.ec[k].json;
  }
  ecj += ']';
  const size_t K = T.k[0] + T.k[1] + T.k[2], I = T.i[0] + T.i[1] + T.i[2];
  const size_t c_urn = o_sec + 32, c_rx = c_urn + 4 * (size_t)N_CODEC_URNS, c_kind = c_rx + 4 * b.rx_rows.size();
  const size_t c_ptr = c_kind + a4(K), c_idx = c_ptr + 4 * (K + 1), c_offs = c_idx + 4 * I;
  const size_t c_sb = c_offs + 4 * (size_t)(n_str2 + 1), c_ecn = c_sb + a4(sb), c_ec = c_ecn + 4;
  const size_t total = c_ec + a4(ecj.size());
  if (K > UINT32_MAX || I > UINT32_MAX || sb > UINT32_MAX || total - o_sec > UINT32_MAX || o_sec > UINT32_MAX)
    fail("store too large");
  uint8_t* out = (uint8_t*)blob_alloc_zeroed(total);  // zeroed: the padding
  if (!out) fail("out of memory");
  const uint32_t hdr[16] = {ACS_BLOB_MAGIC, ACS_ABI_VERSION, (uint32_t)T.s, (uint32_t)T.p, (uint32_t)T.r,
                            (uint32_t)T.rres, (uint32_t)T.pairs, (uint32_t)T.u32, id_user, (uint32_t)o_sec,
                            (uint32_t)(total - o_sec), 0, 0, 0, 0, 0};
  memcpy(out, hdr, sizeof hdr);
  const size_t kb[3] = {0, T.k[0], T.k[0] + T.k[1]}, ib[3] = {0, T.i[0], T.i[0] + T.i[1]};
  uint32_t* ptr = (uint32_t*)(out + c_ptr);  // ptr[0] = 0 (zeroed)
  auto write = [&](size_t f0, size_t f1) {
    for (size_t f = f0; f < f1; ++f) {
      const Fragment& x = *F[f];
      const Off& at = o[f];
      const uint32_t P0 = (uint32_t)at.p, R0 = (uint32_t)at.r, RR0 = (uint32_t)at.rres, PA0 = (uint32_t)at.pairs,
                     U0 = (uint32_t)at.u32;
      NodeRec* S = (NodeRec*)(out + o_sets) + at.s;
      for (size_t k = 0; k < x.sets.size(); ++k) {
        NodeRec n = x.sets[k];
        n.child_begin += P0;
        n.child_end += P0;
        shift_target(n, PA0, RR0, U0);
        S[k] = n;
      }
      NodeRec* Pp = (NodeRec*)(out + o_pols) + at.p;
      for (size_t k = 0; k < x.pols.size(); ++k) {
        NodeRec n = x.pols[k];
        n.child_begin += R0;
        n.child_end += R0;
        n.fe += R0;
        shift_target(n, PA0, RR0, U0);
        Pp[k] = n;
      }
      NodeRec* Rr = (NodeRec*)(out + o_rules) + at.r;
      for (size_t k = 0; k < x.rules.size(); ++k) {
        NodeRec n = x.rules[k];
        shift_target(n, PA0, RR0, U0);
        Rr[k] = n;
      }
      if (!x.rres.empty()) memcpy(out + o_rres + at.rres * sizeof(RuleResAttr), x.rres.data(), x.rres.size() * sizeof(RuleResAttr));
      if (!x.pairs.empty()) memcpy(out + o_pairs + at.pairs * sizeof(Pair), x.pairs.data(), x.pairs.size() * sizeof(Pair));
      if (!x.u32pool.empty()) memcpy(out + o_u32 + at.u32 * 4, x.u32pool.data(), x.u32pool.size() * 4);
      for (int q = 0; q < 3; ++q) {
        const size_t k0 = kb[q] + at.k[q], i0 = ib[q] + at.i[q];
        if (!x.spec_kind[q].empty()) memcpy(out + c_kind + k0, x.spec_kind[q].data(), x.spec_kind[q].size());
        for (size_t k = 0; k < x.spec_end[q].size(); ++k) ptr[k0 + k + 1] = (uint32_t)(i0 + x.spec_end[q][k]);
        if (!x.spec_idx[q].empty()) memcpy(out + c_idx + 4 * i0, x.spec_idx[q].data(), x.spec_idx[q].size() * 4);
      }
    }
  };
  // fragments split by node count over the threads
  const size_t nodes = T.s + T.p + T.r;
  int nt = (int)std::min<size_t>(std::max(1u, std::thread::hardware_concurrency()), 16);
  if ((size_t)nt > nodes / 65536 + 1) nt = (int)(nodes / 65536 + 1);
  if ((size_t)nt > nf) nt = (int)(nf ? nf : 1);
  std::vector<size_t> cut(nt + 1, nf);
  cut[0] = 0;
  for (int t = 1; t < nt; ++t) {
    const size_t want = nodes * t / nt;
    size_t f = cut[t - 1];
    while (f < nf && o[f].s + o[f].p + o[f].r < want) ++f;
    cut[t] = f;
  }
  std::vector<std::thread> pool;
  for (int t = 1; t < nt; ++t) pool.emplace_back(write, cut[t], cut[t + 1]);
  write(cut[0], cut[1]);
  for (auto& th : pool) th.join();
  mark_clean_below((NodeRec*)(out + o_sets), T.s, (const NodeRec*)(out + o_pols));
  // codec section (compiler.codec_section)
  const uint32_t hd[8] = {0x43534341u, 2u, n_str2, (uint32_t)N_CODEC_URNS, (uint32_t)b.rx_rows.size(),
                          (uint32_t)K, (uint32_t)I, (uint32_t)sb};
  memcpy(out + o_sec, hd, sizeof hd);
  memcpy(out + c_urn, urn_ids.data(), 4 * urn_ids.size());
  if (!b.rx_rows.empty()) memcpy(out + c_rx, b.rx_rows.data(), 4 * b.rx_rows.size());
  memcpy(out + c_offs, offs.data(), 4 * offs.size());
  uint8_t* w = out + c_sb;
  for (uint32_t i = ID_EMPTY + 1; i < n_str2; ++i) {
    memcpy(w, b.strings[i].data(), b.strings[i].size());
    w += b.strings[i].size();
  }
  const uint32_t ecn = (uint32_t)ecj.size();
  memcpy(out + c_ecn, &ecn, 4);
  memcpy(out + c_ec, ecj.data(), ecj.size());
  *len_out = total;
  return out;
}

// Two independent 64-bit hashes of a set's text in one pass (fragment identity: 128 bits and
// the length).
void text_hash(const char* p, size_t n, uint64_t* h1_out, uint64_t* h2_out) {
  uint64_t h1 = 0x243F6A8885A308D3ull ^ (n * 0x9E3779B97F4A7C15ull), h2 = 0x13198A2E03707344ull ^ n;
  size_t k = 0;
  for (; k + 8 <= n; k += 8) {
    uint64_t w;
    memcpy(&w, p + k, 8);
    h1 = (h1 ^ w) * 0xFF51AFD7ED558CCDull;
    h1 ^= h1 >> 29;
    h2 = (h2 + w) * 0xC4CEB9FE1A85EC53ull;
    h2 ^= h2 >> 31;
  }
  uint64_t w = 0;
  memcpy(&w, p + k, n - k);
  h1 = (h1 ^ w) * 0xC4CEB9FE1A85EC53ull;
  h2 = (h2 + w) * 0xFF51AFD7ED558CCDull;
  *h1_out = h1 ^ (h1 >> 31);
  *h2_out = h2 ^ (h2 >> 29);
}

thread_local std::string g_compile_err;

}  // namespace

struct acs_store_builder {
  std::string urns_text, cas_text;  // the parsed config's bytes (the Builder points into them)
  Arena ar;
  Builder b;
  std::vector<Fragment> frags;      // the last compile's sets, in Map order
  // sets staged for the next compile (acs_store_builder_stage): compiled, or the previous
  // compile's fragment reuse_of with the same text (reserved so two stagings never share one)
  struct Staged {
    Fragment f;
    size_t reuse_of = SIZE_MAX;
  };
  std::vector<Staged> staged;
  std::vector<bool> reserved;       // frags reserved by a staging
  std::unordered_multimap<uint64_t, size_t> by_hash;  // frags by text hash (h1)
};

namespace {

// Compile one set's text into a fragment (the builder's per-set state is empty between
// compiles; the dictionary and regex rows grow).
void compile_fragment(Builder& b, const char* text, size_t len, uint64_t h1, uint64_t h2, Fragment& f) {
  Arena ar;
  Parser p(ar);
  const JV* ps = p.parse(text, text + len);
  swap_state(b, f);
  try {
    b.compile_set(ps);
  } catch (...) {
    swap_state(b, f);
    f = Fragment{};
    throw;
  }
  swap_state(b, f);
  f.h1 = h1;
  f.h2 = h2;
  f.len = len;
}

}  // namespace

extern "C" {

int acs_store_compile(const char* store_json, size_t store_len, const char* urns_json, size_t urns_len,
                      const char* cas_json, size_t cas_len, void** blob_out, size_t* blob_len) {
  if (!store_json || !urns_json || !cas_json || !blob_out || !blob_len) {
    acs_internal_set_error("acs_store_compile: null argument");
    return -1;
  }
  *blob_out = nullptr;
  *blob_len = 0;
  try {
    Arena ar;
    Parser p1(ar), p2(ar), p3(ar);
    const JV* urns = p1.parse(urns_json, urns_json + urns_len);
    const JV* cas = p2.parse(cas_json, cas_json + cas_len);
    const JV* st = p3.parse(store_json, store_json + store_len);
    if (st->t != J_ARR) fail("store: expected a JSON array of policy sets (Map values in order)");
    Builder b;
    configure(b, urns, cas);
    for (uint32_t k = 0; k < st->n; ++k) b.compile_set(&st->a[k]);
    Fragment all;  // every set: one fragment
    swap_state(b, all);
    *blob_out = write_image(b, {&all}, blob_len);
    return 0;
  } catch (const CompileError& e) {
    g_compile_err = "acs_store_compile: " + e.why;
  } catch (const ParseError& e) {
    g_compile_err = std::string("acs_store_compile: ") + e.what;
  }
  acs_internal_set_error(g_compile_err.c_str());
  return -1;
}

void acs_blob_free(void* blob) { blob_release(blob); }

// (internal) zeroed storage for a blob the caller frees with acs_blob_free
void* acs_internal_blob_alloc(size_t n) { return blob_alloc_zeroed(n); }

acs_store_builder* acs_store_builder_create(const char* urns_json, size_t urns_len, const char* cas_json,
                                            size_t cas_len) {
  if (!urns_json || !cas_json) {
    acs_internal_set_error("acs_store_builder_create: null argument");
    return nullptr;
  }
  auto* sb = new acs_store_builder();
  try {
    sb->urns_text.assign(urns_json, urns_len);
    sb->cas_text.assign(cas_json, cas_len);
    Parser p1(sb->ar), p2(sb->ar);
    const JV* urns = p1.parse(sb->urns_text.data(), sb->urns_text.data() + sb->urns_text.size());
    const JV* cas = p2.parse(sb->cas_text.data(), sb->cas_text.data() + sb->cas_text.size());
    configure(sb->b, urns, cas);
    return sb;
  } catch (const CompileError& e) {
    g_compile_err = "acs_store_builder_create: " + e.why;
  } catch (const ParseError& e) {
    g_compile_err = std::string("acs_store_builder_create: ") + e.what;
  }
  acs_internal_set_error(g_compile_err.c_str());
  delete sb;
  return nullptr;
}

void acs_store_builder_free(acs_store_builder* sb) { delete sb; }

long long acs_store_builder_stage(acs_store_builder* sb, const char* set_json, size_t len) {
  if (!sb || !set_json) {
    acs_internal_set_error("acs_store_builder_stage: null argument");
    return -1;
  }
  try {
    uint64_t h1, h2;
    text_hash(set_json, len, &h1, &h2);
    acs_store_builder::Staged st;
    if (sb->reserved.size() != sb->frags.size()) sb->reserved.assign(sb->frags.size(), false);
    auto range = sb->by_hash.equal_range(h1);
    for (auto it = range.first; it != range.second; ++it) {
      const Fragment& f = sb->frags[it->second];
      if (!sb->reserved[it->second] && f.h2 == h2 && f.len == len) {
        st.reuse_of = it->second;
        sb->reserved[it->second] = true;
        break;
      }
    }
    if (st.reuse_of == SIZE_MAX) compile_fragment(sb->b, set_json, len, h1, h2, st.f);
    sb->staged.push_back(std::move(st));
    return (long long)sb->staged.size() - 1;
  } catch (const CompileError& e) {
    g_compile_err = "acs_store_builder_stage: " + e.why;
  } catch (const ParseError& e) {
    g_compile_err = std::string("acs_store_builder_stage: ") + e.what;
  } catch (const std::exception& e) {
    g_compile_err = std::string("acs_store_builder_stage: ") + e.what();
  }
  acs_internal_set_error(g_compile_err.c_str());
  return -1;
}

int acs_store_builder_compile(acs_store_builder* sb, const char* const* sets, const size_t* lens, size_t n,
                              void** blob_out, size_t* blob_len, size_t* recompiled) {
  if (!sb || (n && (!sets || !lens)) || !blob_out || !blob_len) {
    acs_internal_set_error("acs_store_builder_compile: null argument");
    return -1;
  }
  *blob_out = nullptr;
  *blob_len = 0;
  size_t fresh = 0;
  Builder& b = sb->b;
  std::vector<Fragment> next(n);
  std::vector<size_t> from(n, SIZE_MAX);  // next[k] moved out of the previous compile's frags[from[k]]
  try {
    // previous fragments by text hash: an unchanged set is reused as compiled
    std::unordered_multimap<uint64_t, size_t> old;
    for (size_t k = 0; k < sb->frags.size(); ++k) old.emplace(sb->frags[k].h1, k);
    std::vector<bool> taken(sb->frags.size(), false);
    std::vector<size_t> taken_by(sb->frags.size(), SIZE_MAX);  // the slot that holds frags[j] now
    std::vector<bool> staged_used(sb->staged.size(), false);
    // pass 1: the caller's unchanged sets (set k is the previous compile's set lens[k])
    for (size_t k = 0; k < n; ++k) {
      if (sets[k] || (lens[k] & ACS_BUILDER_STAGED)) continue;
      const size_t j = lens[k];
      if (j >= sb->frags.size() || taken[j]) fail("unchanged-set index out of range or repeated");
      next[k] = std::move(sb->frags[j]);
      from[k] = j;
      taken[j] = true;
      taken_by[j] = k;
    }
    // pass 2: staged sets and texts
    for (size_t k = 0; k < n; ++k) {
      if (!sets[k] && !(lens[k] & ACS_BUILDER_STAGED)) continue;
      if (!sets[k]) {  // a staged set
        const size_t h = lens[k] & ~ACS_BUILDER_STAGED;
        if (h >= sb->staged.size() || staged_used[h]) fail("staged-set handle out of range or repeated");
        staged_used[h] = true;
        acs_store_builder::Staged& st = sb->staged[h];
        if (st.reuse_of == SIZE_MAX) {
          next[k] = std::move(st.f);
          ++fresh;
          continue;
        }
        const size_t j = st.reuse_of;
        if (taken[j]) {  // the same text is also an unchanged set: a copy of its fragment
          next[k] = next[taken_by[j]];
          continue;
        }
        next[k] = std::move(sb->frags[j]);
        from[k] = j;
        taken[j] = true;
        taken_by[j] = k;
        continue;
      }
      uint64_t h1, h2;
      text_hash(sets[k], lens[k], &h1, &h2);
      bool reused = false;
      auto range = old.equal_range(h1);
      for (auto it = range.first; it != range.second && !reused; ++it) {
        Fragment& f = sb->frags[it->second];
        if (!taken[it->second] && f.h2 == h2 && f.len == lens[k]) {
          next[k] = std::move(f);
          from[k] = it->second;
          taken[it->second] = true;
          taken_by[it->second] = k;
          reused = true;
        }
      }
      if (reused) continue;
      compile_fragment(b, sets[k], lens[k], h1, h2, next[k]);
      ++fresh;
    }
    std::vector<const Fragment*> parts(n);
    for (size_t k = 0; k < n; ++k) parts[k] = &next[k];
    void* img = write_image(b, parts, blob_len);
    sb->frags = std::move(next);
    sb->staged.clear();
    sb->reserved.assign(sb->frags.size(), false);
    sb->by_hash.clear();
    for (size_t k = 0; k < sb->frags.size(); ++k) sb->by_hash.emplace(sb->frags[k].h1, k);
    if (recompiled) *recompiled = fresh;
    *blob_out = img;
    return 0;
  } catch (const CompileError& e) {
    g_compile_err = "acs_store_builder_compile: " + e.why;
  } catch (const ParseError& e) {
    g_compile_err = std::string("acs_store_builder_compile: ") + e.what;
  } catch (const std::exception& e) {
    g_compile_err = std::string("acs_store_builder_compile: ") + e.what();
  }
  Fragment empty;
  swap_state(b, empty);
  // a failed compile leaves the builder as the last successful one left it: the fragments it
  // moved out go back (the dictionary only grew), so a caller's unchanged-set indices stay valid
  for (size_t k = 0; k < n; ++k)
    if (from[k] != SIZE_MAX) sb->frags[from[k]] = std::move(next[k]);
  sb->staged.clear();  // consumed either way (the caller stages again)
  sb->reserved.assign(sb->frags.size(), false);
  acs_internal_set_error(g_compile_err.c_str());
  return -1;
}

}  // extern "C"
