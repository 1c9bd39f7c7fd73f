// acs_json.h — the JSON reader of the native request codec (acs_codec.cpp).
//
// Requests arrive as the JSON the reference's handler gets after unmarshallContext
// (src/accessControlService.ts:103-125): JSON.parse semantics, so an absent member is JS
// undefined, `null` is null, a repeated member keeps its last value.  Values are parsed
// into a bump arena that the codec resets per request; strings without escapes point into
// the source text.  One member can be left unparsed: with `raw_key` set, that member's
// value is only delimited (JV::t = J_RAW over the source bytes) — the codec does this for
// `hierarchical_scopes`, whose trees it caches per distinct text instead of re-parsing.
#pragma once
#include <stdint.h>
#include <string.h>

#include <memory>
#include <string>
#include <string_view>
#include <vector>

namespace acs_json {

enum JT : uint8_t { J_UNDEF, J_NULL, J_FALSE, J_TRUE, J_NUM, J_STR, J_ARR, J_OBJ, J_RAW };

struct JKV;
struct JV {  // 16 B: the parse of a 1.2 KB request touches a few hundred of these
  JT t = J_UNDEF;
  JT raw = J_UNDEF;      // J_RAW: the JSON type of the skipped value
  uint32_t n = 0;       // string bytes / array items / object members / raw bytes
  union {
    double num;
    const char* s;   // J_STR / J_RAW bytes
    const JV* a;     // J_ARR items
    const JKV* o;    // J_OBJ members (source order)
  };
  JV() : s(nullptr) {}
  std::string_view str() const { return std::string_view(s, n); }
};
struct JKV {
  const char* k;
  uint32_t kn;
  JV v;
  std::string_view key() const { return std::string_view(k, kn); }
};
static_assert(sizeof(JV) == 16, "JV layout");

extern const JV kUndef;

// Bump allocator: blocks kept across reset() so a steady state allocates nothing.
class Arena {
 public:
  void* alloc(size_t n, size_t align = 8) {
    size_t p = (used_ + align - 1) & ~(align - 1);
    if (cur_ < blocks_.size() && p + n <= cap_[cur_]) {
      used_ = p + n;
      return blocks_[cur_].get() + p;
    }
    return slow(n, align);
  }
  void reset() {
    cur_ = 0;
    used_ = 0;
  }

 private:
  void* slow(size_t n, size_t align);
  std::vector<std::unique_ptr<char[]>> blocks_;
  std::vector<size_t> cap_;
  size_t cur_ = 0, used_ = 0;
};

struct ParseError {
  const char* what;
};

class Parser {
 public:
  Parser(Arena& a) : ar_(a) {}
  // Parse one value from [p, e); `raw_key`: a member name whose value is only delimited.
  const JV* parse(const char* p, const char* e, std::string_view raw_key = {});

 private:
  void value(JV& out);
  void string(JV& out);
  void skip_ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\n' || *p_ == '\r' || *p_ == '\t')) ++p_;
  }
  Arena& ar_;
  const char* p_ = nullptr;
  const char* e_ = nullptr;
  std::string_view raw_key_;
  std::vector<JV> vstack_;
  std::vector<JKV> kvstack_;
};

// End of the JSON value starting at p (first non-space byte), for delimiting top-level
// array items and J_RAW members: strings are skipped escape-aware, brackets counted.
const char* skip_value(const char* p, const char* e);

// Member lookup (last occurrence wins, as JSON.parse keeps it); kUndef when absent or when
// `v` is not an object.
inline const JV* get(const JV* v, std::string_view key) {
  if (v->t != J_OBJ) return &kUndef;
  const JV* hit = &kUndef;
  const size_t kn = key.size();
  for (uint32_t k = 0; k < v->n; ++k) {
    const JKV& m = v->o[k];
    if (m.kn == kn && (kn == 0 || (m.k[0] == key[0] && memcmp(m.k, key.data(), kn) == 0))) hit = &m.v;
  }
  return hit;
}

inline bool nullish(const JV* v) { return v->t == J_UNDEF || v->t == J_NULL; }
bool truthy(const JV* v);
bool is_empty(const JV* v);  // lodash isEmpty for JSON values

}  // namespace acs_json
