// acs_json.cpp — see acs_json.h.
#include "acs_json.h"

#include <cmath>
#include <cstdlib>

namespace acs_json {

const JV kUndef{};

void* Arena::slow(size_t n, size_t align) {
  // next block (reused after reset) or a new one at least twice the request
  ++cur_;
  while (cur_ < blocks_.size() && cap_[cur_] < n + align) ++cur_;
  if (cur_ >= blocks_.size()) {
    const size_t cap = n + align > (1u << 20) ? n + align : (1u << 20);
    blocks_.emplace_back(new char[cap]);
    cap_.push_back(cap);
    cur_ = blocks_.size() - 1;
  }
  used_ = 0;
  size_t p = (used_ + align - 1) & ~(align - 1);
  used_ = p + n;
  return blocks_[cur_].get() + p;
}

const char* skip_value(const char* p, const char* e) {
  if (p >= e) throw ParseError{"unexpected end"};
  const char c = *p;
  if (c == '"') {
    ++p;
    for (;;) {
      const char* q = (const char*)memchr(p, '"', (size_t)(e - p));
      if (!q) throw ParseError{"unterminated string"};
      // an escaped quote has an odd run of backslashes in front of it
      size_t bs = 0;
      for (const char* b = q - 1; b >= p && *b == '\\'; --b) ++bs;
      p = q + 1;
      if (!(bs & 1)) return p;
    }
  }
  if (c == '{' || c == '[') {
    int depth = 0;
    while (p < e) {
      const char d = *p;
      if (d == '"') {
        p = skip_value(p, e);
        continue;
      }
      if (d == '{' || d == '[') ++depth;
      else if (d == '}' || d == ']') {
        if (--depth == 0) return p + 1;
      }
      ++p;
    }
    throw ParseError{"unterminated container"};
  }
  // literal or number: up to the next delimiter
  while (p < e && *p != ',' && *p != '}' && *p != ']' && *p != ' ' && *p != '\n' && *p != '\r' && *p != '\t') ++p;
  return p;
}

static void utf8(std::string& out, uint32_t c) {
  if (c < 0x80) {
    out += (char)c;
  } else if (c < 0x800) {
    out += (char)(0xC0 | (c >> 6));
    out += (char)(0x80 | (c & 0x3F));
  } else if (c < 0x10000) {  // lone surrogates too (surrogatepass, as the host dictionary encodes them)
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

// The next '"' or '\\' in [p, e): 8 bytes at a time (zero-byte test on the XOR with each
// target byte), then the tail.
static inline const char* find_quote_or_escape(const char* p, const char* e) {
  constexpr uint64_t ONES = 0x0101010101010101ull, HIGH = 0x8080808080808080ull;
  constexpr uint64_t QQ = ONES * (uint8_t)'"', BS = ONES * (uint8_t)'\\';
  while (p + 8 <= e) {
    uint64_t w;
    memcpy(&w, p, 8);
    const uint64_t a = w ^ QQ, b = w ^ BS;
    const uint64_t hit = ((a - ONES) & ~a & HIGH) | ((b - ONES) & ~b & HIGH);
    if (hit) return p + (__builtin_ctzll(hit) >> 3);
    p += 8;
  }
  while (p < e && *p != '"' && *p != '\\') ++p;
  return p;
}

void Parser::string(JV& out) {
  ++p_;  // opening quote
  const char* b = p_;
  bool esc = false;
  for (;;) {
    p_ = find_quote_or_escape(p_, e_);
    if (p_ >= e_) throw ParseError{"unterminated string"};
    if (*p_ == '"') break;
    esc = true;  // a backslash: skip it and the escaped byte
    p_ += 2;
    if (p_ > e_) throw ParseError{"unterminated string"};
  }
  out.t = J_STR;
  if (!esc) {
    out.s = b;
    out.n = (uint32_t)(p_ - b);
    ++p_;
    return;
  }
  std::string tmp;
  for (const char* q = b; q < p_; ++q) {
    if (*q != '\\') {
      tmp += *q;
      continue;
    }
    ++q;
    switch (*q) {
      case '"': tmp += '"'; break;
      case '\\': tmp += '\\'; break;
      case '/': tmp += '/'; break;
      case 'b': tmp += '\b'; break;
      case 'f': tmp += '\f'; break;
      case 'n': tmp += '\n'; break;
      case 'r': tmp += '\r'; break;
      case 't': tmp += '\t'; break;
      case 'u': {
        auto hex4 = [&](const char* h) -> uint32_t {
          if (h + 4 > p_) throw ParseError{"bad \\u escape"};
          uint32_t v = 0;
          for (int k = 0; k < 4; ++k) {
            const char c = h[k];
            v <<= 4;
            if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
            else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
            else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
            else throw ParseError{"bad \\u escape"};
          }
          return v;
        };
        uint32_t c = hex4(q + 1);
        q += 4;
        if (c >= 0xD800 && c < 0xDC00 && q + 6 < p_ && q[1] == '\\' && q[2] == 'u') {
          const uint32_t lo = hex4(q + 3);
          if (lo >= 0xDC00 && lo < 0xE000) {
            c = 0x10000 + ((c - 0xD800) << 10) + (lo - 0xDC00);
            q += 6;
          }
        }
        utf8(tmp, c);
        break;
      }
      default: throw ParseError{"bad escape"};
    }
  }
  char* d = (char*)ar_.alloc(tmp.size() + 1, 1);
  memcpy(d, tmp.data(), tmp.size());
  out.s = d;
  out.n = (uint32_t)tmp.size();
  ++p_;
}

void Parser::value(JV& out) {
  skip_ws();
  if (p_ >= e_) throw ParseError{"unexpected end"};
  const char c = *p_;
  if (c == '{') {
    ++p_;
    const size_t base = kvstack_.size();
    skip_ws();
    if (p_ < e_ && *p_ == '}') {
      ++p_;
    } else {
      for (;;) {
        skip_ws();
        if (p_ >= e_ || *p_ != '"') throw ParseError{"expected member name"};
        JV k;
        string(k);
        skip_ws();
        if (p_ >= e_ || *p_ != ':') throw ParseError{"expected ':'"};
        ++p_;
        JKV kv;
        kv.k = k.s;
        kv.kn = k.n;
        if (!raw_key_.empty() && kv.key() == raw_key_) {
          skip_ws();
          const char* b = p_;
          const char f = b < e_ ? *b : 0;
          p_ = skip_value(p_, e_);
          kv.v.t = J_RAW;
          kv.v.raw = f == '[' ? J_ARR : f == '{' ? J_OBJ : f == '"' ? J_STR : f == 'n' ? J_NULL
                   : f == 't' ? J_TRUE : f == 'f' ? J_FALSE : J_NUM;
          kv.v.s = b;
          kv.v.n = (uint32_t)(p_ - b);
        } else {
          value(kv.v);
        }
        kvstack_.push_back(kv);
        skip_ws();
        if (p_ < e_ && *p_ == ',') {
          ++p_;
          continue;
        }
        if (p_ < e_ && *p_ == '}') {
          ++p_;
          break;
        }
        throw ParseError{"expected ',' or '}'"};
      }
    }
    const size_t m = kvstack_.size() - base;
    JKV* o = (JKV*)ar_.alloc(sizeof(JKV) * (m ? m : 1));
    for (size_t k = 0; k < m; ++k) new (&o[k]) JKV(kvstack_[base + k]);
    kvstack_.resize(base);
    out.t = J_OBJ;
    out.o = o;
    out.n = (uint32_t)m;
    return;
  }
  if (c == '[') {
    ++p_;
    const size_t base = vstack_.size();
    skip_ws();
    if (p_ < e_ && *p_ == ']') {
      ++p_;
    } else {
      for (;;) {
        JV x;
        value(x);
        vstack_.push_back(x);
        skip_ws();
        if (p_ < e_ && *p_ == ',') {
          ++p_;
          continue;
        }
        if (p_ < e_ && *p_ == ']') {
          ++p_;
          break;
        }
        throw ParseError{"expected ',' or ']'"};
      }
    }
    const size_t m = vstack_.size() - base;
    JV* a = (JV*)ar_.alloc(sizeof(JV) * (m ? m : 1));
    for (size_t k = 0; k < m; ++k) new (&a[k]) JV(vstack_[base + k]);
    vstack_.resize(base);
    out.t = J_ARR;
    out.a = a;
    out.n = (uint32_t)m;
    return;
  }
  if (c == '"') {
    string(out);
    return;
  }
  if (e_ - p_ >= 4 && memcmp(p_, "null", 4) == 0) {
    p_ += 4;
    out.t = J_NULL;
    return;
  }
  if (e_ - p_ >= 4 && memcmp(p_, "true", 4) == 0) {
    p_ += 4;
    out.t = J_TRUE;
    return;
  }
  if (e_ - p_ >= 5 && memcmp(p_, "false", 5) == 0) {
    p_ += 5;
    out.t = J_FALSE;
    return;
  }
  const char* b = p_;
  const char* q = skip_value(p_, e_);
  if (q == b || q - b > 63) throw ParseError{"bad number"};
  char buf[64];
  memcpy(buf, b, (size_t)(q - b));
  buf[q - b] = 0;
  char* end = nullptr;
  out.num = strtod(buf, &end);
  if (end != buf + (q - b)) throw ParseError{"bad number"};
  out.t = J_NUM;
  p_ = q;
}

const JV* Parser::parse(const char* p, const char* e, std::string_view raw_key) {
  p_ = p;
  e_ = e;
  raw_key_ = raw_key;
  JV* v = (JV*)ar_.alloc(sizeof(JV));
  new (v) JV();
  value(*v);
  skip_ws();
  if (p_ != e_) throw ParseError{"trailing text"};
  return v;
}

bool truthy(const JV* v) {
  switch (v->t) {
    case J_UNDEF: case J_NULL: case J_FALSE: return false;
    case J_NUM: return v->num == v->num && v->num != 0;
    case J_STR: return v->n != 0;
    case J_RAW:
      if (v->raw == J_NULL || v->raw == J_FALSE) return false;
      if (v->raw == J_STR) return v->n > 2;
      if (v->raw == J_NUM) {
        std::string t(v->s, v->n);
        const double d = strtod(t.c_str(), nullptr);
        return d == d && d != 0;
      }
      return true;
    default: return true;
  }
}

bool is_empty(const JV* v) {
  switch (v->t) {
    case J_STR: case J_ARR: case J_OBJ: return v->n == 0;
    case J_RAW: {
      if (v->raw != J_STR && v->raw != J_ARR && v->raw != J_OBJ) return true;
      if (v->raw == J_STR) return v->n <= 2;
      // [ ws ] / { ws }
      for (uint32_t k = 1; k + 1 < v->n; ++k) {
        const char c = v->s[k];
        if (c != ' ' && c != '\n' && c != '\r' && c != '\t') return false;
      }
      return true;
    }
    default: return true;
  }
}

}  // namespace acs_json
