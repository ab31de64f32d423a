// json_lite.h -- the small JSON reader/writer the HPACK drivers need
// (deflatehd / inflatehd read and write hpack-test-case documents).
//
// The reference tools use jansson (src/deflatehd.cc:42), which this image
// lacks.  This covers what those documents hold: objects with ordered keys,
// arrays, strings, integers, reals, true/false/null.  The writer follows
// jansson's json_dumpf(JSON_INDENT(2) | JSON_PRESERVE_ORDER) layout so the
// drivers print what the reference tools print: two-space indentation,
// "key": value, empty containers as {} / [], reals as %.17g with ".0"
// appended to integral values, and \uXXXX for control bytes.
#pragma once

#include <errno.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <memory>
#include <string>
#include <utility>
#include <vector>

namespace jl {

struct Value;
using Ptr = std::shared_ptr<Value>;

struct Value {
  enum Kind { NUL, BOOL, INT, REAL, STR, ARR, OBJ } kind = NUL;
  bool b = false;
  int64_t i = 0;
  double d = 0;
  std::string s;
  std::vector<Ptr> arr;
  std::vector<std::pair<std::string, Ptr>> obj;  // insertion order

  const Value *get(const char *key) const {
    if (kind != OBJ) return nullptr;
    for (auto &kv : obj)
      if (kv.first == key) return kv.second.get();
    return nullptr;
  }
  void set(const std::string &key, Ptr v) {
    for (auto &kv : obj)
      if (kv.first == key) {
        kv.second = std::move(v);
        return;
      }
    obj.emplace_back(key, std::move(v));
  }
};

inline Ptr make(Value::Kind k) {
  auto v = std::make_shared<Value>();
  v->kind = k;
  return v;
}
inline Ptr integer(int64_t x) {
  auto v = make(Value::INT);
  v->i = x;
  return v;
}
inline Ptr real(double x) {
  auto v = make(Value::REAL);
  v->d = x;
  return v;
}
inline Ptr string(std::string x) {
  auto v = make(Value::STR);
  v->s = std::move(x);
  return v;
}

// ---- reader -------------------------------------------------------------
class Reader {
 public:
  explicit Reader(const std::string &text) : p_(text.data()), e_(text.data() + text.size()) {}

  // Returns nullptr on malformed input (err() says where).
  Ptr parse() {
    Ptr v = value(0);
    ws();
    if (v && p_ != e_) return fail("trailing characters");
    return v;
  }
  const std::string &err() const { return err_; }

 private:
  const char *p_, *e_;
  std::string err_;

  Ptr fail(const char *what) {
    if (err_.empty()) err_ = what;
    return nullptr;
  }
  void ws() {
    while (p_ < e_ && (*p_ == ' ' || *p_ == '\t' || *p_ == '\n' || *p_ == '\r')) ++p_;
  }
  bool lit(const char *w) {
    const size_t n = strlen(w);
    if ((size_t)(e_ - p_) < n || memcmp(p_, w, n) != 0) return false;
    p_ += n;
    return true;
  }
  static void utf8(std::string &o, uint32_t cp) {
    if (cp < 0x80) {
      o.push_back((char)cp);
    } else if (cp < 0x800) {
      o.push_back((char)(0xC0 | (cp >> 6)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    } else if (cp < 0x10000) {
      o.push_back((char)(0xE0 | (cp >> 12)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    } else {
      o.push_back((char)(0xF0 | (cp >> 18)));
      o.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
      o.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
      o.push_back((char)(0x80 | (cp & 0x3F)));
    }
  }
  bool hex4(uint32_t *out) {
    if (e_ - p_ < 4) return false;
    uint32_t v = 0;
    for (int k = 0; k < 4; ++k) {
      const char c = p_[k];
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else return false;
    }
    p_ += 4;
    *out = v;
    return true;
  }
  bool str(std::string &o) {
    ++p_;  // opening quote
    while (p_ < e_ && *p_ != '"') {
      const char c = *p_++;
      if ((unsigned char)c < 0x20) return false;
      if (c != '\\') {
        o.push_back(c);
        continue;
      }
      if (p_ >= e_) return false;
      const char x = *p_++;
      switch (x) {
        case '"': o.push_back('"'); break;
        case '\\': o.push_back('\\'); break;
        case '/': o.push_back('/'); break;
        case 'b': o.push_back('\b'); break;
        case 'f': o.push_back('\f'); break;
        case 'n': o.push_back('\n'); break;
        case 'r': o.push_back('\r'); break;
        case 't': o.push_back('\t'); break;
        case 'u': {
          uint32_t cp;
          if (!hex4(&cp)) return false;
          if (cp >= 0xD800 && cp < 0xDC00) {  // surrogate pair
            uint32_t lo;
            if (!lit("\\u") || !hex4(&lo) || lo < 0xDC00 || lo >= 0xE000) return false;
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          } else if (cp >= 0xDC00 && cp < 0xE000) {
            return false;
          }
          utf8(o, cp);
          break;
        }
        default: return false;
      }
    }
    if (p_ >= e_) return false;
    ++p_;
    return true;
  }
  Ptr number() {
    const char *s = p_;
    if (p_ < e_ && *p_ == '-') ++p_;
    bool isreal = false;
    while (p_ < e_ && ((*p_ >= '0' && *p_ <= '9') || *p_ == '.' || *p_ == 'e' || *p_ == 'E' ||
                       *p_ == '+' || *p_ == '-')) {
      if (*p_ == '.' || *p_ == 'e' || *p_ == 'E') isreal = true;
      ++p_;
    }
    const std::string t(s, p_);
    if (t.empty() || t == "-") return fail("bad number");
    char *end = nullptr;
    if (!isreal) {
      errno = 0;
      const long long x = strtoll(t.c_str(), &end, 10);
      if (*end == '\0' && errno == 0) return integer(x);
    }
    const double d = strtod(t.c_str(), &end);
    if (*end != '\0') return fail("bad number");
    return real(d);
  }
  Ptr value(int depth) {
    if (depth > 512) return fail("too deep");
    ws();
    if (p_ >= e_) return fail("unexpected end");
    const char c = *p_;
    if (c == '{') {
      ++p_;
      auto v = make(Value::OBJ);
      ws();
      if (p_ < e_ && *p_ == '}') {
        ++p_;
        return v;
      }
      for (;;) {
        ws();
        std::string k;
        if (p_ >= e_ || *p_ != '"' || !str(k)) return fail("bad object key");
        ws();
        if (p_ >= e_ || *p_ != ':') return fail("missing ':'");
        ++p_;
        Ptr x = value(depth + 1);
        if (!x) return nullptr;
        v->set(k, x);  // a repeated key keeps its first position, last value
        ws();
        if (p_ < e_ && *p_ == ',') {
          ++p_;
          continue;
        }
        if (p_ < e_ && *p_ == '}') {
          ++p_;
          return v;
        }
        return fail("bad object");
      }
    }
    if (c == '[') {
      ++p_;
      auto v = make(Value::ARR);
      ws();
      if (p_ < e_ && *p_ == ']') {
        ++p_;
        return v;
      }
      for (;;) {
        Ptr x = value(depth + 1);
        if (!x) return nullptr;
        v->arr.push_back(x);
        ws();
        if (p_ < e_ && *p_ == ',') {
          ++p_;
          continue;
        }
        if (p_ < e_ && *p_ == ']') {
          ++p_;
          return v;
        }
        return fail("bad array");
      }
    }
    if (c == '"') {
      auto v = make(Value::STR);
      if (!str(v->s)) return fail("bad string");
      return v;
    }
    if (lit("true")) {
      auto v = make(Value::BOOL);
      v->b = true;
      return v;
    }
    if (lit("false")) return make(Value::BOOL);
    if (lit("null")) return make(Value::NUL);
    return number();
  }
};

// ---- writer (jansson JSON_INDENT(2) | JSON_PRESERVE_ORDER layout) ---------
inline void put_string(std::string &o, const std::string &s) {
  static const char hx[] = "0123456789abcdef";
  o.push_back('"');
  for (unsigned char c : s) {
    switch (c) {
      case '"': o += "\\\""; break;
      case '\\': o += "\\\\"; break;
      case '\b': o += "\\b"; break;
      case '\f': o += "\\f"; break;
      case '\n': o += "\\n"; break;
      case '\r': o += "\\r"; break;
      case '\t': o += "\\t"; break;
      default:
        if (c < 0x20 || c == 0x7F) {
          o += "\\u00";
          o.push_back(hx[c >> 4]);
          o.push_back(hx[c & 15]);
        } else {
          o.push_back((char)c);
        }
    }
  }
  o.push_back('"');
}

inline void put_real(std::string &o, double d) {
  char b[64];
  snprintf(b, sizeof b, "%.17g", d);
  std::string t(b);
  if (t.find_first_of(".eE") == std::string::npos && t != "inf" && t != "-inf" && t != "nan")
    t += ".0";
  o += t;
}

inline void dump(std::string &o, const Value &v, int depth, int indent = 2) {
  auto nl = [&](int d) {
    o.push_back('\n');
    o.append((size_t)(d * indent), ' ');
  };
  switch (v.kind) {
    case Value::NUL: o += "null"; break;
    case Value::BOOL: o += v.b ? "true" : "false"; break;
    case Value::INT: o += std::to_string(v.i); break;
    case Value::REAL: put_real(o, v.d); break;
    case Value::STR: put_string(o, v.s); break;
    case Value::ARR:
      if (v.arr.empty()) {
        o += "[]";
        break;
      }
      o.push_back('[');
      for (size_t k = 0; k < v.arr.size(); ++k) {
        nl(depth + 1);
        dump(o, *v.arr[k], depth + 1, indent);
        if (k + 1 < v.arr.size()) o.push_back(',');
      }
      nl(depth);
      o.push_back(']');
      break;
    case Value::OBJ:
      if (v.obj.empty()) {
        o += "{}";
        break;
      }
      o.push_back('{');
      for (size_t k = 0; k < v.obj.size(); ++k) {
        nl(depth + 1);
        put_string(o, v.obj[k].first);
        o += ": ";
        dump(o, *v.obj[k].second, depth + 1, indent);
        if (k + 1 < v.obj.size()) o.push_back(',');
      }
      nl(depth);
      o.push_back('}');
      break;
  }
}

inline bool read_file(FILE *f, std::string &out) {
  char buf[1 << 16];
  size_t n;
  while ((n = fread(buf, 1, sizeof buf, f)) > 0) out.append(buf, n);
  return !ferror(f);
}

}  // namespace jl
