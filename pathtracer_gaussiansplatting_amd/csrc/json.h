// Minimal JSON DOM for the host-side scene readers (rt-box JSON, scene JSON, glTF 2.0).
// Numbers are kept as double (and whether they were written as integers), strings are UTF-8 with
// \uXXXX escapes (and surrogate pairs) decoded.
#pragma once
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

namespace ptgs {

struct JVal {
  enum Kind { NUL, BOOL, NUM, STR, ARR, OBJ } kind = NUL;
  double num = 0;
  bool is_int = false;
  bool b = false;
  std::string str;
  std::vector<JVal> arr;
  std::map<std::string, JVal> obj;

  const JVal* get(const std::string& k) const {
    if (kind != OBJ) return nullptr;
    auto it = obj.find(k);
    return it == obj.end() ? nullptr : &it->second;
  }
  bool has(const std::string& k) const { return get(k) != nullptr; }
  const JVal* at(size_t i) const { return (kind == ARR && i < arr.size()) ? &arr[i] : nullptr; }
  size_t size() const { return kind == ARR ? arr.size() : (kind == OBJ ? obj.size() : 0); }
  bool is_num() const { return kind == NUM; }
};

inline double jdouble(const JVal* v, double def) { return (v && v->kind == JVal::NUM) ? v->num : def; }
inline float jnum(const JVal* v, float def) { return (v && v->kind == JVal::NUM) ? (float)v->num : def; }
inline int jint(const JVal* v, int def) { return (v && v->kind == JVal::NUM) ? (int)v->num : def; }
inline bool jbool(const JVal* v, bool def) {
  if (!v) return def;
  if (v->kind == JVal::BOOL) return v->b;
  if (v->kind == JVal::NUM) return v->num != 0;
  return def;
}
inline std::string jstr(const JVal* v, const std::string& def) { return (v && v->kind == JVal::STR) ? v->str : def; }

struct JParser {
  const char* p;
  const char* end;
  bool ok = true;
  int depth = 0;

  void ws() {
    while (p < end && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) ++p;
  }
  bool lit(const char* s) {
    size_t n = strlen(s);
    if ((size_t)(end - p) >= n && strncmp(p, s, n) == 0) { p += n; return true; }
    return false;
  }
  static void put_utf8(std::string& s, uint32_t c) {
    if (c < 0x80) s.push_back((char)c);
    else if (c < 0x800) { s.push_back((char)(0xC0 | (c >> 6))); s.push_back((char)(0x80 | (c & 63))); }
    else if (c < 0x10000) {
      s.push_back((char)(0xE0 | (c >> 12))); s.push_back((char)(0x80 | ((c >> 6) & 63)));
      s.push_back((char)(0x80 | (c & 63)));
    } else {
      s.push_back((char)(0xF0 | (c >> 18))); s.push_back((char)(0x80 | ((c >> 12) & 63)));
      s.push_back((char)(0x80 | ((c >> 6) & 63))); s.push_back((char)(0x80 | (c & 63)));
    }
  }
  bool hex4(uint32_t& v) {
    if (end - p < 4) return false;
    v = 0;
    for (int i = 0; i < 4; ++i) {
      char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else return false;
    }
    return true;
  }
  bool string(std::string& out) {
    ++p;  // opening quote
    while (p < end && *p != '"') {
      if (*p != '\\') { out.push_back(*p++); continue; }
      if (++p >= end) return false;
      char e = *p++;
      switch (e) {
        case '"': out.push_back('"'); break;
        case '\\': out.push_back('\\'); break;
        case '/': out.push_back('/'); break;
        case 'b': out.push_back('\b'); break;
        case 'f': out.push_back('\f'); break;
        case 'n': out.push_back('\n'); break;
        case 'r': out.push_back('\r'); break;
        case 't': out.push_back('\t'); break;
        case 'u': {
          uint32_t c;
          if (!hex4(c)) return false;
          if (c >= 0xD800 && c < 0xDC00 && end - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            p += 2;
            uint32_t lo;
            if (!hex4(lo)) return false;
            c = 0x10000 + ((c - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(out, c);
          break;
        }
        default: return false;
      }
    }
    if (p >= end) return false;
    ++p;
    return true;
  }
  JVal parse() {
    JVal v;
    ws();
    if (p >= end || ++depth > 512) { ok = false; return v; }
    if (*p == '{') {
      ++p; v.kind = JVal::OBJ; ws();
      if (p < end && *p == '}') { ++p; --depth; return v; }
      while (ok) {
        ws();
        if (p >= end || *p != '"') { ok = false; break; }
        std::string key;
        if (!string(key)) { ok = false; break; }
        ws();
        if (p >= end || *p != ':') { ok = false; break; }
        ++p;
        v.obj[key] = parse();
        ws();
        if (p < end && *p == ',') { ++p; continue; }
        if (p < end && *p == '}') { ++p; break; }
        ok = false;
      }
    } else if (*p == '[') {
      ++p; v.kind = JVal::ARR; ws();
      if (p < end && *p == ']') { ++p; --depth; return v; }
      while (ok) {
        v.arr.push_back(parse());
        ws();
        if (p < end && *p == ',') { ++p; continue; }
        if (p < end && *p == ']') { ++p; break; }
        ok = false;
      }
    } else if (*p == '"') {
      v.kind = JVal::STR;
      if (!string(v.str)) ok = false;
    } else if (lit("true")) { v.kind = JVal::BOOL; v.b = true; }
    else if (lit("false")) { v.kind = JVal::BOOL; v.b = false; }
    else if (lit("null")) { v.kind = JVal::NUL; }
    else {
      // the number's characters (JSON grammar: sign, digits, '.', exponent), copied into a bounded
      // NUL-terminated buffer: the document itself is not NUL-terminated, strtod must not run past it
      const char* q = p;
      while (q < end && q - p < 63 &&
             ((*q >= '0' && *q <= '9') || *q == '-' || *q == '+' || *q == '.' || *q == 'e' || *q == 'E'))
        ++q;
      char buf[64];
      const size_t len = (size_t)(q - p);
      memcpy(buf, p, len);
      buf[len] = '\0';
      char* e = nullptr;
      v.num = strtod(buf, &e);
      if (e == buf) { ok = false; --depth; return v; }
      v.kind = JVal::NUM;
      v.is_int = true;
      for (const char* c = buf; c < e; ++c)
        if (*c == '.' || *c == 'e' || *c == 'E') v.is_int = false;
      p += e - buf;
    }
    --depth;
    return v;
  }
};

// Parse a whole document; returns false on syntax errors or trailing garbage.
inline bool parse_json(const char* data, size_t size, JVal& out) {
  JParser jp{data, data + size};
  out = jp.parse();
  jp.ws();
  return jp.ok && jp.p == jp.end;
}

}  // namespace ptgs
