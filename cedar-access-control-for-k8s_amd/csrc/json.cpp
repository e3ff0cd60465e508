// Minimal JSON reader/writer used by the encoder (Cedar entity/request JSON, SubjectAccessReview
// JSON) and by the diagnostic renderer (Go encoding/json byte-compatible strings, as produced by
// json.Marshal(diagnostic) at internal/server/authorizer/authorizer.go:118).
#include <cerrno>
#include <cstdlib>
#include <cstring>

#include "cedar.h"

namespace cg {

namespace {
struct JP {
  const char* p;
  const char* e;
  [[noreturn]] void fail(const char* m) { throw CedarError(std::string("json: ") + m); }
  void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++; }
  void lit(const char* s) {
    size_t n = std::strlen(s);
    if ((size_t)(e - p) < n || std::memcmp(p, s, n)) fail("bad literal");
    p += n;
  }
  static void put_utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
    else if (cp < 0x10000) { o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
    else { o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
  }
  uint32_t hex4() {
    if (e - p < 4) fail("bad \\u");
    uint32_t v = 0;
    for (int k = 0; k < 4; k++) {
      char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= c - '0';
      else if (c >= 'a' && c <= 'f') v |= c - 'a' + 10;
      else if (c >= 'A' && c <= 'F') v |= c - 'A' + 10;
      else fail("bad hex");
    }
    return v;
  }
  std::string str() {
    if (p >= e || *p != '"') fail("expected string");
    p++;
    std::string o;
    while (p < e && *p != '"') {
      char c = *p++;
      if (c != '\\') { o += c; continue; }
      if (p >= e) fail("bad escape");
      char x = *p++;
      switch (x) {
        case '"': o += '"'; break;
        case '\\': o += '\\'; break;
        case '/': o += '/'; break;
        case 'b': o += '\b'; break;
        case 'f': o += '\f'; break;
        case 'n': o += '\n'; break;
        case 'r': o += '\r'; break;
        case 't': o += '\t'; break;
        case 'u': {
          uint32_t cp = hex4();
          if (cp >= 0xD800 && cp < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
            p += 2;
            uint32_t lo = hex4();
            cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00);
          }
          put_utf8(o, cp);
          break;
        }
        default: fail("bad escape");
      }
    }
    if (p >= e) fail("unterminated string");
    p++;
    return o;
  }
  JVal val(int depth) {
    if (depth > 256) fail("nesting too deep");
    ws();
    if (p >= e) fail("unexpected end");
    JVal v;
    char c = *p;
    if (c == '{') {
      p++;
      v.t = JVal::Obj;
      ws();
      if (p < e && *p == '}') { p++; return v; }
      for (;;) {
        ws();
        std::string k = str();
        ws();
        if (p >= e || *p != ':') fail("expected ':'");
        p++;
        v.obj.emplace_back(std::move(k), val(depth + 1));
        ws();
        if (p < e && *p == ',') { p++; continue; }
        if (p < e && *p == '}') { p++; break; }
        fail("expected ',' or '}'");
      }
      return v;
    }
    if (c == '[') {
      p++;
      v.t = JVal::Arr;
      ws();
      if (p < e && *p == ']') { p++; return v; }
      for (;;) {
        v.arr.push_back(val(depth + 1));
        ws();
        if (p < e && *p == ',') { p++; continue; }
        if (p < e && *p == ']') { p++; break; }
        fail("expected ',' or ']'");
      }
      return v;
    }
    if (c == '"') { v.t = JVal::Str; v.s = str(); return v; }
    if (c == 't') { lit("true"); v.t = JVal::Bool; v.b = true; return v; }
    if (c == 'f') { lit("false"); v.t = JVal::Bool; v.b = false; return v; }
    if (c == 'n') { lit("null"); v.t = JVal::Null; return v; }
    const char* st = p;
    bool isf = false;
    if (p < e && (*p == '-' || *p == '+')) p++;
    while (p < e && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E' || *p == '-' || *p == '+')) {
      if (*p == '.' || *p == 'e' || *p == 'E') isf = true;
      p++;
    }
    if (p == st) fail("unexpected character");
    std::string num(st, p);
    if (isf) { v.t = JVal::Num; v.d = std::stod(num); }
    else {
      v.t = JVal::Int;
      errno = 0;
      char* endp = nullptr;
      long long x = std::strtoll(num.c_str(), &endp, 10);
      if (errno == ERANGE) { v.t = JVal::Num; v.d = std::stod(num); }
      else v.i = x;
    }
    return v;
  }
};
}  // namespace

JVal json_parse(const char* p, size_t n) {
  JP jp{p, p + n};
  JVal v = jp.val(0);
  jp.ws();
  if (jp.p != jp.e) throw CedarError("json: trailing data");
  return v;
}

void go_json_string(std::string& out, const std::string& s) {
  static const char* hex = "0123456789abcdef";
  out += '"';
  for (size_t i = 0; i < s.size(); i++) {
    unsigned char c = (unsigned char)s[i];
    if (c == '"') { out += "\\\""; continue; }
    if (c == '\\') { out += "\\\\"; continue; }
    if (c == '\n') { out += "\\n"; continue; }
    if (c == '\r') { out += "\\r"; continue; }
    if (c == '\t') { out += "\\t"; continue; }
    if (c < 0x20 || c == '<' || c == '>' || c == '&') {
      out += "\\u00"; out += hex[c >> 4]; out += hex[c & 15];
      continue;
    }
    // U+2028 / U+2029 (E2 80 A8 / E2 80 A9)
    if (c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
        ((unsigned char)s[i + 2] == 0xA8 || (unsigned char)s[i + 2] == 0xA9)) {
      out += ((unsigned char)s[i + 2] == 0xA8) ? "\\u2028" : "\\u2029";
      i += 2;
      continue;
    }
    out += (char)c;
  }
  out += '"';
}

void hval_to_json(const HVal& v, std::string& out) {
  switch (v.k) {
    case VK::Bool: out += v.b ? "true" : "false"; return;
    case VK::Long: out += std::to_string(v.i); return;
    case VK::Str: go_json_string(out, v.s); return;
    case VK::Ent:
      out += "{\"__entity\":{\"type\":";
      go_json_string(out, v.etype);
      out += ",\"id\":";
      go_json_string(out, v.s);
      out += "}}";
      return;
    case VK::Set:
      out += '[';
      for (size_t i = 0; i < v.elems.size(); i++) { if (i) out += ','; hval_to_json(v.elems[i], out); }
      out += ']';
      return;
    case VK::Rec:
      out += '{';
      for (size_t i = 0; i < v.fields.size(); i++) {
        if (i) out += ',';
        go_json_string(out, v.fields[i].first);
        out += ':';
        hval_to_json(v.fields[i].second, out);
      }
      out += '}';
      return;
    case VK::Dec: {
      int64_t a = v.i < 0 ? -v.i : v.i;
      std::string f = std::to_string(a % 10000);
      while (f.size() < 4) f = "0" + f;
      out += "{\"__extn\":{\"fn\":\"decimal\",\"arg\":\"" + std::string(v.i < 0 ? "-" : "") + std::to_string(a / 10000) + "." + f + "\"}}";
      return;
    }
    case VK::Ip: {
      std::string s;
      if (!v.ip.v6) {
        for (int k = 0; k < 4; k++) { if (k) s += '.'; s += std::to_string(v.ip.addr[k]); }
      } else {
        static const char* hx = "0123456789abcdef";
        for (int k = 0; k < 8; k++) {
          if (k) s += ':';
          unsigned w = ((unsigned)v.ip.addr[2 * k] << 8) | v.ip.addr[2 * k + 1];
          std::string g;
          do { g = hx[w & 15] + g; w >>= 4; } while (w);
          s += g;
        }
      }
      s += "/" + std::to_string(v.ip.prefix);
      out += "{\"__extn\":{\"fn\":\"ip\",\"arg\":\"" + s + "\"}}";
      return;
    }
  }
}

HVal hval_from_json(const JVal& j) {
  switch (j.t) {
    case JVal::Bool: return HVal::Bool(j.b);
    case JVal::Int: return HVal::Long(j.i);
    case JVal::Str: return HVal::Str(j.s);
    case JVal::Arr: {
      HVal h; h.k = VK::Set;
      for (auto& x : j.arr) {
        HVal e = hval_from_json(x);
        bool dup = false;
        for (auto& y : h.elems) if (hval_eq(e, y)) { dup = true; break; }
        if (!dup) h.elems.push_back(std::move(e));
      }
      return h;
    }
    case JVal::Obj: {
      if (j.obj.size() == 1 && j.obj[0].first == "__entity") {
        const JVal& u = j.obj[0].second;
        return HVal::Ent(u.str_or("type"), u.str_or("id"));
      }
      if (j.obj.size() == 1 && j.obj[0].first == "__extn") {
        const JVal& x = j.obj[0].second;
        std::string fn = x.str_or("fn"), arg = x.str_or("arg");
        HVal h;
        if (fn == "decimal") { h.k = VK::Dec; if (!parse_decimal(arg, &h.i)) throw CedarError("bad decimal " + arg); return h; }
        if (fn == "ip" || fn == "ipaddr") { h.k = VK::Ip; if (!parse_ip(arg, &h.ip)) throw CedarError("bad ip " + arg); return h; }
        throw CedarError("unknown extension " + fn);
      }
      HVal h; h.k = VK::Rec;
      for (auto& kv : j.obj) h.fields.emplace_back(kv.first, hval_from_json(kv.second));
      return h;
    }
    default: throw CedarError("unsupported JSON value in Cedar data (null or float)");
  }
}

}  // namespace cg
