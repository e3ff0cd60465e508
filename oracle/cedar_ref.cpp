// cedar_ref — C++ restatement of Cedar authorization (cedar-go v1.1.0 semantics) for the
// cedar-access-control-for-k8s hot path. TEST INFRASTRUCTURE ONLY.
//
// Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library, and
// only as the checker / the CPU baseline ("kind": "port"). The product (libcedargpu.so) never
// links it. It shares no code with the product: its own JSON reader, Cedar lexer/parser, value
// model and tree-walking evaluator, written from the Cedar language semantics and the reference's
// call sites:
//   internal/server/store/store.go:25-42   TieredPolicyStores.IsAuthorized (tier walk, fall-through
//                                           only on Deny with no reasons and no errors)
//   internal/server/store/store.go:31      (*cedar.PolicySet).IsAuthorized: every policy evaluated,
//                                           erroring policies skipped and reported, forbid overrides
//                                           permit, default deny
//   internal/server/store/memory.go:17-27  cedar.NewPolicySetFromBytes: IDs policy<i>
//   internal/server/store/directory.go:76, crd.go:60, verified_permissions.go:95: ID conventions
//   internal/server/authorizer/authorizer.go:113-124  json.Marshal(cedar.Diagnostic) (omitempty)
//   internal/server/admission/handler.go:64-66        json.Marshal(diagnostic.Reasons)
// It mirrors oracle/cedar_oracle.py (the readable restatement, pinned against the reference's
// TestAuthorize / TestTieredIsAuthorized vectors in tests/golden) operation for operation,
// including the (parity-unpinned) error message texts, and is cross-checked against it by
// tests/test_oracle_cxx.py.
//
// Like cedar-go, evaluation is a per-request linear scan over every policy of a tier with a
// tree-walking evaluator and hash-map entity lookups keyed by (type, id) strings. The CPU baseline
// runs it on N host threads over disjoint shards of pre-built (EntityMap, Request) items.
#include <arpa/inet.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <functional>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <unordered_map>
#include <string_view>
#include <vector>

namespace cref {

// ------------------------------------------------------------------------------------------------
// Values. Scalars inline; strings point at storage that outlives the evaluation (policy ASTs,
// entity data, or the per-request arena); sets/records are arena- or item-owned aggregates.
// ------------------------------------------------------------------------------------------------
enum class VT : uint8_t { Bool, Long, Str, Ent, Set, Rec, Dec, IP };

struct Agg;
struct IPv {
  uint8_t v6 = 0, prefix = 0;
  uint8_t a[16] = {0};
};
struct Val {
  VT t = VT::Bool;
  int64_t i = 0;                // bool / long / decimal
  const std::string* s = nullptr;   // string / entity id
  const std::string* et = nullptr;  // entity type
  const Agg* agg = nullptr;         // set / record
  const IPv* ip = nullptr;
};
struct Agg {
  std::vector<Val> el;                                       // set elements (deduplicated)
  std::vector<std::pair<const std::string*, Val>> fields;    // record fields sorted by key
};

bool veq(const Val& a, const Val& b);

bool ip_eq(const IPv& x, const IPv& y) { return x.v6 == y.v6 && x.prefix == y.prefix && memcmp(x.a, y.a, 16) == 0; }

bool veq(const Val& a, const Val& b) {
  if (a.t != b.t) return false;
  switch (a.t) {
    case VT::Bool:
    case VT::Long:
    case VT::Dec: return a.i == b.i;
    case VT::Str: return *a.s == *b.s;
    case VT::Ent: return *a.et == *b.et && *a.s == *b.s;
    case VT::IP: return ip_eq(*a.ip, *b.ip);
    case VT::Set: {
      const auto& x = a.agg->el;
      const auto& y = b.agg->el;
      if (x.size() != y.size()) return false;  // both deduplicated
      for (auto& e : x) {
        bool f = false;
        for (auto& g : y) if (veq(e, g)) { f = true; break; }
        if (!f) return false;
      }
      return true;
    }
    case VT::Rec: {
      const auto& x = a.agg->fields;
      const auto& y = b.agg->fields;
      if (x.size() != y.size()) return false;
      for (size_t k = 0; k < x.size(); k++)
        if (*x[k].first != *y[k].first || !veq(x[k].second, y[k].second)) return false;
      return true;
    }
  }
  return false;
}

const char* type_name(const Val& v) {
  switch (v.t) {
    case VT::Bool: return "bool";
    case VT::Long: return "long";
    case VT::Str: return "string";
    case VT::Ent: return "entity";
    case VT::Set: return "set";
    case VT::Rec: return "record";
    case VT::Dec: return "decimal";
    case VT::IP: return "IP";
  }
  return "unknown";
}

// Storage for values built while evaluating (one per request on one thread).
struct Arena {
  std::vector<std::unique_ptr<Agg>> aggs;
  std::vector<std::unique_ptr<std::string>> strs;
  std::vector<std::unique_ptr<IPv>> ips;
  Agg* agg() { aggs.emplace_back(new Agg()); return aggs.back().get(); }
  const std::string* str(std::string s) { strs.emplace_back(new std::string(std::move(s))); return strs.back().get(); }
  const IPv* ip(const IPv& x) { ips.emplace_back(new IPv(x)); return ips.back().get(); }
  void clear() { aggs.clear(); strs.clear(); ips.clear(); }
};

void set_add(Agg* a, const Val& v) {
  for (auto& e : a->el) if (veq(e, v)) return;
  a->el.push_back(v);
}
void rec_sort(Agg* a) {
  std::sort(a->fields.begin(), a->fields.end(), [](auto& x, auto& y) { return *x.first < *y.first; });
}
const Val* rec_get(const Agg* a, const std::string& k) {
  for (auto& f : a->fields) if (*f.first == k) return &f.second;
  return nullptr;
}

struct EvalError {
  std::string msg;
};
[[noreturn]] void type_error(const char* expected, const Val& got) {
  throw EvalError{std::string("type error: expected ") + expected + ", got " + type_name(got)};
}

std::string go_quote(const std::string& s) {
  std::string o = "\"";
  for (char c : s) {
    if (c == '\\' || c == '"') o += '\\';
    o += c;
  }
  return o + "\"";
}
std::string uid_str(const Val& v) { return *v.et + "::" + go_quote(*v.s); }

// Go encoding/json string (HTML-escaped <, >, &, U+2028/2029; control characters \u00XX).
void go_json_string(const std::string& s, std::string& o) {
  static const char* hex = "0123456789abcdef";
  o += '"';
  for (size_t i = 0; i < s.size(); i++) {
    unsigned char c = (unsigned char)s[i];
    if (c == '"') o += "\\\"";
    else if (c == '\\') o += "\\\\";
    else if (c == '\n') o += "\\n";
    else if (c == '\r') o += "\\r";
    else if (c == '\t') o += "\\t";
    else if (c < 0x20 || c == '<' || c == '>' || c == '&') {
      o += "\\u00"; o += hex[c >> 4]; o += hex[c & 15];
    } else if (c == 0xE2 && i + 2 < s.size() && (unsigned char)s[i + 1] == 0x80 &&
               ((unsigned char)s[i + 2] == 0xA8 || (unsigned char)s[i + 2] == 0xA9)) {
      o += (unsigned char)s[i + 2] == 0xA8 ? "\\u2028" : "\\u2029";
      i += 2;
    } else {
      o += (char)c;
    }
  }
  o += '"';
}

// ------------------------------------------------------------------------------------------------
// Extension parsing (decimal, ip) — Cedar decimal: <=4 fractional digits, int64 range;
// ip: dotted quad (no leading zeros) or RFC 4291 text, optional /prefix.
// ------------------------------------------------------------------------------------------------
bool all_digits(const std::string& s) {
  if (s.empty()) return false;
  for (char c : s) if (c < '0' || c > '9') return false;
  return true;
}

int64_t parse_decimal(const std::string& s) {
  auto bad = [&]() { return EvalError{"error parsing decimal value: " + s}; };
  bool neg = !s.empty() && s[0] == '-';
  std::string body = neg ? s.substr(1) : s;
  size_t dot = body.find('.');
  if (dot == std::string::npos) throw bad();
  std::string ip = body.substr(0, dot), fp = body.substr(dot + 1);
  if (!all_digits(ip) || !all_digits(fp) || fp.size() > 4) throw bad();
  while (fp.size() < 4) fp += '0';
  // |value| <= 2^63 (the negative side reaches INT64_MIN)
  unsigned __int128 v = 0;
  for (char c : ip) {
    v = v * 10 + (unsigned)(c - '0');
    if (v > ((unsigned __int128)1 << 64)) throw bad();
  }
  v = v * 10000 + (unsigned)std::stoul(fp);
  const unsigned __int128 lim = neg ? ((unsigned __int128)1 << 63) : (((unsigned __int128)1 << 63) - 1);
  if (v > lim) throw bad();
  return neg ? (int64_t)(-(__int128)v) : (int64_t)v;
}

bool parse_v4(const std::string& s, uint8_t* out) {
  int part = 0;
  size_t i = 0;
  while (part < 4) {
    size_t j = i;
    while (j < s.size() && s[j] >= '0' && s[j] <= '9') j++;
    if (j == i || j - i > 3) return false;
    if (j - i > 1 && s[i] == '0') return false;
    int v = std::stoi(s.substr(i, j - i));
    if (v > 255) return false;
    out[part++] = (uint8_t)v;
    if (part < 4) {
      if (j >= s.size() || s[j] != '.') return false;
      i = j + 1;
    } else if (j != s.size()) {
      return false;
    }
  }
  return true;
}

IPv parse_ip(const std::string& s) {
  auto bad = [&]() { return EvalError{"error parsing ip value: " + s}; };
  std::string addr = s, pre;
  size_t slash = s.find('/');
  if (slash != std::string::npos) { addr = s.substr(0, slash); pre = s.substr(slash + 1); }
  IPv r;
  if (addr.find(':') != std::string::npos) {
    r.v6 = 1;
    if (inet_pton(AF_INET6, addr.c_str(), r.a) != 1) throw bad();
  } else {
    if (!parse_v4(addr, r.a)) throw bad();
  }
  const int maxp = r.v6 ? 128 : 32;
  if (slash != std::string::npos) {
    if (pre.empty() || !all_digits(pre) || pre.size() > 3 || (pre.size() > 1 && pre[0] == '0')) throw bad();
    int p = std::stoi(pre);
    if (p > maxp) throw bad();
    r.prefix = (uint8_t)p;
  } else {
    r.prefix = (uint8_t)maxp;
  }
  return r;
}

// network bytes of an interface (host bits cleared)
void ip_network(const IPv& x, uint8_t* net) {
  const int n = x.v6 ? 16 : 4;
  for (int k = 0; k < n; k++) {
    int bits = (int)x.prefix - 8 * k;
    uint8_t m = bits >= 8 ? 0xFF : bits <= 0 ? 0 : (uint8_t)(0xFF << (8 - bits));
    net[k] = x.a[k] & m;
  }
}

// ------------------------------------------------------------------------------------------------
// JSON reader (items, entities, values)
// ------------------------------------------------------------------------------------------------
struct J {
  enum K { Null, Bool, Num, Str, Arr, Obj } k = Null;
  bool b = false;
  std::string s;  // string, or number text
  std::vector<J> a;
  std::vector<std::pair<std::string, J>> o;
  const J* get(const char* key) const {
    for (auto& kv : o) if (kv.first == key) return &kv.second;
    return nullptr;
  }
};

struct JParser {
  const char* p;
  const char* e;
  [[noreturn]] void fail(const char* what) { throw std::runtime_error(std::string("json: ") + what); }
  void ws() { while (p < e && (*p == ' ' || *p == '\n' || *p == '\r' || *p == '\t')) p++; }
  static void utf8(std::string& o, uint32_t cp) {
    if (cp < 0x80) o += (char)cp;
    else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 63)); }
    else if (cp < 0x10000) { o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 63)); o += (char)(0x80 | (cp & 63)); }
    else { o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 63)); o += (char)(0x80 | ((cp >> 6) & 63)); o += (char)(0x80 | (cp & 63)); }
  }
  uint32_t hex4() {
    if (e - p < 4) fail("bad \\u");
    uint32_t v = 0;
    for (int k = 0; k < 4; k++) {
      char c = *p++;
      v <<= 4;
      if (c >= '0' && c <= '9') v |= (uint32_t)(c - '0');
      else if (c >= 'a' && c <= 'f') v |= (uint32_t)(c - 'a' + 10);
      else if (c >= 'A' && c <= 'F') v |= (uint32_t)(c - 'A' + 10);
      else fail("bad hex");
    }
    return v;
  }
  std::string str() {
    if (p >= e || *p != '"') fail("expected string");
    p++;
    std::string o;
    while (p < e && *p != '"') {
      if (*p == '\\') {
        p++;
        if (p >= e) fail("bad escape");
        char c = *p++;
        switch (c) {
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
            utf8(o, cp);
            break;
          }
          default: fail("bad escape");
        }
      } else {
        o += *p++;
      }
    }
    if (p >= e) fail("unterminated string");
    p++;
    return o;
  }
  J val() {
    ws();
    if (p >= e) fail("unexpected end");
    J j;
    char c = *p;
    if (c == '{') {
      j.k = J::Obj;
      p++;
      ws();
      if (p < e && *p == '}') { p++; return j; }
      for (;;) {
        ws();
        std::string k = str();
        ws();
        if (p >= e || *p != ':') fail("expected :");
        p++;
        j.o.emplace_back(std::move(k), val());
        ws();
        if (p < e && *p == ',') { p++; continue; }
        if (p < e && *p == '}') { p++; return j; }
        fail("expected , or }");
      }
    }
    if (c == '[') {
      j.k = J::Arr;
      p++;
      ws();
      if (p < e && *p == ']') { p++; return j; }
      for (;;) {
        j.a.push_back(val());
        ws();
        if (p < e && *p == ',') { p++; continue; }
        if (p < e && *p == ']') { p++; return j; }
        fail("expected , or ]");
      }
    }
    if (c == '"') { j.k = J::Str; j.s = str(); return j; }
    if (e - p >= 4 && !strncmp(p, "true", 4)) { j.k = J::Bool; j.b = true; p += 4; return j; }
    if (e - p >= 5 && !strncmp(p, "false", 5)) { j.k = J::Bool; j.b = false; p += 5; return j; }
    if (e - p >= 4 && !strncmp(p, "null", 4)) { p += 4; return j; }
    if (c == '-' || (c >= '0' && c <= '9')) {
      const char* s0 = p;
      p++;
      while (p < e && ((*p >= '0' && *p <= '9') || *p == '.' || *p == 'e' || *p == 'E' || *p == '+' || *p == '-')) p++;
      j.k = J::Num;
      j.s.assign(s0, p);
      return j;
    }
    fail("unexpected character");
  }
};

J parse_json(const char* s, size_t n) {
  JParser jp{s, s + n};
  J v = jp.val();
  jp.ws();
  if (jp.p != jp.e) jp.fail("trailing data");
  return v;
}

// ------------------------------------------------------------------------------------------------
// Entities and requests (owned per item; values point into the item's storage)
// ------------------------------------------------------------------------------------------------
struct UidKey {
  std::string type, id;
};
// (type, id) views into storage that outlives the map (the item's arena); hashed like Go's map key
struct KV {
  std::string_view t, i;
  bool operator==(const KV& o) const { return t == o.t && i == o.i; }
};
struct KVHash {
  size_t operator()(const KV& k) const {
    return std::hash<std::string_view>()(k.t) * 1000003u ^ std::hash<std::string_view>()(k.i);
  }
};

struct Entity {
  Val attrs;  // record
  std::vector<KV> parents;
};

struct Item {
  Arena store;  // owns attribute values and UID strings
  std::unordered_map<KV, Entity, KVHash> ents;
  Val principal, action, resource, context;
};

Val value_from_json(const J& j, Arena& A);

Val mk_ent(Arena& A, const std::string& type, const std::string& id) {
  Val v;
  v.t = VT::Ent;
  v.et = A.str(type);
  v.s = A.str(id);
  return v;
}

UidKey uid_from_json(const J& j0) {
  const J* j = &j0;
  if (const J* x = j->get("__entity")) j = x;
  const J* t = j->get("type");
  const J* i = j->get("id");
  if (!t || !i || t->k != J::Str || i->k != J::Str) throw std::runtime_error("bad entity uid");
  return UidKey{t->s, i->s};
}

Val value_from_json(const J& j, Arena& A) {
  Val v;
  switch (j.k) {
    case J::Bool: v.t = VT::Bool; v.i = j.b; return v;
    case J::Num: v.t = VT::Long; v.i = std::stoll(j.s); return v;
    case J::Str: v.t = VT::Str; v.s = A.str(j.s); return v;
    case J::Arr: {
      Agg* a = A.agg();
      for (auto& x : j.a) set_add(a, value_from_json(x, A));
      v.t = VT::Set; v.agg = a;
      return v;
    }
    case J::Obj: {
      if (j.o.size() == 1 && j.o[0].first == "__entity") {
        UidKey u = uid_from_json(j.o[0].second);
        return mk_ent(A, u.type, u.id);
      }
      if (j.o.size() == 1 && j.o[0].first == "__extn") {
        const J* fn = j.o[0].second.get("fn");
        const J* arg = j.o[0].second.get("arg");
        if (!fn || !arg) throw std::runtime_error("bad __extn");
        if (fn->s == "decimal") { v.t = VT::Dec; v.i = parse_decimal(arg->s); return v; }
        v.t = VT::IP; v.ip = A.ip(parse_ip(arg->s));
        return v;
      }
      Agg* a = A.agg();
      for (auto& kv : j.o) {
        const std::string* k = A.str(kv.first);
        Val x = value_from_json(kv.second, A);
        bool dup = false;
        for (auto& f : a->fields) if (*f.first == *k) { f.second = x; dup = true; }
        if (!dup) a->fields.emplace_back(k, x);
      }
      rec_sort(a);
      v.t = VT::Rec; v.agg = a;
      return v;
    }
    default: throw std::runtime_error("bad value json");
  }
}

void item_from_json(const J& j, Item& it) {
  Arena& A = it.store;
  const J* ents = j.get("entities");
  if (ents && ents->k == J::Arr) {
    for (auto& e : ents->a) {
      UidKey u = uid_from_json(*e.get("uid"));
      Entity en;
      const J* at = e.get("attrs");
      if (at) en.attrs = value_from_json(*at, A);
      else { en.attrs.t = VT::Rec; en.attrs.agg = A.agg(); }
      if (const J* ps = e.get("parents"))
        for (auto& p : ps->a) {
          UidKey q = uid_from_json(p);
          en.parents.push_back(KV{*A.str(q.type), *A.str(q.id)});
        }
      it.ents[KV{*A.str(u.type), *A.str(u.id)}] = std::move(en);
    }
  }
  const J* r = j.get("request");
  if (!r) throw std::runtime_error("item without request");
  UidKey p = uid_from_json(*r->get("principal")), a = uid_from_json(*r->get("action")),
         s = uid_from_json(*r->get("resource"));
  it.principal = mk_ent(A, p.type, p.id);
  it.action = mk_ent(A, a.type, a.id);
  it.resource = mk_ent(A, s.type, s.id);
  if (const J* c = r->get("context")) it.context = value_from_json(*c, A);
  else { it.context.t = VT::Rec; it.context.agg = A.agg(); }
}

// ------------------------------------------------------------------------------------------------
// Cedar policy text: lexer, AST, parser
// ------------------------------------------------------------------------------------------------
enum class TK { Ident, Str, Int, Op, Eof };
struct Tok {
  TK k;
  std::string text;  // raw (strings: without quotes, unescaped later)
  int offset, line, col;
};

struct ParseError {
  std::string msg;
};

std::vector<Tok> tokenize(const std::string& src) {
  std::vector<Tok> out;
  size_t i = 0, n = src.size();
  int line = 1, col = 1;
  auto adv = [&](size_t k) {
    for (size_t q = 0; q < k; q++) {
      unsigned char c = (unsigned char)src[i];
      // columns count characters: UTF-8 continuation bytes do not advance the column
      if (c == '\n') { line++; col = 1; }
      else if ((c & 0xC0) != 0x80) col++;
      i++;
    }
  };
  auto is_alpha = [](unsigned char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || c == '_'; };
  auto is_digit = [](unsigned char c) { return c >= '0' && c <= '9'; };
  while (i < n) {
    unsigned char c = (unsigned char)src[i];
    if (c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\f' || c == '\v') { adv(1); continue; }
    if (c == '/' && i + 1 < n && src[i + 1] == '/') {
      while (i < n && src[i] != '\n') adv(1);
      continue;
    }
    Tok t{TK::Op, "", (int)i, line, col};
    if (is_alpha(c)) {
      size_t j = i;
      while (j < n && (is_alpha((unsigned char)src[j]) || is_digit((unsigned char)src[j]))) j++;
      t.k = TK::Ident; t.text = src.substr(i, j - i);
      adv(j - i);
      out.push_back(t);
      continue;
    }
    if (is_digit(c)) {
      size_t j = i;
      while (j < n && is_digit((unsigned char)src[j])) j++;
      t.k = TK::Int; t.text = src.substr(i, j - i);
      adv(j - i);
      out.push_back(t);
      continue;
    }
    if (c == '"') {
      size_t j = i + 1;
      while (j < n && src[j] != '"') {
        if (src[j] == '\\') j++;
        j++;
      }
      if (j >= n) throw ParseError{"unterminated string at line " + std::to_string(line)};
      t.k = TK::Str; t.text = src.substr(i + 1, j - i - 1);
      adv(j + 1 - i);
      out.push_back(t);
      continue;
    }
    static const char* ops2[] = {"==", "!=", "<=", ">=", "&&", "||", "::"};
    bool two = false;
    for (auto o : ops2)
      if (i + 1 < n && src[i] == o[0] && src[i + 1] == o[1]) { t.text = o; two = true; break; }
    if (two) { adv(2); out.push_back(t); continue; }
    if (strchr("()[]{},;.@<>!+-*:", (int)c) && c != 0) {
      t.text = std::string(1, (char)c);
      adv(1);
      out.push_back(t);
      continue;
    }
    throw ParseError{"unexpected character at line " + std::to_string(line) + " column " + std::to_string(col)};
  }
  out.push_back(Tok{TK::Eof, "", (int)i, line, col});
  return out;
}

void put_utf8(std::string& o, uint32_t cp) { JParser::utf8(o, cp); }

// Cedar string escapes. pattern=true: returns pieces (lit / star) in `pieces`.
struct Piece {
  bool star;
  std::string lit;
};
std::string unescape(const std::string& raw, bool pattern, std::vector<Piece>* pieces) {
  std::string lit;
  size_t i = 0;
  while (i < raw.size()) {
    char ch = raw[i];
    if (ch == '\\') {
      i++;
      if (i >= raw.size()) throw ParseError{"bad escape"};
      char e = raw[i];
      switch (e) {
        case 'n': lit += '\n'; break;
        case 'r': lit += '\r'; break;
        case 't': lit += '\t'; break;
        case '\\': lit += '\\'; break;
        case '0': lit += '\0'; break;
        case '\'': lit += '\''; break;
        case '"': lit += '"'; break;
        case 'x': {
          std::string h = raw.substr(i + 1, 2);
          if (h.size() != 2 || !isxdigit((unsigned char)h[0]) || !isxdigit((unsigned char)h[1])) throw ParseError{"bad \\x escape"};
          int v = std::stoi(h, nullptr, 16);
          if (v > 0x7F) throw ParseError{"bad \\x escape"};
          lit += (char)v;
          i += 2;
          break;
        }
        case 'u': {
          if (i + 1 >= raw.size() || raw[i + 1] != '{') throw ParseError{"bad \\u escape"};
          size_t j = raw.find('}', i);
          if (j == std::string::npos) throw ParseError{"bad \\u escape"};
          put_utf8(lit, (uint32_t)std::stoul(raw.substr(i + 2, j - i - 2), nullptr, 16));
          i = j;
          break;
        }
        case '*':
          if (pattern) { lit += '*'; break; }
          throw ParseError{"bad escape \\*"};
        default: throw ParseError{std::string("bad escape \\") + e};
      }
      i++;
      continue;
    }
    if (ch == '*' && pattern) {
      if (!lit.empty()) { pieces->push_back(Piece{false, lit}); lit.clear(); }
      pieces->push_back(Piece{true, ""});
      i++;
      continue;
    }
    lit += ch;
    i++;
  }
  if (pattern && !lit.empty()) pieces->push_back(Piece{false, lit});
  return lit;
}

enum class EK { Lit, Var, And, Or, Not, Neg, If, Bin, Has, Attr, Like, Is, Set, Rec, Call, Method };
enum class Bin { Eq, Ne, Lt, Le, Gt, Ge, Add, Sub, Mul, In };
struct Expr {
  EK k;
  Bin op = Bin::Eq;
  int var = 0;              // 0 principal 1 action 2 resource 3 context
  std::string name;         // attr key / has key / is type / call or method name
  Val lit;                  // literal (strings point into `strs`)
  std::vector<Piece> pat;   // like
  std::vector<std::unique_ptr<Expr>> kids;
  std::vector<std::string> keys;  // record literal keys
  std::vector<std::unique_ptr<std::string>> strs;  // literal string storage
  bool has_in = false;      // is ... in
};
using EP = std::unique_ptr<Expr>;

enum class SK { Any, Eq, In, Is, IsIn, InSet };
struct Uid {
  std::string type, id;
};
struct Scope {
  SK k = SK::Any;
  std::string etype;
  Uid ent;
  std::vector<Uid> ents;
};

struct Policy {
  bool forbid = false;
  Scope p, a, r;
  std::vector<std::pair<bool, EP>> conds;  // (is_when, expr)
  int offset = 0, line = 0, col = 0;
  std::string filename, id;
};

EP mk(EK k) { EP e(new Expr()); e->k = k; return e; }

struct Parser {
  std::vector<Tok> t;
  size_t i = 0;
  std::string filename;
  const Tok& peek(size_t k = 0) const { return t[std::min(i + k, t.size() - 1)]; }
  const Tok& next() { return t[i++]; }
  bool is_op(const char* s, size_t k = 0) const { const Tok& x = peek(k); return x.k == TK::Op && x.text == s; }
  bool is_kw(const char* s, size_t k = 0) const { const Tok& x = peek(k); return x.k == TK::Ident && x.text == s; }
  void expect(const char* s) {
    const Tok& x = next();
    if (x.text != s || (x.k != TK::Op && x.k != TK::Ident))
      throw ParseError{filename + ":" + std::to_string(x.line) + ":" + std::to_string(x.col) + ": expected '" + s + "', got '" + x.text + "'"};
  }

  std::vector<Policy> policies() {
    std::vector<Policy> out;
    while (peek().k != TK::Eof) out.push_back(policy());
    return out;
  }
  Policy policy() {
    const Tok first = peek();
    std::vector<std::string> seen;
    while (is_op("@")) {
      next();
      const Tok& nm = next();
      if (nm.k != TK::Ident) throw ParseError{"bad annotation"};
      if (is_op("(")) {
        next();
        const Tok& s = next();
        if (s.k != TK::Str) throw ParseError{"annotation value must be a string"};
        unescape(s.text, false, nullptr);
        expect(")");
      }
      if (std::find(seen.begin(), seen.end(), nm.text) != seen.end()) throw ParseError{"duplicate annotation @" + nm.text};
      seen.push_back(nm.text);
    }
    const Tok& eff = next();
    if (eff.k != TK::Ident || (eff.text != "permit" && eff.text != "forbid"))
      throw ParseError{filename + ": expected permit or forbid, got '" + eff.text + "'"};
    Policy p;
    p.forbid = eff.text == "forbid";
    expect("(");
    p.p = scope("principal");
    expect(",");
    p.a = action_scope();
    expect(",");
    p.r = scope("resource");
    expect(")");
    while (is_kw("when") || is_kw("unless")) {
      bool when = next().text == "when";
      expect("{");
      EP e = expr();
      expect("}");
      p.conds.emplace_back(when, std::move(e));
    }
    expect(";");
    p.offset = first.offset; p.line = first.line; p.col = first.col;
    p.filename = filename;
    return p;
  }
  std::string path() {
    const Tok& x = next();
    if (x.k != TK::Ident) throw ParseError{"expected identifier, got '" + x.text + "'"};
    std::string s = x.text;
    while (is_op("::") && peek(1).k == TK::Ident) { next(); s += "::" + next().text; }
    return s;
  }
  Uid entity_ref() {
    const Tok& x = next();
    if (x.k != TK::Ident) throw ParseError{"expected entity, got '" + x.text + "'"};
    std::string ty = x.text;
    for (;;) {
      expect("::");
      const Tok& n = next();
      if (n.k == TK::Str) return Uid{ty, unescape(n.text, false, nullptr)};
      if (n.k != TK::Ident) throw ParseError{"bad entity reference"};
      ty += "::" + n.text;
    }
  }
  Scope scope(const char* var) {
    expect(var);
    Scope s;
    if (is_op("==")) { next(); s.k = SK::Eq; s.ent = entity_ref(); return s; }
    if (is_kw("is")) {
      next();
      s.etype = path();
      if (is_kw("in")) { next(); s.k = SK::IsIn; s.ent = entity_ref(); return s; }
      s.k = SK::Is;
      return s;
    }
    if (is_kw("in")) { next(); s.k = SK::In; s.ent = entity_ref(); return s; }
    return s;
  }
  Scope action_scope() {
    expect("action");
    Scope s;
    if (is_op("==")) { next(); s.k = SK::Eq; s.ent = entity_ref(); return s; }
    if (is_kw("in")) {
      next();
      if (is_op("[")) {
        next();
        s.k = SK::InSet;
        if (!is_op("]")) {
          s.ents.push_back(entity_ref());
          while (is_op(",")) {
            next();
            if (is_op("]")) break;
            s.ents.push_back(entity_ref());
          }
        }
        expect("]");
        return s;
      }
      s.k = SK::In; s.ent = entity_ref();
      return s;
    }
    return s;
  }
  EP expr() {
    if (is_kw("if")) {
      next();
      EP e = mk(EK::If);
      e->kids.push_back(expr());
      expect("then");
      e->kids.push_back(expr());
      expect("else");
      e->kids.push_back(expr());
      return e;
    }
    return or_();
  }
  EP bin2(EK k, EP a, EP b) { EP e = mk(k); e->kids.push_back(std::move(a)); e->kids.push_back(std::move(b)); return e; }
  EP binop(Bin op, EP a, EP b) { EP e = bin2(EK::Bin, std::move(a), std::move(b)); e->op = op; return e; }
  EP or_() {
    EP l = and_();
    while (is_op("||")) { next(); l = bin2(EK::Or, std::move(l), and_()); }
    return l;
  }
  EP and_() {
    EP l = relation();
    while (is_op("&&")) { next(); l = bin2(EK::And, std::move(l), relation()); }
    return l;
  }
  EP relation() {
    EP l = add();
    const Tok& x = peek();
    if (x.k == TK::Op) {
      static const std::pair<const char*, Bin> rel[] = {{"==", Bin::Eq}, {"!=", Bin::Ne}, {"<", Bin::Lt},
                                                         {"<=", Bin::Le}, {">", Bin::Gt}, {">=", Bin::Ge}};
      for (auto& r : rel)
        if (x.text == r.first) { next(); return binop(r.second, std::move(l), add()); }
    }
    if (is_kw("in")) { next(); return binop(Bin::In, std::move(l), add()); }
    if (is_kw("has")) {
      next();
      const Tok& k = next();
      EP e = mk(EK::Has);
      if (k.k == TK::Str) e->name = unescape(k.text, false, nullptr);
      else if (k.k == TK::Ident) e->name = k.text;
      else throw ParseError{"expected attribute after has"};
      e->kids.push_back(std::move(l));
      return e;
    }
    if (is_kw("like")) {
      next();
      const Tok& s = next();
      if (s.k != TK::Str) throw ParseError{"expected pattern after like"};
      EP e = mk(EK::Like);
      unescape(s.text, true, &e->pat);
      e->kids.push_back(std::move(l));
      return e;
    }
    if (is_kw("is")) {
      next();
      EP e = mk(EK::Is);
      e->name = path();
      e->kids.push_back(std::move(l));
      if (is_kw("in")) { next(); e->has_in = true; e->kids.push_back(add()); }
      return e;
    }
    return l;
  }
  EP add() {
    EP l = mult();
    while (is_op("+") || is_op("-")) {
      Bin op = next().text == "+" ? Bin::Add : Bin::Sub;
      l = binop(op, std::move(l), mult());
    }
    return l;
  }
  EP mult() {
    EP l = unary();
    while (is_op("*")) { next(); l = binop(Bin::Mul, std::move(l), unary()); }
    return l;
  }
  EP long_lit(const std::string& digits, bool neg) {
    unsigned __int128 v = 0;
    for (char c : digits) {
      v = v * 10 + (unsigned)(c - '0');
      if (v > ((unsigned __int128)1 << 64)) throw ParseError{"integer literal out of range"};
    }
    const unsigned __int128 lim = neg ? ((unsigned __int128)1 << 63) : (((unsigned __int128)1 << 63) - 1);
    if (v > lim) throw ParseError{"integer literal out of range"};
    EP e = mk(EK::Lit);
    e->lit.t = VT::Long;
    e->lit.i = neg ? (int64_t)(-(__int128)v) : (int64_t)v;
    return e;
  }
  EP unary() {
    std::vector<std::string> ops;
    while (is_op("!") || is_op("-")) ops.push_back(next().text);
    if (ops.size() > 4) throw ParseError{"too many unary operators"};
    EP e;
    if (!ops.empty() && ops.back() == "-" && peek().k == TK::Int) {
      ops.pop_back();
      e = member_tail(long_lit(next().text, true));
    } else {
      e = member_tail(primary());
    }
    for (auto it = ops.rbegin(); it != ops.rend(); ++it) {
      EP u = mk(*it == "!" ? EK::Not : EK::Neg);
      u->kids.push_back(std::move(e));
      e = std::move(u);
    }
    return e;
  }
  EP member_tail(EP e) {
    for (;;) {
      if (is_op(".")) {
        next();
        const Tok& nm = next();
        if (nm.k != TK::Ident) throw ParseError{"expected attribute name"};
        if (is_op("(")) {
          next();
          EP m = mk(EK::Method);
          m->name = nm.text;
          m->kids.push_back(std::move(e));
          expr_list(")", m->kids);
          e = std::move(m);
        } else {
          EP a = mk(EK::Attr);
          a->name = nm.text;
          a->kids.push_back(std::move(e));
          e = std::move(a);
        }
      } else if (is_op("[")) {
        next();
        const Tok& s = next();
        if (s.k != TK::Str) throw ParseError{"expected string index"};
        expect("]");
        EP a = mk(EK::Attr);
        a->name = unescape(s.text, false, nullptr);
        a->kids.push_back(std::move(e));
        e = std::move(a);
      } else {
        return e;
      }
    }
  }
  void expr_list(const char* close, std::vector<EP>& out) {
    if (!is_op(close)) {
      out.push_back(expr());
      while (is_op(",")) {
        next();
        if (is_op(close)) break;
        out.push_back(expr());
      }
    }
    expect(close);
  }
  EP str_lit(std::string s) {
    EP e = mk(EK::Lit);
    e->strs.emplace_back(new std::string(std::move(s)));
    e->lit.t = VT::Str;
    e->lit.s = e->strs.back().get();
    return e;
  }
  EP primary() {
    const Tok x = peek();
    if (x.k == TK::Int) { next(); return long_lit(x.text, false); }
    if (x.k == TK::Str) { next(); return str_lit(unescape(x.text, false, nullptr)); }
    if (x.k == TK::Op && x.text == "(") {
      next();
      EP e = expr();
      expect(")");
      return e;
    }
    if (x.k == TK::Op && x.text == "[") {
      next();
      EP e = mk(EK::Set);
      expr_list("]", e->kids);
      return e;
    }
    if (x.k == TK::Op && x.text == "{") {
      next();
      EP e = mk(EK::Rec);
      if (!is_op("}")) {
        for (;;) {
          const Tok& k = next();
          std::string key;
          if (k.k == TK::Str) key = unescape(k.text, false, nullptr);
          else if (k.k == TK::Ident) key = k.text;
          else throw ParseError{"bad record key"};
          if (std::find(e->keys.begin(), e->keys.end(), key) != e->keys.end()) throw ParseError{"duplicate record key '" + key + "'"};
          e->keys.push_back(key);
          expect(":");
          e->kids.push_back(expr());
          if (is_op(",")) {
            next();
            if (is_op("}")) break;
            continue;
          }
          break;
        }
      }
      expect("}");
      return e;
    }
    if (x.k == TK::Ident) {
      if (x.text == "true" || x.text == "false") {
        next();
        EP e = mk(EK::Lit);
        e->lit.t = VT::Bool;
        e->lit.i = x.text == "true";
        return e;
      }
      static const char* vars[] = {"principal", "action", "resource", "context"};
      for (int v = 0; v < 4; v++)
        if (x.text == vars[v] && !is_op("::", 1)) {
          next();
          EP e = mk(EK::Var);
          e->var = v;
          return e;
        }
      size_t j = 1;
      while (is_op("::", j) && peek(j + 1).k == TK::Ident) j += 2;
      if (is_op("::", j) && peek(j + 1).k == TK::Str) {
        Uid u = entity_ref();
        EP e = mk(EK::Lit);
        e->strs.emplace_back(new std::string(u.type));
        e->strs.emplace_back(new std::string(u.id));
        e->lit.t = VT::Ent;
        e->lit.et = e->strs[0].get();
        e->lit.s = e->strs[1].get();
        return e;
      }
      if (is_op("(", j)) {
        EP e = mk(EK::Call);
        e->name = path();
        expect("(");
        expr_list(")", e->kids);
        return e;
      }
      throw ParseError{filename + ":" + std::to_string(x.line) + ":" + std::to_string(x.col) + ": unexpected identifier '" + x.text + "'"};
    }
    throw ParseError{filename + ":" + std::to_string(x.line) + ":" + std::to_string(x.col) + ": unexpected token '" + x.text + "'"};
  }
};

// ------------------------------------------------------------------------------------------------
// Evaluator
// ------------------------------------------------------------------------------------------------
bool like_match(const std::string& s, const std::vector<Piece>& pat, size_t si, size_t pi) {
  while (pi < pat.size()) {
    const Piece& p = pat[pi];
    if (!p.star) {
      if (si + p.lit.size() > s.size() || s.compare(si, p.lit.size(), p.lit) != 0) return false;
      si += p.lit.size();
      pi++;
    } else {
      if (pi + 1 == pat.size()) return true;
      for (size_t k = si; k <= s.size(); k++)
        if (like_match(s, pat, k, pi + 1)) return true;
      return false;
    }
  }
  return si == s.size();
}

struct Evaluator {
  const Item& it;
  Arena& A;
  const Item* st = nullptr;  // static entities of the image, merged into the map (may be null)

  // The merged EntityMap (cedar_oracle.merge_static_entities): the request's entity, else the
  // static one; a UID in both keeps the request's attributes and unites both parent lists.
  const Entity* find(const Val& u) const {
    auto f = it.ents.find(KV{*u.et, *u.s});
    if (f != it.ents.end()) return &f->second;
    if (!st) return nullptr;
    auto g = st->ents.find(KV{*u.et, *u.s});
    return g == st->ents.end() ? nullptr : &g->second;
  }
  // X in E: X == E, or E is reachable through the entity map's parent edges (absent entities have
  // no parents). Early-exit depth-first walk with a visited list, as cedar-go's entityInOne.
  bool reach(const Val& a, const KV* targets, size_t nt) const {
    for (size_t k = 0; k < nt; k++) if (KV{*a.et, *a.s} == targets[k]) return true;
    thread_local std::vector<KV> todo, known;  // reused: no allocation per test
    todo.clear();
    known.clear();
    KV cur{*a.et, *a.s};
    auto visit = [&](const std::vector<KV>& ps) {
      for (auto& p : ps) {
        if (std::find(known.begin(), known.end(), p) != known.end()) continue;
        for (size_t k = 0; k < nt; k++) if (p == targets[k]) return true;
        known.push_back(p);
        todo.push_back(p);
      }
      return false;
    };
    for (;;) {
      auto f = it.ents.find(cur);
      if (f != it.ents.end() && visit(f->second.parents)) return true;
      if (st) {
        auto g = st->ents.find(cur);
        if (g != st->ents.end() && visit(g->second.parents)) return true;
      }
      if (todo.empty()) return false;
      cur = todo.back();
      todo.pop_back();
    }
  }
  bool entity_in(const Val& a, const std::string& bt, const std::string& bi) const {
    KV t{bt, bi};
    return reach(a, &t, 1);
  }

  // Errors are values, as in cedar-go (an evaluation returns (Value, error)): a failing step sets
  // `failed` and the message, and every caller returns at once (CHK). No exception crosses the
  // evaluator, so a policy that errors costs what a false one does.
  bool failed = false;
  std::string emsg;
  Val fail(std::string m) {
    failed = true;
    emsg = std::move(m);
    return Val();
  }
  Val terr(const char* expected, const Val& got) {
    return fail(std::string("type error: expected ") + expected + ", got " + type_name(got));
  }
#define CHK(x)             \
  do {                     \
    (x);                   \
    if (failed) return {}; \
  } while (0)
  // v must be a bool: false on a type error (failed set)
  bool as_bool(const Val& v) {
    if (v.t != VT::Bool) { terr("bool", v); return false; }
    return v.i != 0;
  }
  static Val B(bool b) { Val v; v.t = VT::Bool; v.i = b; return v; }
  static Val L(int64_t x) { Val v; v.t = VT::Long; v.i = x; return v; }

  Val ev(const Expr& e) {
    switch (e.k) {
      case EK::Lit: return e.lit;
      case EK::Var: return e.var == 0 ? it.principal : e.var == 1 ? it.action : e.var == 2 ? it.resource : it.context;
      case EK::And: {
        Val x;
        CHK(x = ev(*e.kids[0]));
        bool bx;
        CHK(bx = as_bool(x));
        if (!bx) return B(false);
        Val y;
        CHK(y = ev(*e.kids[1]));
        bool by;
        CHK(by = as_bool(y));
        return B(by);
      }
      case EK::Or: {
        Val x;
        CHK(x = ev(*e.kids[0]));
        bool bx;
        CHK(bx = as_bool(x));
        if (bx) return B(true);
        Val y;
        CHK(y = ev(*e.kids[1]));
        bool by;
        CHK(by = as_bool(y));
        return B(by);
      }
      case EK::Not: {
        Val x;
        CHK(x = ev(*e.kids[0]));
        bool bx;
        CHK(bx = as_bool(x));
        return B(!bx);
      }
      case EK::Neg: {
        Val v;
        CHK(v = ev(*e.kids[0]));
        if (v.t != VT::Long) return terr("long", v);
        if (v.i == INT64_MIN) return fail("integer overflow");
        return L(-v.i);
      }
      case EK::If: {
        Val c;
        CHK(c = ev(*e.kids[0]));
        bool bc;
        CHK(bc = as_bool(c));
        return bc ? ev(*e.kids[1]) : ev(*e.kids[2]);
      }
      case EK::Bin: {
        Val a, b;
        CHK(a = ev(*e.kids[0]));
        CHK(b = ev(*e.kids[1]));
        return binop(e.op, a, b);
      }
      case EK::Has: {
        Val v;
        CHK(v = ev(*e.kids[0]));
        if (v.t == VT::Ent) {
          const Entity* en = find(v);
          return B(en && rec_get(en->attrs.agg, e.name));
        }
        if (v.t == VT::Rec) return B(rec_get(v.agg, e.name) != nullptr);
        return terr("entity or record", v);
      }
      case EK::Attr: {
        Val v;
        CHK(v = ev(*e.kids[0]));
        if (v.t == VT::Ent) {
          const Entity* en = find(v);
          if (!en) return fail("entity `" + uid_str(v) + "` does not exist");
          const Val* x = rec_get(en->attrs.agg, e.name);
          if (!x) return fail("`" + uid_str(v) + "` does not have the attribute `" + e.name + "`");
          return *x;
        }
        if (v.t == VT::Rec) {
          const Val* x = rec_get(v.agg, e.name);
          if (!x) return fail("record does not have the attribute `" + e.name + "`");
          return *x;
        }
        return terr("entity or record", v);
      }
      case EK::Like: {
        Val v;
        CHK(v = ev(*e.kids[0]));
        if (v.t != VT::Str) return terr("string", v);
        return B(like_match(*v.s, e.pat, 0, 0));
      }
      case EK::Is: {
        Val v;
        CHK(v = ev(*e.kids[0]));
        if (v.t != VT::Ent) return terr("entity", v);
        if (*v.et != e.name) return B(false);
        if (!e.has_in) return B(true);
        Val w;
        CHK(w = ev(*e.kids[1]));
        bool r;
        CHK(r = in_op(v, w));
        return B(r);
      }
      case EK::Set: {
        Agg* a = A.agg();
        for (auto& k : e.kids) {
          Val x;
          CHK(x = ev(*k));
          set_add(a, x);
        }
        Val v; v.t = VT::Set; v.agg = a;
        return v;
      }
      case EK::Rec: {
        Agg* a = A.agg();
        for (size_t k = 0; k < e.kids.size(); k++) {
          Val x;
          CHK(x = ev(*e.kids[k]));
          a->fields.emplace_back(&e.keys[k], x);
        }
        rec_sort(a);
        Val v; v.t = VT::Rec; v.agg = a;
        return v;
      }
      case EK::Call: {
        std::vector<Val> args;
        for (auto& k : e.kids) {
          Val x;
          CHK(x = ev(*k));
          args.push_back(x);
        }
        if (args.size() != 1 || args[0].t != VT::Str) return fail(e.name + " takes one string argument");
        Val v;
        // (the literal parsers report a malformed text by exception, shared with the JSON reader;
        // converted to a value here, on the extension-call path only)
        try {
          if (e.name == "decimal") { v.t = VT::Dec; v.i = parse_decimal(*args[0].s); return v; }
          if (e.name == "ip") { v.t = VT::IP; v.ip = A.ip(parse_ip(*args[0].s)); return v; }
        } catch (EvalError& x) {
          return fail(x.msg);
        }
        return fail("unknown extension function " + e.name);
      }
      case EK::Method: {
        Val recv;
        CHK(recv = ev(*e.kids[0]));
        std::vector<Val> args;
        for (size_t k = 1; k < e.kids.size(); k++) {
          Val x;
          CHK(x = ev(*e.kids[k]));
          args.push_back(x);
        }
        return method(recv, e.name, args);
      }
    }
    return fail("bad expression");
  }

  // a in b; false with `failed` set on a type error
  bool in_op(const Val& a, const Val& b) {
    if (a.t != VT::Ent) { terr("entity", a); return false; }
    if (b.t == VT::Ent) return entity_in(a, *b.et, *b.s);
    if (b.t == VT::Set) {
      for (auto& x : b.agg->el)
        if (x.t != VT::Ent) { terr("entity", x); return false; }
      std::vector<KV> ts;
      for (auto& x : b.agg->el) ts.push_back(KV{*x.et, *x.s});
      return reach(a, ts.data(), ts.size());
    }
    terr("set or entity", b);
    return false;
  }

  Val binop(Bin op, const Val& a, const Val& b) {
    switch (op) {
      case Bin::Eq: return B(veq(a, b));
      case Bin::Ne: return B(!veq(a, b));
      case Bin::In: {
        bool r;
        CHK(r = in_op(a, b));
        return B(r);
      }
      default: break;
    }
    if (a.t != VT::Long) return terr("long", a);
    if (b.t != VT::Long) return terr("long", b);
    const int64_t x = a.i, y = b.i;
    int64_t z = 0;
    switch (op) {
      case Bin::Lt: return B(x < y);
      case Bin::Le: return B(x <= y);
      case Bin::Gt: return B(x > y);
      case Bin::Ge: return B(x >= y);
      case Bin::Add: if (__builtin_add_overflow(x, y, &z)) return fail("integer overflow"); return L(z);
      case Bin::Sub: if (__builtin_sub_overflow(x, y, &z)) return fail("integer overflow"); return L(z);
      default: if (__builtin_mul_overflow(x, y, &z)) return fail("integer overflow"); return L(z);
    }
  }

  Val method(const Val& recv, const std::string& name, const std::vector<Val>& args) {
    if (name == "contains" || name == "containsAll" || name == "containsAny") {
      if (recv.t != VT::Set) return terr("set", recv);
      if (args.size() != 1) return fail(name + " takes one argument");
      if (name == "contains") {
        for (auto& x : recv.agg->el) if (veq(x, args[0])) return B(true);
        return B(false);
      }
      const Val& o = args[0];
      if (o.t != VT::Set) return terr("set", o);
      if (name == "containsAll") {
        for (auto& y : o.agg->el) {
          bool f = false;
          for (auto& x : recv.agg->el) if (veq(x, y)) { f = true; break; }
          if (!f) return B(false);
        }
        return B(true);
      }
      for (auto& y : o.agg->el)
        for (auto& x : recv.agg->el) if (veq(x, y)) return B(true);
      return B(false);
    }
    if (name == "isEmpty") {
      if (recv.t != VT::Set) return terr("set", recv);
      return B(recv.agg->el.empty());
    }
    if (name == "lessThan" || name == "lessThanOrEqual" || name == "greaterThan" || name == "greaterThanOrEqual") {
      if (recv.t != VT::Dec) return terr("decimal", recv);
      // a missing argument reports the Python oracle's "unknown" type name
      if (args.empty()) return fail("type error: expected decimal, got unknown");
      if (args[0].t != VT::Dec) return terr("decimal", args[0]);
      const int64_t x = recv.i, y = args[0].i;
      if (name == "lessThan") return B(x < y);
      if (name == "lessThanOrEqual") return B(x <= y);
      if (name == "greaterThan") return B(x > y);
      return B(x >= y);
    }
    if (name == "isIpv4" || name == "isIpv6" || name == "isLoopback" || name == "isMulticast" || name == "isInRange") {
      if (recv.t != VT::IP) return terr("IP", recv);
      const IPv& ip = *recv.ip;
      if (name == "isIpv4") return B(!ip.v6);
      if (name == "isIpv6") return B(ip.v6);
      if (name == "isLoopback") {
        if (!ip.v6) return B(ip.a[0] == 127);
        for (int k = 0; k < 15; k++) if (ip.a[k]) return B(false);
        return B(ip.a[15] == 1);
      }
      if (name == "isMulticast") return B(ip.v6 ? ip.a[0] == 0xFF : (ip.a[0] >> 4) == 0xE);
      if (args.empty()) return fail("type error: expected IP, got unknown");
      if (args[0].t != VT::IP) return terr("IP", args[0]);
      const IPv& o = *args[0].ip;
      if (o.v6 != ip.v6) return B(false);
      if (ip.prefix < o.prefix) return B(false);
      uint8_t na[16], nb[16];
      ip_network(ip, na);
      ip_network(o, nb);
      // ip.network within o.network: o's prefix bits of ip's network equal o's network
      const int n = ip.v6 ? 16 : 4;
      for (int k = 0; k < n; k++) {
        int bits = (int)o.prefix - 8 * k;
        uint8_t m = bits >= 8 ? 0xFF : bits <= 0 ? 0 : (uint8_t)(0xFF << (8 - bits));
        if ((na[k] & m) != nb[k]) return B(false);
      }
      return B(true);
    }
    return fail("unknown method " + name);
  }
#undef CHK

  bool scope_match(const Scope& sc, const Val& v) {
    switch (sc.k) {
      case SK::Any: return true;
      case SK::Eq: return *v.et == sc.ent.type && *v.s == sc.ent.id;
      case SK::In: return entity_in(v, sc.ent.type, sc.ent.id);
      case SK::Is: return *v.et == sc.etype;
      case SK::IsIn: return *v.et == sc.etype && entity_in(v, sc.ent.type, sc.ent.id);
      case SK::InSet: {
        std::vector<KV> ts;
        for (auto& x : sc.ents) ts.push_back(KV{x.type, x.id});
        return reach(v, ts.data(), ts.size());
      }
    }
    return false;
  }

  // satisfied? On an error: false with `failed` set and the message in emsg (the policy is then
  // skipped and reported); the caller clears `failed` before the next policy.
  bool eval_policy(const Policy& p) {
    if (!scope_match(p.p, it.principal)) return false;
    if (!scope_match(p.a, it.action)) return false;
    if (!scope_match(p.r, it.resource)) return false;
    for (auto& c : p.conds) {
      const Val x = ev(*c.second);
      if (failed) return false;
      const bool v = as_bool(x);
      if (failed) return false;
      if (c.first && !v) return false;
      if (!c.first && v) return false;
    }
    return true;
  }
};

// ------------------------------------------------------------------------------------------------
// PolicySet / tiers / diagnostics
// ------------------------------------------------------------------------------------------------
struct Tier {
  std::vector<Policy> pols;
  std::unordered_map<std::string, size_t> ids;
  void add(Policy p) {  // cedar PolicySet.Add: a repeated ID replaces the earlier policy in place
    auto f = ids.find(p.id);
    if (f != ids.end()) { pols[f->second] = std::move(p); return; }
    ids.emplace(p.id, pols.size());
    pols.push_back(std::move(p));
  }
};

struct Result {
  int allow = 0;
  uint32_t tier = 0;
  std::vector<uint32_t> reasons;                           // policy indices (insertion order)
  std::vector<std::pair<uint32_t, std::string>> errors;     // (policy index, message)
};

void is_authorized(const Tier& t, Evaluator& ev, Result& r) {
  std::vector<uint32_t> forbids, permits;
  r.errors.clear();
  for (uint32_t k = 0; k < t.pols.size(); k++) {
    const Policy& p = t.pols[k];
    ev.failed = false;
    const bool sat = ev.eval_policy(p);
    if (ev.failed) {
      r.errors.emplace_back(k, "while evaluating policy `" + p.id + "`: " + ev.emsg);
      continue;
    }
    if (!sat) continue;
    (p.forbid ? forbids : permits).push_back(k);
  }
  if (!forbids.empty()) { r.allow = 0; r.reasons = std::move(forbids); }
  else if (!permits.empty()) { r.allow = 1; r.reasons = std::move(permits); }
  else { r.allow = 0; r.reasons.clear(); }
}

void tiered(const std::vector<Tier>& tiers, const Item& it, Arena& A, Result& r, const Item* statics) {
  Evaluator ev{it, A, statics, false, {}};
  r = Result();
  for (uint32_t t = 0; t < tiers.size(); t++) {
    A.clear();
    is_authorized(tiers[t], ev, r);
    r.tier = t;
    if (t + 1 == tiers.size()) break;
    if (!r.allow && r.reasons.empty() && r.errors.empty()) continue;
    break;
  }
}

void pos_json(const Policy& p, std::string& o) {
  o += "{\"filename\":";
  go_json_string(p.filename, o);
  o += ",\"offset\":" + std::to_string(p.offset) + ",\"line\":" + std::to_string(p.line) + ",\"column\":" + std::to_string(p.col) + "}";
}
void reason_json(const Policy& p, std::string& o) {
  o += "{\"policy\":";
  go_json_string(p.id, o);
  o += ",\"position\":";
  pos_json(p, o);
  o += "}";
}
void diag_json(const Tier& t, const Result& r, bool reasons_only, std::string& o) {
  if (reasons_only) {
    o += "[";
    for (size_t k = 0; k < r.reasons.size(); k++) {
      if (k) o += ",";
      reason_json(t.pols[r.reasons[k]], o);
    }
    o += "]";
    return;
  }
  o += "{";
  if (!r.reasons.empty()) {
    o += "\"reasons\":[";
    for (size_t k = 0; k < r.reasons.size(); k++) {
      if (k) o += ",";
      reason_json(t.pols[r.reasons[k]], o);
    }
    o += "]";
  }
  if (!r.errors.empty()) {
    if (!r.reasons.empty()) o += ",";
    o += "\"errors\":[";
    for (size_t k = 0; k < r.errors.size(); k++) {
      if (k) o += ",";
      const Policy& p = t.pols[r.errors[k].first];
      o += "{\"policy\":";
      go_json_string(p.id, o);
      o += ",\"position\":";
      pos_json(p, o);
      o += ",\"message\":";
      go_json_string(r.errors[k].second, o);
      o += "}";
    }
    o += "]";
  }
  o += "}";
}

struct Set {
  std::vector<Tier> tiers;
  std::string err;
  std::vector<std::unique_ptr<Item>> items;  // loaded items (bench / batch)
  std::unique_ptr<Item> statics;             // static entities (cref_set_entities)
};

}  // namespace cref

using namespace cref;

extern "C" {

typedef struct cref_set cref_set;

cref_set* cref_create(void) { return reinterpret_cast<cref_set*>(new Set()); }
void cref_destroy(cref_set* s) { delete reinterpret_cast<Set*>(s); }
const char* cref_last_error(cref_set* s) { return reinterpret_cast<Set*>(s)->err.c_str(); }

int cref_add_tier(cref_set* s0) {
  reinterpret_cast<Set*>(s0)->tiers.emplace_back();
  return 0;
}

static int add_doc(Set* s, const char* filename, const char* text, size_t len, const char* pre, const char* suf,
                   const char* explicit_id, int zero_position) {
  if (s->tiers.empty()) s->tiers.emplace_back();
  try {
    Parser P{tokenize(std::string(text, len)), 0, filename ? filename : ""};
    std::vector<Policy> ps = P.policies();
    if (explicit_id && ps.size() != 1) { s->err = "document must hold exactly one policy"; return -1; }
    for (size_t i = 0; i < ps.size(); i++) {
      Policy& p = ps[i];
      p.id = explicit_id ? std::string(explicit_id) : std::string(pre ? pre : "") + std::to_string(i) + (suf ? suf : "");
      if (zero_position) { p.offset = p.line = p.col = 0; p.filename.clear(); }
      s->tiers.back().add(std::move(p));
    }
  } catch (ParseError& e) {
    s->err = e.msg;
    return -2;
  }
  return 0;
}

int cref_add_document(cref_set* s, const char* filename, const char* text, size_t len, const char* id_prefix,
                      const char* id_suffix) {
  return add_doc(reinterpret_cast<Set*>(s), filename, text, len, id_prefix, id_suffix, nullptr, 0);
}

int cref_add_policy(cref_set* s, const char* policy_id, const char* filename, const char* text, size_t len,
                    int zero_position) {
  return add_doc(reinterpret_cast<Set*>(s), filename, text, len, nullptr, nullptr, policy_id, zero_position);
}

// Static entities (a JSON entity array) merged into every item's EntityMap; empty: none.
int cref_set_entities(cref_set* s0, const char* json, size_t len) {
  Set* s = reinterpret_cast<Set*>(s0);
  try {
    s->statics.reset();
    if (!len) return 0;
    std::string item = "{\"entities\":" + std::string(json, len) +
                       ",\"request\":{\"principal\":{\"type\":\"_\",\"id\":\"\"},\"action\":{\"type\":\"_\",\"id\":\"\"},"
                       "\"resource\":{\"type\":\"_\",\"id\":\"\"}}}";
    J j = parse_json(item.data(), item.size());
    std::unique_ptr<Item> it(new Item());
    item_from_json(j, *it);
    s->statics = std::move(it);
  } catch (std::exception& e) {
    s->err = e.what();
    return -1;
  } catch (EvalError& e) {
    s->err = e.msg;
    return -1;
  }
  return 0;
}

// Loads a JSON array of {"entities":[...],"request":{...}} items (replacing earlier ones).
int cref_load_items(cref_set* s0, const char* json, size_t len, uint32_t* n) {
  Set* s = reinterpret_cast<Set*>(s0);
  try {
    J j = parse_json(json, len);
    if (j.k != J::Arr) { s->err = "items must be a JSON array"; return -1; }
    s->items.clear();
    for (auto& x : j.a) {
      std::unique_ptr<Item> it(new Item());
      item_from_json(x, *it);
      s->items.push_back(std::move(it));
    }
  } catch (std::exception& e) {
    s->err = e.what();
    return -1;
  } catch (EvalError& e) {
    s->err = e.msg;
    return -1;
  }
  *n = (uint32_t)s->items.size();
  return 0;
}

// Evaluates every loaded item on `threads` threads. Output (malloc'd, free with cref_free): one line
// per item: "<allow>\t<tier>\t<json.Marshal(Diagnostic)>\t<json.Marshal(Reasons)>\n".
int cref_eval(cref_set* s0, int threads, char** out, size_t* out_len) {
  Set* s = reinterpret_cast<Set*>(s0);
  const size_t n = s->items.size();
  std::vector<std::string> lines(n);
  threads = std::max(1, threads);
  std::atomic<size_t> next{0};
  auto work = [&]() {
    Arena A;
    Result r;
    for (;;) {
      size_t k = next.fetch_add(1);
      if (k >= n) break;
      tiered(s->tiers, *s->items[k], A, r, s->statics.get());
      std::string& o = lines[k];
      o = std::to_string(r.allow) + "\t" + std::to_string(r.tier) + "\t";
      diag_json(s->tiers[r.tier], r, false, o);
      o += "\t";
      diag_json(s->tiers[r.tier], r, true, o);
      o += "\n";
    }
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads; t++) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  size_t total = 0;
  for (auto& l : lines) total += l.size();
  char* buf = (char*)malloc(total + 1);
  size_t o = 0;
  for (auto& l : lines) { memcpy(buf + o, l.data(), l.size()); o += l.size(); }
  buf[o] = 0;
  *out = buf;
  *out_len = o;
  return 0;
}

// CPU baseline: `threads` threads evaluate disjoint round-robin shards of the loaded items (each
// thread walks its own items in a loop) for `seconds`; reports decisions done and wall time. The
// decision work matches cedar-go's IsAuthorized per request (entity maps pre-built, as §8(d) says).
int cref_bench(cref_set* s0, int threads, double seconds, uint64_t* decisions, double* wall_s) {
  Set* s = reinterpret_cast<Set*>(s0);
  const size_t n = s->items.size();
  if (!n) { *decisions = 0; *wall_s = 0; return 0; }
  threads = std::max(1, threads);
  std::atomic<uint64_t> total{0};
  std::atomic<uint32_t> sink{0};
  const auto t0 = std::chrono::steady_clock::now();
  const auto deadline = t0 + std::chrono::duration<double>(seconds);
  auto work = [&](int w) {
    Arena A;
    Result r;
    uint64_t done = 0;
    uint32_t acc = 0;
    size_t k = (size_t)w % n;
    while (std::chrono::steady_clock::now() < deadline) {
      for (int rep = 0; rep < 16; rep++) {
        tiered(s->tiers, *s->items[k], A, r, s->statics.get());
        acc += (uint32_t)r.allow + (uint32_t)r.reasons.size();
        done++;
        k += (size_t)threads;
        if (k >= n) k = (size_t)w % n;
      }
    }
    total += done;
    sink += acc;
  };
  std::vector<std::thread> th;
  for (int t = 1; t < threads; t++) th.emplace_back(work, t);
  work(0);
  for (auto& t : th) t.join();
  *wall_s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  *decisions = total.load();
  return (int)(sink.load() & 0);
}

void cref_free(void* p) { free(p); }

}  // extern "C"
