// Cedar policy-text parser (host side of the compiler).
//
// Replaces cedar.NewPolicySetFromBytes / cedar.NewPolicyListFromBytes as used by the reference's
// stores (internal/server/store/memory.go:18, directory.go:69, crd.go:51,91,
// verified_permissions.go:89). Grammar: the Cedar policy language (annotations, permit/forbid,
// principal/action/resource scope, when/unless conditions, full expression grammar without
// templates). A policy's Position is the byte offset / 1-based line / 1-based character column
// of its first token (annotation or effect), as pinned by authorizer_test.go:504 and
// store_test.go:102-103.
#include <cctype>
#include <cstring>

#include "cedar.h"

namespace cg {

namespace {

enum class TK : uint8_t { Ident, Str, Int, Op, Eof };

struct Tok {
  TK k;
  std::string text;  // raw (strings: undecoded body)
  int64_t off, line, col;
};

struct Lexer {
  const std::string& s;
  size_t i = 0;
  int64_t line = 1, col = 1;
  explicit Lexer(const std::string& src) : s(src) {}

  void adv() {
    unsigned char c = (unsigned char)s[i++];
    if (c == '\n') { line++; col = 1; }
    else if ((c & 0xC0) != 0x80) col++;  // count characters, not continuation bytes
  }
  // a continuation byte must not advance the column, but the lead byte already did
  std::vector<Tok> run() {
    std::vector<Tok> out;
    const size_t n = s.size();
    while (i < n) {
      unsigned char c = (unsigned char)s[i];
      if (c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\f' || c == '\v') { adv(); continue; }
      if (c == '/' && i + 1 < n && s[i + 1] == '/') { while (i < n && s[i] != '\n') adv(); continue; }
      Tok t; t.off = (int64_t)i; t.line = line; t.col = col;
      if (std::isalpha(c) || c == '_') {
        size_t j = i;
        while (j < n && (std::isalnum((unsigned char)s[j]) || s[j] == '_')) j++;
        t.k = TK::Ident; t.text = s.substr(i, j - i);
        while (i < j) adv();
        out.push_back(std::move(t));
        continue;
      }
      if (std::isdigit(c)) {
        size_t j = i;
        while (j < n && std::isdigit((unsigned char)s[j])) j++;
        t.k = TK::Int; t.text = s.substr(i, j - i);
        while (i < j) adv();
        out.push_back(std::move(t));
        continue;
      }
      if (c == '"') {
        size_t j = i + 1;
        while (j < n && s[j] != '"') { if (s[j] == '\\') j++; j++; }
        if (j >= n) throw CedarError("unterminated string literal at line " + std::to_string(line));
        t.k = TK::Str; t.text = s.substr(i + 1, j - i - 1);
        while (i <= j) adv();
        out.push_back(std::move(t));
        continue;
      }
      static const char* ops2[] = {"==", "!=", "<=", ">=", "&&", "||", "::"};
      bool got = false;
      for (const char* o : ops2) {
        if (i + 1 < n && s[i] == o[0] && s[i + 1] == o[1]) {
          t.k = TK::Op; t.text = o; adv(); adv(); out.push_back(t); got = true; break;
        }
      }
      if (got) continue;
      if (std::strchr("()[]{},;.@<>!+-*:", c)) {
        t.k = TK::Op; t.text = std::string(1, (char)c); adv(); out.push_back(std::move(t));
        continue;
      }
      throw CedarError("unexpected character '" + std::string(1, (char)c) + "' at line " +
                       std::to_string(line) + " column " + std::to_string(col));
    }
    Tok e; e.k = TK::Eof; e.off = (int64_t)i; e.line = line; e.col = col;
    out.push_back(e);
    return out;
  }
};

void put_utf8(std::string& o, uint32_t cp) {
  if (cp < 0x80) o += (char)cp;
  else if (cp < 0x800) { o += (char)(0xC0 | (cp >> 6)); o += (char)(0x80 | (cp & 0x3F)); }
  else if (cp < 0x10000) { o += (char)(0xE0 | (cp >> 12)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
  else { o += (char)(0xF0 | (cp >> 18)); o += (char)(0x80 | ((cp >> 12) & 0x3F)); o += (char)(0x80 | ((cp >> 6) & 0x3F)); o += (char)(0x80 | (cp & 0x3F)); }
}

// Decodes Cedar escapes. With `pat`, unescaped '*' becomes a wildcard piece and "\*" a literal.
std::string unescape(const std::string& raw, std::vector<PatPiece>* pat) {
  std::string lit;
  for (size_t i = 0; i < raw.size(); i++) {
    char c = raw[i];
    if (c == '\\') {
      if (++i >= raw.size()) throw CedarError("bad escape");
      char e = raw[i];
      switch (e) {
        case 'n': lit += '\n'; break;
        case 'r': lit += '\r'; break;
        case 't': lit += '\t'; break;
        case '\\': lit += '\\'; break;
        case '0': lit += '\0'; break;
        case '\'': lit += '\''; break;
        case '"': lit += '"'; break;
        case '*':
          if (!pat) throw CedarError("bad escape \\*");
          lit += '*';
          break;
        case 'x': {
          if (i + 2 >= raw.size() + 0 && i + 2 > raw.size()) throw CedarError("bad \\x escape");
          std::string h = raw.substr(i + 1, 2);
          if (h.size() != 2 || !std::isxdigit((unsigned char)h[0]) || !std::isxdigit((unsigned char)h[1]))
            throw CedarError("bad \\x escape");
          unsigned v = (unsigned)std::stoul(h, nullptr, 16);
          if (v > 0x7F) throw CedarError("bad \\x escape");
          lit += (char)v;
          i += 2;
          break;
        }
        case 'u': {
          if (i + 1 >= raw.size() || raw[i + 1] != '{') throw CedarError("bad \\u escape");
          size_t j = raw.find('}', i);
          if (j == std::string::npos) throw CedarError("bad \\u escape");
          put_utf8(lit, (uint32_t)std::stoul(raw.substr(i + 2, j - i - 2), nullptr, 16));
          i = j;
          break;
        }
        default: throw CedarError(std::string("bad escape \\") + e);
      }
      continue;
    }
    if (c == '*' && pat) {
      if (!lit.empty()) { pat->push_back({false, lit}); lit.clear(); }
      pat->push_back({true, ""});
      continue;
    }
    lit += c;
  }
  if (pat) {
    if (!lit.empty()) pat->push_back({false, lit});
    return std::string();
  }
  return lit;
}

ExprP mk(EK k) { auto e = std::make_shared<Expr>(); e->k = k; return e; }

struct Parser {
  std::vector<Tok> t;
  size_t i = 0;
  std::string fname;

  const Tok& peek(size_t k = 0) const { return t[std::min(i + k, t.size() - 1)]; }
  const Tok& next() { return t[i++]; }
  bool is_op(const char* s, size_t k = 0) const { const Tok& x = peek(k); return x.k == TK::Op && x.text == s; }
  bool is_kw(const char* s, size_t k = 0) const { const Tok& x = peek(k); return x.k == TK::Ident && x.text == s; }
  [[noreturn]] void fail(const std::string& m) const {
    const Tok& x = peek();
    throw CedarError(fname + ":" + std::to_string(x.line) + ":" + std::to_string(x.col) + ": " + m);
  }
  void expect(const char* s) {
    const Tok& x = peek();
    if ((x.k != TK::Op && x.k != TK::Ident) || x.text != s) fail(std::string("expected '") + s + "', got '" + x.text + "'");
    i++;
  }

  std::vector<Policy> policies() {
    std::vector<Policy> out;
    while (peek().k != TK::Eof) out.push_back(policy());
    return out;
  }

  Policy policy() {
    Policy p;
    p.filename = fname;
    const Tok& first = peek();
    p.pos.offset = first.off; p.pos.line = first.line; p.pos.column = first.col;
    while (is_op("@")) {
      next();
      const Tok& nm = next();
      if (nm.k != TK::Ident) fail("bad annotation");
      std::string val;
      if (is_op("(")) {
        next();
        const Tok& sv = next();
        if (sv.k != TK::Str) fail("annotation value must be a string");
        val = unescape(sv.text, nullptr);
        expect(")");
      }
      for (auto& a : p.annotations) if (a.first == nm.text) fail("duplicate annotation @" + nm.text);
      p.annotations.emplace_back(nm.text, val);
    }
    const Tok& eff = next();
    if (eff.k != TK::Ident || (eff.text != "permit" && eff.text != "forbid")) {
      i--;
      fail("expected permit or forbid, got '" + eff.text + "'");
    }
    p.forbid = eff.text == "forbid";
    expect("(");
    p.principal = scope("principal");
    expect(",");
    p.action = action_scope();
    expect(",");
    p.resource = scope("resource");
    expect(")");
    while (is_kw("when") || is_kw("unless")) {
      bool when = next().text == "when";
      expect("{");
      ExprP e = expr();
      expect("}");
      p.conds.emplace_back(when, e);
    }
    expect(";");
    return p;
  }

  std::string path() {
    const Tok& x = next();
    if (x.k != TK::Ident) { i--; fail("expected identifier"); }
    std::string s = x.text;
    while (is_op("::") && peek(1).k == TK::Ident) { next(); s += "::"; s += next().text; }
    return s;
  }

  std::pair<std::string, std::string> entity_ref() {
    const Tok& x = next();
    if (x.k != TK::Ident) { i--; fail("expected entity reference"); }
    std::string ty = x.text;
    for (;;) {
      expect("::");
      const Tok& n = next();
      if (n.k == TK::Str) return {ty, unescape(n.text, nullptr)};
      if (n.k != TK::Ident) { i--; fail("bad entity reference"); }
      ty += "::"; ty += n.text;
    }
  }

  Scope scope(const char* var) {
    expect(var);
    Scope s;
    if (is_op("==")) { next(); s.kind = ScopeKind::Eq; s.ent = entity_ref(); return s; }
    if (is_kw("is")) {
      next();
      s.etype = path();
      if (is_kw("in")) { next(); s.kind = ScopeKind::IsIn; s.ent = entity_ref(); return s; }
      s.kind = ScopeKind::Is;
      return s;
    }
    if (is_kw("in")) { next(); s.kind = ScopeKind::In; s.ent = entity_ref(); return s; }
    return s;
  }

  Scope action_scope() {
    expect("action");
    Scope s;
    if (is_op("==")) { next(); s.kind = ScopeKind::Eq; s.ent = entity_ref(); return s; }
    if (is_kw("in")) {
      next();
      if (is_op("[")) {
        next();
        s.kind = ScopeKind::InSet;
        if (!is_op("]")) {
          s.ents.push_back(entity_ref());
          while (is_op(",")) { next(); if (is_op("]")) break; s.ents.push_back(entity_ref()); }
        }
        expect("]");
        return s;
      }
      s.kind = ScopeKind::In; s.ent = entity_ref();
      return s;
    }
    return s;
  }

  ExprP expr() {
    if (is_kw("if")) {
      next();
      auto e = mk(EK::If);
      e->kids.push_back(expr());
      expect("then");
      e->kids.push_back(expr());
      expect("else");
      e->kids.push_back(expr());
      return e;
    }
    return or_();
  }
  ExprP or_() {
    ExprP l = and_();
    while (is_op("||")) { next(); auto e = mk(EK::Or); { ExprP rhs = and_(); e->kids = {l, rhs}; } l = e; }
    return l;
  }
  ExprP and_() {
    ExprP l = relation();
    while (is_op("&&")) { next(); auto e = mk(EK::And); { ExprP rhs = relation(); e->kids = {l, rhs}; } l = e; }
    return l;
  }
  ExprP relation() {
    ExprP l = add();
    const Tok& x = peek();
    if (x.k == TK::Op) {
      static const std::pair<const char*, BinOp> rel[] = {{"==", BinOp::Eq}, {"!=", BinOp::Ne}, {"<", BinOp::Lt},
                                                          {"<=", BinOp::Le}, {">", BinOp::Gt}, {">=", BinOp::Ge}};
      for (auto& r : rel) {
        if (x.text == r.first) {
          next();
          auto e = mk(EK::Bin); e->op = r.second; { ExprP rhs = add(); e->kids = {l, rhs}; }
          return e;
        }
      }
    }
    if (is_kw("in")) { next(); auto e = mk(EK::Bin); e->op = BinOp::In; { ExprP rhs = add(); e->kids = {l, rhs}; } return e; }
    if (is_kw("has")) {
      next();
      const Tok& k = next();
      auto e = mk(EK::Has);
      e->kids = {l};
      if (k.k == TK::Str) e->name = unescape(k.text, nullptr);
      else if (k.k == TK::Ident) e->name = k.text;
      else { i--; fail("expected attribute after has"); }
      return e;
    }
    if (is_kw("like")) {
      next();
      const Tok& sv = next();
      if (sv.k != TK::Str) { i--; fail("expected pattern after like"); }
      auto e = mk(EK::Like);
      e->kids = {l};
      unescape(sv.text, &e->pat);
      return e;
    }
    if (is_kw("is")) {
      next();
      auto e = mk(EK::Is);
      e->name = path();
      e->kids = {l};
      if (is_kw("in")) { next(); e->has_in = true; e->kids.push_back(add()); }
      return e;
    }
    return l;
  }
  ExprP add() {
    ExprP l = mult();
    while (is_op("+") || is_op("-")) {
      bool plus = next().text == "+";
      auto e = mk(EK::Bin); e->op = plus ? BinOp::Add : BinOp::Sub; { ExprP rhs = mult(); e->kids = {l, rhs}; } l = e;
    }
    return l;
  }
  ExprP mult() {
    ExprP l = unary();
    while (is_op("*")) { next(); auto e = mk(EK::Bin); e->op = BinOp::Mul; { ExprP rhs = unary(); e->kids = {l, rhs}; } l = e; }
    return l;
  }
  ExprP unary() {
    std::vector<char> ops;
    while (is_op("!") || is_op("-")) ops.push_back(next().text[0]);
    if (ops.size() > 4) fail("too many unary operators");
    ExprP e;
    if (!ops.empty() && ops.back() == '-' && peek().k == TK::Int) {
      ops.pop_back();
      const Tok& it = next();
      // -9223372036854775808 is representable only as a negated literal
      if (it.text.size() > 19 || (it.text.size() == 19 && it.text > "9223372036854775808")) fail("integer literal out of range");
      int64_t v;
      if (it.text == "9223372036854775808") v = INT64_MIN;
      else v = -(int64_t)std::stoll(it.text);
      auto l = mk(EK::Lit); l->lit = HVal::Long(v);
      e = member_tail(l);
    } else {
      e = member();
    }
    for (auto it = ops.rbegin(); it != ops.rend(); ++it) {
      auto u = mk(*it == '!' ? EK::Not : EK::Neg);
      u->kids = {e};
      e = u;
    }
    return e;
  }
  // The extension functions and methods Cedar defines (ip/decimal plus the set, decimal and ipaddr
  // methods): anything else, or another argument count, is a parse error, so a document that
  // names one is rejected (or skipped by the stores that skip bad documents) as a whole.
  static int method_arity(const std::string& m) {
    static const char* one[] = {"contains", "containsAll", "containsAny", "lessThan", "lessThanOrEqual",
                                "greaterThan", "greaterThanOrEqual", "isInRange"};
    static const char* zero[] = {"isEmpty", "isIpv4", "isIpv6", "isLoopback", "isMulticast"};
    for (const char* x : one) if (m == x) return 1;
    for (const char* x : zero) if (m == x) return 0;
    return -1;
  }
  ExprP member() { return member_tail(primary()); }
  ExprP member_tail(ExprP e) {
    for (;;) {
      if (is_op(".")) {
        next();
        const Tok& nm = next();
        if (nm.k != TK::Ident) { i--; fail("expected attribute name"); }
        if (is_op("(")) {
          next();
          auto m = mk(EK::Method);
          m->name = nm.text;
          m->kids.push_back(e);
          auto args = expr_list(")");
          const int want = method_arity(nm.text);
          if (want < 0) fail("`" + nm.text + "` is not a method");
          if ((int)args.size() != want) fail(nm.text + " expects " + std::to_string(want) + " argument(s)");
          m->kids.insert(m->kids.end(), args.begin(), args.end());
          e = m;
        } else {
          auto a = mk(EK::Attr); a->name = nm.text; a->kids = {e}; e = a;
        }
      } else if (is_op("[")) {
        next();
        const Tok& sv = next();
        if (sv.k != TK::Str) { i--; fail("expected string index"); }
        expect("]");
        auto a = mk(EK::Attr); a->name = unescape(sv.text, nullptr); a->kids = {e}; e = a;
      } else {
        return e;
      }
    }
  }
  std::vector<ExprP> expr_list(const char* close) {
    std::vector<ExprP> v;
    if (!is_op(close)) {
      v.push_back(expr());
      while (is_op(",")) { next(); if (is_op(close)) break; v.push_back(expr()); }
    }
    expect(close);
    return v;
  }
  ExprP primary() {
    const Tok& x = peek();
    if (x.k == TK::Int) {
      next();
      if (x.text.size() > 19 || (x.text.size() == 19 && x.text > "9223372036854775807")) fail("integer literal out of range");
      auto l = mk(EK::Lit); l->lit = HVal::Long((int64_t)std::stoll(x.text));
      return l;
    }
    if (x.k == TK::Str) { next(); auto l = mk(EK::Lit); l->lit = HVal::Str(unescape(x.text, nullptr)); return l; }
    if (x.k == TK::Op && x.text == "(") { next(); ExprP e = expr(); expect(")"); return e; }
    if (x.k == TK::Op && x.text == "[") { next(); auto e = mk(EK::Set); e->kids = expr_list("]"); return e; }
    if (x.k == TK::Op && x.text == "{") {
      next();
      auto e = mk(EK::Rec);
      if (!is_op("}")) {
        for (;;) {
          const Tok& k = next();
          std::string key;
          if (k.k == TK::Str) key = unescape(k.text, nullptr);
          else if (k.k == TK::Ident) key = k.text;
          else { i--; fail("bad record key"); }
          for (auto& kk : e->keys) if (kk == key) fail("duplicate record key '" + key + "'");
          expect(":");
          e->keys.push_back(key);
          e->kids.push_back(expr());
          if (is_op(",")) { next(); if (is_op("}")) break; continue; }
          break;
        }
      }
      expect("}");
      return e;
    }
    if (x.k == TK::Ident) {
      if (x.text == "true" || x.text == "false") { next(); auto l = mk(EK::Lit); l->lit = HVal::Bool(x.text == "true"); return l; }
      if ((x.text == "principal" || x.text == "action" || x.text == "resource" || x.text == "context") && !is_op("::", 1)) {
        next();
        auto v = mk(EK::Var); v->name = x.text;
        return v;
      }
      size_t j = 1;
      while (is_op("::", j) && peek(j + 1).k == TK::Ident) j += 2;
      if (is_op("::", j) && peek(j + 1).k == TK::Str) {
        auto l = mk(EK::Lit);
        auto er = entity_ref();
        l->lit = HVal::Ent(er.first, er.second);
        return l;
      }
      if (is_op("(", j)) {
        auto c = mk(EK::Call);
        c->name = path();
        if (c->name != "ip" && c->name != "decimal") fail("`" + c->name + "` is not a function");
        expect("(");
        c->kids = expr_list(")");
        if (c->kids.size() != 1) fail(c->name + " expects 1 argument");
        return c;
      }
      fail("unexpected identifier '" + x.text + "'");
    }
    fail("unexpected token '" + x.text + "'");
  }
};

}  // namespace

std::vector<Policy> parse_policies(const std::string& src, const std::string& filename) {
  Lexer lx(src);
  Parser ps;
  ps.t = lx.run();
  ps.fname = filename;
  return ps.policies();
}

// ---------------------------------------------------------------------------------------------
// Values
// ---------------------------------------------------------------------------------------------
bool hval_eq(const HVal& a, const HVal& b) {
  if (a.k != b.k) return false;
  switch (a.k) {
    case VK::Bool: return a.b == b.b;
    case VK::Long: case VK::Dec: return a.i == b.i;
    case VK::Str: return a.s == b.s;
    case VK::Ent: return a.etype == b.etype && a.s == b.s;
    case VK::Ip: return a.ip.v6 == b.ip.v6 && a.ip.prefix == b.ip.prefix && !std::memcmp(a.ip.addr, b.ip.addr, 16);
    case VK::Set: {
      for (auto& x : a.elems) { bool f = false; for (auto& y : b.elems) if (hval_eq(x, y)) { f = true; break; } if (!f) return false; }
      for (auto& y : b.elems) { bool f = false; for (auto& x : a.elems) if (hval_eq(x, y)) { f = true; break; } if (!f) return false; }
      return true;
    }
    case VK::Rec: {
      if (a.fields.size() != b.fields.size()) return false;
      for (auto& kv : a.fields) {
        bool f = false;
        for (auto& kw : b.fields) if (kw.first == kv.first) { f = hval_eq(kv.second, kw.second); break; }
        if (!f) return false;
      }
      return true;
    }
  }
  return false;
}

bool parse_decimal(const std::string& s, int64_t* out) {
  size_t i = 0;
  bool neg = false;
  if (i < s.size() && s[i] == '-') { neg = true; i++; }
  size_t dot = s.find('.', i);
  if (dot == std::string::npos || dot == i) return false;
  std::string ip = s.substr(i, dot - i), fp = s.substr(dot + 1);
  if (fp.empty() || fp.size() > 4) return false;
  for (char c : ip) if (!std::isdigit((unsigned char)c)) return false;
  for (char c : fp) if (!std::isdigit((unsigned char)c)) return false;
  while (fp.size() < 4) fp += '0';
  __int128 v = 0;
  for (char c : ip) { v = v * 10 + (c - '0'); if (v > ((__int128)1 << 64)) return false; }
  v = v * 10000 + std::stoll(fp);
  if (neg) v = -v;
  if (v < INT64_MIN || v > INT64_MAX) return false;
  *out = (int64_t)v;
  return true;
}

static bool parse_ipv4(const std::string& s, uint8_t* a) {
  int parts = 0;
  size_t i = 0;
  while (parts < 4) {
    if (i >= s.size() || !std::isdigit((unsigned char)s[i])) return false;
    unsigned v = 0; size_t st = i;
    while (i < s.size() && std::isdigit((unsigned char)s[i])) { v = v * 10 + (s[i] - '0'); i++; if (v > 255) return false; }
    if (i - st > 1 && s[st] == '0') return false;  // no leading zeros
    a[parts++] = (uint8_t)v;
    if (parts < 4) { if (i >= s.size() || s[i] != '.') return false; i++; }
  }
  return i == s.size();
}

static bool parse_ipv6(const std::string& s, uint8_t* a) {
  // RFC 4291 text forms with "::" compression; optional embedded IPv4 tail
  std::vector<uint16_t> head, tail;
  bool dbl = false;
  size_t i = 0;
  if (s.compare(0, 2, "::") == 0) { dbl = true; i = 2; }
  std::vector<uint16_t>* cur = dbl ? &tail : &head;
  bool v4tail = false;
  uint8_t v4[4];
  while (i < s.size()) {
    size_t j = i;
    while (j < s.size() && s[j] != ':') j++;
    std::string g = s.substr(i, j - i);
    if (g.find('.') != std::string::npos) {
      if (j != s.size() || !parse_ipv4(g, v4)) return false;
      v4tail = true;
      i = j;
      break;
    }
    if (g.empty() || g.size() > 4) return false;
    for (char c : g) if (!std::isxdigit((unsigned char)c)) return false;
    cur->push_back((uint16_t)std::stoul(g, nullptr, 16));
    if (j == s.size()) { i = j; break; }
    if (j + 1 < s.size() && s[j + 1] == ':') {
      if (dbl) return false;
      dbl = true; cur = &tail; i = j + 2;
      if (i == s.size()) break;
    } else {
      i = j + 1;
      if (i == s.size()) return false;
    }
  }
  size_t groups = head.size() + tail.size() + (v4tail ? 2 : 0);
  if (groups > 8 || (!dbl && groups != 8) || (dbl && groups == 8)) return false;
  uint16_t w[8] = {0};
  for (size_t k = 0; k < head.size(); k++) w[k] = head[k];
  size_t tstart = 8 - tail.size() - (v4tail ? 2 : 0);
  for (size_t k = 0; k < tail.size(); k++) w[tstart + k] = tail[k];
  if (v4tail) { w[6] = (uint16_t)((v4[0] << 8) | v4[1]); w[7] = (uint16_t)((v4[2] << 8) | v4[3]); }
  for (int k = 0; k < 8; k++) { a[2 * k] = (uint8_t)(w[k] >> 8); a[2 * k + 1] = (uint8_t)(w[k] & 0xFF); }
  return true;
}

bool parse_ip(const std::string& s, IpVal* out) {
  std::string a = s;
  int prefix = -1;
  size_t sl = s.find('/');
  if (sl != std::string::npos) {
    a = s.substr(0, sl);
    std::string p = s.substr(sl + 1);
    if (p.empty() || p.size() > 3) return false;
    for (char c : p) if (!std::isdigit((unsigned char)c)) return false;
    if (p.size() > 1 && p[0] == '0') return false;
    prefix = std::stoi(p);
  }
  IpVal v;
  std::memset(v.addr, 0, 16);
  if (a.find(':') != std::string::npos) {
    if (!parse_ipv6(a, v.addr)) return false;
    v.v6 = 1;
    if (prefix > 128) return false;
    v.prefix = (uint8_t)(prefix < 0 ? 128 : prefix);
  } else {
    if (!parse_ipv4(a, v.addr)) return false;
    v.v6 = 0;
    if (prefix > 32) return false;
    v.prefix = (uint8_t)(prefix < 0 ? 32 : prefix);
  }
  *out = v;
  return true;
}

}  // namespace cg
