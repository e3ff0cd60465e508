// SubjectAccessReview -> (EntityMap, Request) encoder and Authorize() decision mapping.
//
// Restates, in C++ for the batching layer, the reference's per-request model:
//   GetAuthorizerAttributes / convertExtraForAuthorizerAttributes   internal/server/server.go:163-214
//   labelSelectorAsSelector / fieldSelectorAsSelector              internal/server/server.go:228-309
//   cedarWebhookAuthorizer.Authorize fast paths + mapping          internal/server/authorizer/authorizer.go:36-85
//   RecordToCedarResource                                          authorizer.go:89-111
//   ActionEntities / Impersonated- / NonResource- / ResourceToCedarEntity  authorizer/entitiy_builders.go:13-143
//   UserToCedarEntity                                              internal/server/entities/user.go:35-100
//   ResourceRequestToPath                                          internal/server/entities/authorization.go:13-30
#include <algorithm>
#include <array>
#include <cctype>
#include <cstring>
#include <deque>
#include <string_view>

#include "encode_impl.h"
#include "sar.h"

namespace cg {

namespace {

const char* kAction = "k8s::Action";
const char* kPrincipalUID = "k8s::PrincipalUID";
const char* kNonResourceURL = "k8s::NonResourceURL";
const char* kResource = "k8s::Resource";
const char* kUser = "k8s::User";
const char* kGroup = "k8s::Group";
const char* kExtra = "k8s::Extra";
const char* kSA = "k8s::ServiceAccount";
const char* kNode = "k8s::Node";
const char* kSelf = "system:authorizer:cedar-authorizer";  // options.go:15

bool starts(const std::string& s, const char* p) { return s.rfind(p, 0) == 0; }
size_t count_colons(const std::string& s) { return (size_t)std::count(s.begin(), s.end(), ':'); }
std::vector<std::string> split_colon(const std::string& s) {
  std::vector<std::string> out;
  size_t st = 0;
  for (;;) {
    size_t p = s.find(':', st);
    if (p == std::string::npos) { out.push_back(s.substr(st)); break; }
    out.push_back(s.substr(st, p - st));
    st = p + 1;
  }
  return out;
}

// k8s.io/apimachinery validation: qualified name (label key) and label value
bool alnum(char c) { return std::isalnum((unsigned char)c) != 0; }
bool valid_name63(const std::string& s) {
  if (s.empty() || s.size() > 63) return false;
  if (!alnum(s.front()) || !alnum(s.back())) return false;
  for (char c : s) if (!alnum(c) && c != '-' && c != '_' && c != '.') return false;
  return true;
}
bool valid_dns1123_subdomain(const std::string& s) {
  if (s.empty() || s.size() > 253) return false;
  size_t st = 0;
  for (;;) {
    size_t p = s.find('.', st);
    std::string lab = s.substr(st, p == std::string::npos ? std::string::npos : p - st);
    if (lab.empty() || lab.size() > 63) return false;
    auto lc = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
    if (!lc(lab.front()) || !lc(lab.back())) return false;
    for (char c : lab) if (!lc(c) && c != '-') return false;
    if (p == std::string::npos) break;
    st = p + 1;
  }
  return true;
}
bool valid_label_key(const std::string& k) {
  size_t sl = k.find('/');
  if (sl == std::string::npos) return valid_name63(k);
  if (k.find('/', sl + 1) != std::string::npos) return false;
  return valid_dns1123_subdomain(k.substr(0, sl)) && valid_name63(k.substr(sl + 1));
}
bool valid_label_value(const std::string& v) { return v.empty() || valid_name63(v); }

HVal rec(std::initializer_list<std::pair<std::string, HVal>> f) {
  HVal h;
  h.k = VK::Rec;
  for (auto& kv : f) h.fields.push_back(kv);
  return h;
}

HVal str_set(const std::vector<std::string>& vs) {
  HVal h;
  h.k = VK::Set;
  for (auto& v : vs) {
    bool dup = false;
    for (auto& e : h.elems) if (e.s == v) { dup = true; break; }
    if (!dup) h.elems.push_back(HVal::Str(v));
  }
  return h;
}

}  // namespace

bool Attributes::is_read_only() const { return verb == "get" || verb == "list" || verb == "watch"; }

Attributes attributes_from_sar(const JVal& sar) {
  Attributes a;
  const JVal* spec = sar.get("spec");
  if (!spec || spec->t != JVal::Obj) throw CedarError("SubjectAccessReview without spec");
  a.user_name = spec->str_or("user");
  a.uid = spec->str_or("uid");
  if (const JVal* g = spec->get("groups"))
    for (auto& x : g->arr) if (x.t == JVal::Str) a.groups.push_back(x.s);
  if (const JVal* ex = spec->get("extra")) {
    if (ex->t == JVal::Obj) {
      for (auto& kv : ex->obj) {
        std::string k = kv.first;
        for (auto& ch : k) ch = (char)std::tolower((unsigned char)ch);  // server.go:210
        std::vector<std::string> vs;
        for (auto& x : kv.second.arr) if (x.t == JVal::Str) vs.push_back(x.s);
        bool merged = false;
        for (auto& e : a.extra) if (e.first == k) { e.second = vs; merged = true; }
        if (!merged) a.extra.emplace_back(k, vs);
      }
    }
  }
  if (const JVal* ra = spec->get("resourceAttributes"); ra && ra->t == JVal::Obj) {
    a.verb = ra->str_or("verb");
    a.ns = ra->str_or("namespace");
    a.api_group = ra->str_or("group");
    a.api_version = ra->str_or("version");
    a.resource = ra->str_or("resource");
    a.subresource = ra->str_or("subresource");
    a.name = ra->str_or("name");
    a.resource_request = true;
    if (const JVal* fs = ra->get("fieldSelector"); fs && fs->t == JVal::Obj) {
      if (const JVal* reqs = fs->get("requirements"); reqs && reqs->t == JVal::Arr) {
        for (auto& r : reqs->arr) {  // server.go:262-300
          std::vector<std::string> vals;
          if (const JVal* v = r.get("values")) for (auto& x : v->arr) if (x.t == JVal::Str) vals.push_back(x.s);
          std::string op = r.str_or("operator");
          if (vals.size() > 1) continue;
          if (op == "In" && vals.size() == 1) a.field_sel.push_back({r.str_or("key"), "=", vals[0]});
          else if (op == "NotIn" && vals.size() == 1) a.field_sel.push_back({r.str_or("key"), "!=", vals[0]});
        }
      }
    }
    if (const JVal* ls = ra->get("labelSelector"); ls && ls->t == JVal::Obj) {
      if (const JVal* reqs = ls->get("requirements"); reqs && reqs->t == JVal::Arr) {
        for (auto& r : reqs->arr) {  // server.go:228-260 + labels.NewRequirement validation
          std::string op = r.str_or("operator"), key = r.str_or("key");
          std::vector<std::string> vals;
          if (const JVal* v = r.get("values")) for (auto& x : v->arr) if (x.t == JVal::Str) vals.push_back(x.s);
          std::string sop;
          if (op == "In") sop = "in";
          else if (op == "NotIn") sop = "notin";
          else if (op == "Exists") sop = "exists";
          else if (op == "DoesNotExist") sop = "!";
          else continue;
          if (!valid_label_key(key)) continue;
          if ((sop == "in" || sop == "notin") && vals.empty()) continue;
          if ((sop == "exists" || sop == "!") && !vals.empty()) continue;
          bool ok = true;
          for (auto& v : vals) if (!valid_label_value(v)) ok = false;
          if (!ok) continue;
          a.label_sel.push_back({key, sop, vals});
        }
      }
    }
  }
  if (const JVal* nra = spec->get("nonResourceAttributes"); nra && nra->t == JVal::Obj) {
    a.path = nra->str_or("path");
    a.resource_request = false;
    a.verb = nra->str_or("verb");
  }
  return a;
}

int authorize_fast_path(const Attributes& a, std::string& reason) {
  if (a.user_name == kSelf && a.is_read_only() && a.api_group == "cedar.k8s.aws" && a.resource == "policies") {
    reason = "cedar authorizer is always allowed to access policies";
    return AUTHZ_ALLOW;
  }
  if (a.user_name == kSelf && a.is_read_only() && a.api_group == "rbac.authorization.k8s.io") {
    reason = "cedar authorizer is always allowed to read RBAC policies";
    return AUTHZ_ALLOW;
  }
  if (starts(a.user_name, "system:") && !starts(a.user_name, "system:serviceaccount:") && !starts(a.user_name, "system:node:")) {
    reason.clear();
    return AUTHZ_NO_OPINION;
  }
  return -1;
}

std::string resource_request_to_path(const Attributes& a) {
  std::string base = "/api";
  if (!a.api_group.empty()) base = "/apis/" + a.api_group;
  std::string ns;
  if (!a.ns.empty()) ns = "/namespaces/" + a.ns;
  std::string resp = base + "/" + a.api_version + ns + "/" + a.resource;
  if (!a.name.empty()) resp += "/" + a.name;
  if (!a.subresource.empty()) resp += "/" + a.subresource;
  return resp;
}

void user_to_cedar(const std::string& name, const std::string& uid, const std::vector<std::string>& groups,
                   const std::vector<std::pair<std::string, std::vector<std::string>>>& extra, std::vector<EntityIn>& ents,
                   std::pair<std::string, std::string>& principal) {
  std::vector<std::pair<std::string, std::string>> parents;
  std::unordered_set<std::string> seen;  // past DEDUP_SCAN groups (a user in thousands of them)
  for (auto& g : groups) {
    EntityIn ge;
    ge.type = kGroup;
    ge.id = g;
    ge.attrs = rec({{"name", HVal::Str(g)}});
    ents.push_back(std::move(ge));
    bool fresh;
    if (parents.size() < DEDUP_SCAN) {
      fresh = std::find(parents.begin(), parents.end(), std::make_pair(std::string(kGroup), g)) == parents.end();
    } else {
      if (seen.empty())
        for (auto& q : parents) seen.insert(q.second);
      fresh = seen.insert(g).second;
    }
    if (fresh) parents.emplace_back(kGroup, g);
  }
  HVal attrs = rec({{"name", HVal::Str(name)}});
  std::string ptype = kUser;
  if (starts(name, "system:node:") && count_colons(name) == 2) {
    ptype = kNode;
    attrs.fields[0].second = HVal::Str(split_colon(name)[2]);
  }
  if (starts(name, "system:serviceaccount:") && count_colons(name) == 3) {
    ptype = kSA;
    auto parts = split_colon(name);
    attrs.fields[0].second = HVal::Str(parts[3]);
    attrs.fields.emplace_back("namespace", HVal::Str(parts[2]));
  }
  if (!extra.empty()) {
    HVal xs;
    xs.k = VK::Set;
    for (auto& kv : extra) xs.elems.push_back(rec({{"key", HVal::Str(kv.first)}, {"values", str_set(kv.second)}}));
    attrs.fields.emplace_back("extra", std::move(xs));
  }
  EntityIn pe;
  pe.type = ptype;
  pe.id = uid;
  pe.attrs = std::move(attrs);
  pe.parents = std::move(parents);
  principal = {ptype, uid};
  ents.push_back(std::move(pe));
}

void record_to_cedar(const Attributes& a, std::vector<EntityIn>& ents, RequestIn& req) {
  ents.clear();
  req.action = {kAction, a.verb};
  user_to_cedar(a.user_name, a.uid, a.groups, a.extra, ents, req.principal);
  EntityIn re;
  re.attrs.k = VK::Rec;
  if (!a.resource_request) {
    re.type = kNonResourceURL;
    re.id = a.path;
    re.attrs = rec({{"path", HVal::Str(a.path)}});
  } else if (a.verb == "impersonate") {
    // entitiy_builders.go:25-76 (unknown resources give the zero EntityUID)
    if (a.resource == "serviceaccounts") {
      re.type = kSA;
      re.id = "system:serviceaccount:" + a.ns + ":" + a.name;
      re.attrs = rec({{"name", HVal::Str(a.name)}, {"namespace", HVal::Str(a.ns)}});
    } else if (a.resource == "uids") {
      re.type = kPrincipalUID;
      re.id = a.name;
    } else if (a.resource == "users") {
      re.type = kUser;
      re.attrs = rec({{"name", HVal::Str(a.name)}});
      if (starts(a.name, "system:node:") && count_colons(a.name) == 2) {
        re.type = kNode;
        re.attrs.fields[0].second = HVal::Str(split_colon(a.name)[2]);
      }
      re.id = a.name;
    } else if (a.resource == "groups") {
      re.type = kGroup;
      re.id = a.name;
      re.attrs = rec({{"name", HVal::Str(a.name)}});
    } else if (a.resource == "userextras") {
      re.type = kExtra;
      re.id = a.subresource;
      re.attrs = rec({{"key", HVal::Str(a.subresource)}});
      if (!a.name.empty()) re.attrs.fields.emplace_back("value", HVal::Str(a.name));
    }
  } else {
    re.type = kResource;
    re.id = resource_request_to_path(a);
    re.attrs = rec({{"apiGroup", HVal::Str(a.api_group)}, {"resource", HVal::Str(a.resource)}});
    if (!a.name.empty()) re.attrs.fields.emplace_back("name", HVal::Str(a.name));
    if (!a.subresource.empty()) re.attrs.fields.emplace_back("subresource", HVal::Str(a.subresource));
    if (!a.ns.empty()) re.attrs.fields.emplace_back("namespace", HVal::Str(a.ns));
    if (!a.label_sel.empty()) {
      HVal s;
      s.k = VK::Set;
      for (auto& l : a.label_sel)
        s.elems.push_back(rec({{"key", HVal::Str(l.key)}, {"operator", HVal::Str(l.op)}, {"values", str_set(l.values)}}));
      re.attrs.fields.emplace_back("labelSelector", std::move(s));
    }
    if (!a.field_sel.empty()) {
      HVal s;
      s.k = VK::Set;
      for (auto& f : a.field_sel)
        s.elems.push_back(rec({{"field", HVal::Str(f.field)}, {"operator", HVal::Str(f.op)}, {"value", HVal::Str(f.value)}}));
      re.attrs.fields.emplace_back("fieldSelector", std::move(s));
    }
  }
  req.resource = {re.type, re.id};
  ents.push_back(std::move(re));
  req.context = HVal();
  req.context.k = VK::Rec;
}

// ---------------------------------------------------------------------------------------------
// Direct path: SubjectAccessReview bytes -> encoded request, without JVal / Attributes / HVal
// trees. It restates the same functions as above over views into the body and hands the entities
// to the shared encode_impl, so it yields the general path's exact words. Anything outside the
// plain shape (escapes, numbers, duplicate extra keys, malformed JSON, ...) returns 0 and the
// caller takes the general path.
namespace {

using SV = std::string_view;
struct Bail {};

struct Scan {
  const char* p;
  const char* e;
  void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++; }
  char peek() { ws(); if (p >= e) throw Bail{}; return *p; }
  void expect(char c) { if (peek() != c) throw Bail{}; p++; }
  SV str() {
    expect('"');
    const char* st = p;
    while (p < e && *p != '"') {
      if (*p == '\\') throw Bail{};
      p++;
    }
    if (p >= e) throw Bail{};
    return SV(st, (size_t)(p++ - st));
  }
  void lit(const char* w, size_t n) {
    if ((size_t)(e - p) < n || std::memcmp(p, w, n)) throw Bail{};
    p += n;
  }
  void skip(int depth) {
    if (depth > 200) throw Bail{};
    switch (peek()) {
      case '{': obj([&](SV) { skip(depth + 1); }); return;
      case '[': arr([&] { skip(depth + 1); }); return;
      case '"': str(); return;
      case 't': lit("true", 4); return;
      case 'f': lit("false", 5); return;
      case 'n': lit("null", 4); return;
      default: throw Bail{};  // numbers and anything else: general path
    }
  }
  template <class F>
  void obj(F&& on_key) {
    expect('{');
    if (peek() == '}') { p++; return; }
    for (;;) {
      SV k = str();
      expect(':');
      on_key(k);
      const char c = peek();
      p++;
      if (c == ',') continue;
      if (c == '}') return;
      throw Bail{};
    }
  }
  template <class F>
  void arr(F&& on_elem) {
    expect('[');
    if (peek() == ']') { p++; return; }
    for (;;) {
      on_elem();
      const char c = peek();
      p++;
      if (c == ',') continue;
      if (c == ']') return;
      throw Bail{};
    }
  }
  // str_or: the string, or "" for any other value (which is skipped)
  SV str_or_skip() {
    if (peek() == '"') return str();
    skip(1);
    return SV();
  }
  void strings(std::vector<SV>& out) {  // an array's string elements; a non-array gives none
    if (peek() != '[') { skip(1); return; }
    arr([&] { if (peek() == '"') out.push_back(str()); else skip(1); });
  }
};

struct Req3 { SV key, op; std::vector<SV> values; bool is_obj = false; };

void requirements(Scan& sc, std::vector<Req3>& out) {  // {"requirements": [{key, operator, values}]}
  if (sc.peek() != '{') { sc.skip(1); return; }
  bool seen_reqs = false;
  sc.obj([&](SV k) {
    if (k != "requirements" || seen_reqs) { sc.skip(1); return; }
    seen_reqs = true;
    if (sc.peek() != '[') { sc.skip(1); return; }
    sc.arr([&] {
      Req3 r;
      if (sc.peek() != '{') { sc.skip(1); out.push_back(std::move(r)); return; }
      r.is_obj = true;
      bool sk = false, so = false, sv = false;
      sc.obj([&](SV f) {
        if (f == "key" && !sk) { sk = true; r.key = sc.str_or_skip(); }
        else if (f == "operator" && !so) { so = true; r.op = sc.str_or_skip(); }
        else if (f == "values" && !sv) { sv = true; sc.strings(r.values); }
        else sc.skip(1);
      });
      out.push_back(std::move(r));
    });
  });
}

struct SarView {
  SV user, uid;
  std::vector<SV> groups;
  std::vector<std::pair<SV, std::vector<SV>>> extra;
  bool ra = false, nra = false;
  SV verb, ns, group, version, resource, subresource, name, path, nra_verb;
  std::vector<Req3> fsel, lsel;
};

void scan_sar(Scan& sc, SarView& v, std::deque<std::string>& arena) {
  bool spec = false;
  if (sc.peek() != '{') throw Bail{};
  sc.obj([&](SV k) {
    if (k != "spec" || spec) { sc.skip(1); return; }
    spec = true;
    if (sc.peek() != '{') throw Bail{};
    uint32_t seen = 0;
    auto first = [&](uint32_t bit) { const bool f = !(seen & bit); seen |= bit; return f; };
    sc.obj([&](SV f) {
      if (f == "user" && first(1)) v.user = sc.str_or_skip();
      else if (f == "uid" && first(2)) v.uid = sc.str_or_skip();
      else if (f == "groups" && first(4)) sc.strings(v.groups);
      else if (f == "extra" && first(8)) {
        if (sc.peek() != '{') { sc.skip(1); return; }
        sc.obj([&](SV ek) {
          SV key = ek;
          if (std::any_of(ek.begin(), ek.end(), [](char c) { return c >= 'A' && c <= 'Z'; })) {
            std::string low(ek);
            for (auto& ch : low) ch = (char)std::tolower((unsigned char)ch);  // server.go:210
            arena.push_back(std::move(low));
            key = arena.back();
          }
          for (auto& x : v.extra) if (x.first == key) throw Bail{};  // merged keys: general path
          v.extra.emplace_back(key, std::vector<SV>());
          sc.strings(v.extra.back().second);
        });
      } else if (f == "resourceAttributes" && first(16)) {
        if (sc.peek() != '{') { sc.skip(1); return; }
        v.ra = true;
        uint32_t rs = 0;
        auto rfirst = [&](uint32_t bit) { const bool fr = !(rs & bit); rs |= bit; return fr; };
        sc.obj([&](SV r) {
          if (r == "verb" && rfirst(1)) v.verb = sc.str_or_skip();
          else if (r == "namespace" && rfirst(2)) v.ns = sc.str_or_skip();
          else if (r == "group" && rfirst(4)) v.group = sc.str_or_skip();
          else if (r == "version" && rfirst(8)) v.version = sc.str_or_skip();
          else if (r == "resource" && rfirst(16)) v.resource = sc.str_or_skip();
          else if (r == "subresource" && rfirst(32)) v.subresource = sc.str_or_skip();
          else if (r == "name" && rfirst(64)) v.name = sc.str_or_skip();
          else if (r == "fieldSelector" && rfirst(128)) requirements(sc, v.fsel);
          else if (r == "labelSelector" && rfirst(256)) requirements(sc, v.lsel);
          else sc.skip(1);
        });
      } else if (f == "nonResourceAttributes" && first(32)) {
        if (sc.peek() != '{') { sc.skip(1); return; }
        v.nra = true;
        uint32_t ns = 0;
        sc.obj([&](SV r) {
          if (r == "path" && !(ns & 1)) { ns |= 1; v.path = sc.str_or_skip(); }
          else if (r == "verb" && !(ns & 2)) { ns |= 2; v.nra_verb = sc.str_or_skip(); }
          else sc.skip(1);
        });
      } else {
        sc.skip(1);
      }
    });
  });
  sc.ws();
  if (sc.p != sc.e) throw Bail{};
  if (!spec) throw Bail{};
}

// Flat value tree: strings, sets and records of the SAR entity model.
struct LTree {
  struct Node { uint8_t k; SV s; uint32_t first, n; };  // k: 0 string, 1 set, 2 record
  std::vector<Node> nodes;
  std::vector<uint32_t> kids;
  std::vector<SV> keys;  // record field names, parallel to kids
  uint32_t str(SV s) { nodes.push_back({0, s, 0, 0}); return (uint32_t)nodes.size() - 1; }
  uint32_t str_set(const std::vector<SV>& vs) {  // str_set above: duplicates dropped
    std::vector<uint32_t> el;
    for (size_t i = 0; i < vs.size(); i++) {
      bool dup = false;
      for (size_t j = 0; j < i && !dup; j++) dup = vs[j] == vs[i];
      if (!dup) el.push_back(str(vs[i]));
    }
    return set(el);
  }
  uint32_t set(const std::vector<uint32_t>& el) {
    nodes.push_back({1, SV(), (uint32_t)kids.size(), (uint32_t)el.size()});
    for (uint32_t x : el) { kids.push_back(x); keys.emplace_back(); }
    return (uint32_t)nodes.size() - 1;
  }
  uint32_t rec(std::initializer_list<std::pair<SV, uint32_t>> f) {
    nodes.push_back({2, SV(), (uint32_t)kids.size(), (uint32_t)f.size()});
    for (auto& kv : f) { kids.push_back(kv.second); keys.push_back(kv.first); }
    return (uint32_t)nodes.size() - 1;
  }
  uint32_t rec(const std::vector<std::pair<SV, uint32_t>>& f) {
    nodes.push_back({2, SV(), (uint32_t)kids.size(), (uint32_t)f.size()});
    for (auto& kv : f) { kids.push_back(kv.second); keys.push_back(kv.first); }
    return (uint32_t)nodes.size() - 1;
  }
  // emit_value_impl (compiler.cpp) for these three kinds
  void emit(uint32_t ni, std::vector<uint32_t>& out, const Image& img, EncodedRequest& E, uint32_t& w0,
            uint32_t& w1) const {
    using namespace cgi;
    const Node& nd = nodes[ni];
    if (nd.k == 0) { w0 = mk_w0(T_STR, 0); w1 = request_sid(img, E, nd.s); return; }
    if (nd.k == 1) {
      uint32_t ew[64];
      std::vector<uint32_t> big;
      uint32_t* w = nd.n <= 32 ? ew : (big.resize(2 * (size_t)nd.n), big.data());
      for (uint32_t j = 0; j < nd.n; j++) emit(kids[nd.first + j], out, img, E, w[2 * j], w[2 * j + 1]);
      const uint32_t off = (uint32_t)out.size();
      out.push_back(nd.n);
      out.insert(out.end(), w, w + 2 * (size_t)nd.n);
      w0 = mk_w0(T_SET, mk_ref(SP_HEAP, off)); w1 = nd.n;
      return;
    }
    std::array<uint32_t, 3> fw[8];  // the model's records have at most 7 fields
    if (nd.n > 8) throw CedarError("record too wide for the direct SAR path");
    for (uint32_t j = 0; j < nd.n; j++) {
      uint32_t a, b;
      emit(kids[nd.first + j], out, img, E, a, b);
      fw[j] = {request_sid(img, E, keys[nd.first + j]), a, b};
    }
    std::sort(fw, fw + nd.n, [](const std::array<uint32_t, 3>& x, const std::array<uint32_t, 3>& y) { return x[0] < y[0]; });
    const uint32_t off = (uint32_t)out.size();
    out.push_back(nd.n);
    for (uint32_t j = 0; j < nd.n; j++) { out.push_back(fw[j][0]); out.push_back(fw[j][1]); out.push_back(fw[j][2]); }
    w0 = mk_w0(T_REC, mk_ref(SP_HEAP, off)); w1 = nd.n;
  }
};

constexpr uint32_t NO_ATTRS = 0xFFFFFFFFu;

struct LEnt {
  SV type, id;
  uint32_t attrs = NO_ATTRS;  // record node, or the empty record
  std::vector<std::pair<SV, SV>> parents;
};

// the SAR's (EntityMap, Request) as an encode_impl source
struct LSrc {
  const LTree& t;
  const std::vector<LEnt>& ents;
  std::pair<SV, SV> p, a, r;
  uint32_t n_ents() const { return (uint32_t)ents.size(); }
  SV type(uint32_t i) const { return ents[i].type; }
  SV id(uint32_t i) const { return ents[i].id; }
  uint32_t n_parents(uint32_t i) const { return (uint32_t)ents[i].parents.size(); }
  std::pair<SV, SV> parent(uint32_t i, uint32_t k) const { return ents[i].parents[k]; }
  std::pair<SV, SV> principal() const { return p; }
  std::pair<SV, SV> action() const { return a; }
  std::pair<SV, SV> resource() const { return r; }
  void emit_ctx(std::vector<uint32_t>& out, const Image&, EncodedRequest&, uint32_t& w0, uint32_t& w1) const {
    enc::emit_empty_record(out, w0, w1);
  }
  void emit_attrs(uint32_t i, std::vector<uint32_t>& out, const Image& img, EncodedRequest& E, uint32_t& w0,
                  uint32_t& w1) const {
    if (ents[i].attrs == NO_ATTRS) enc::emit_empty_record(out, w0, w1);
    else t.emit(ents[i].attrs, out, img, E, w0, w1);
  }
};

bool sv_starts(SV s, SV p) { return s.substr(0, p.size()) == p; }

// i-th ':'-separated field of s
SV colon_field(SV s, int i) {
  size_t st = 0;
  for (int k = 0; k < i; k++) st = s.find(':', st) + 1;
  const size_t e = s.find(':', st);
  return s.substr(st, e == SV::npos ? SV::npos : e - st);
}

}  // namespace

int encode_sar_direct(const Image& img, const char* json, size_t n, EncodedRequest& out, int& fast, std::string& reason) {
  SarView v;
  std::deque<std::string> arena;
  try {
    Scan sc{json, json + n};
    scan_sar(sc, v, arena);
  } catch (const Bail&) {
    return 0;
  }
  const bool resource_request = v.nra ? false : v.ra;
  const SV verb = v.nra ? v.nra_verb : v.verb;
  const SV api_group = v.group, resource = v.resource;
  // Authorize fast paths (authorize_fast_path above)
  const bool ro = verb == "get" || verb == "list" || verb == "watch";
  if (v.user == kSelf && ro && api_group == "cedar.k8s.aws" && resource == "policies") {
    fast = AUTHZ_ALLOW;
    reason = "cedar authorizer is always allowed to access policies";
    return 2;
  }
  if (v.user == kSelf && ro && api_group == "rbac.authorization.k8s.io") {
    fast = AUTHZ_ALLOW;
    reason = "cedar authorizer is always allowed to read RBAC policies";
    return 2;
  }
  if (sv_starts(v.user, "system:") && !sv_starts(v.user, "system:serviceaccount:") && !sv_starts(v.user, "system:node:")) {
    fast = AUTHZ_NO_OPINION;
    reason.clear();
    return 2;
  }
  // RecordToCedarResource / UserToCedarEntity (record_to_cedar, user_to_cedar above)
  LTree t;
  std::vector<LEnt> ents;
  ents.reserve(v.groups.size() + 2);
  LEnt pe;
  std::unordered_set<SV> seen;  // past DEDUP_SCAN groups
  for (SV g : v.groups) {
    LEnt ge;
    ge.type = kGroup;
    ge.id = g;
    ge.attrs = t.rec({{"name", t.str(g)}});
    ents.push_back(std::move(ge));
    const std::pair<SV, SV> pu{kGroup, g};
    bool fresh;
    if (pe.parents.size() < DEDUP_SCAN) {
      fresh = std::find(pe.parents.begin(), pe.parents.end(), pu) == pe.parents.end();
    } else {
      if (seen.empty())
        for (auto& q : pe.parents) seen.insert(q.second);
      fresh = seen.insert(g).second;
    }
    if (fresh) pe.parents.push_back(pu);
  }
  SV ptype = kUser, pname = v.user, pns;
  bool sa = false;
  const auto colons = std::count(v.user.begin(), v.user.end(), ':');
  if (sv_starts(v.user, "system:node:") && colons == 2) { ptype = kNode; pname = colon_field(v.user, 2); }
  if (sv_starts(v.user, "system:serviceaccount:") && colons == 3) {
    ptype = kSA;
    sa = true;
    pname = colon_field(v.user, 3);
    pns = colon_field(v.user, 2);
  }
  {
    std::vector<std::pair<SV, uint32_t>> f{{"name", t.str(pname)}};
    if (sa) f.emplace_back("namespace", t.str(pns));
    if (!v.extra.empty()) {
      std::vector<uint32_t> xs;
      for (auto& kv : v.extra) xs.push_back(t.rec({{"key", t.str(kv.first)}, {"values", t.str_set(kv.second)}}));
      f.emplace_back("extra", t.set(xs));
    }
    pe.attrs = t.rec(f);
  }
  pe.type = ptype;
  pe.id = v.uid;
  ents.push_back(std::move(pe));
  LEnt re;
  if (!resource_request) {
    re.type = kNonResourceURL;
    re.id = v.path;
    re.attrs = t.rec({{"path", t.str(v.path)}});
  } else if (verb == "impersonate") {
    if (resource == "serviceaccounts") {
      re.type = kSA;
      arena.push_back("system:serviceaccount:" + std::string(v.ns) + ":" + std::string(v.name));
      re.id = arena.back();
      re.attrs = t.rec({{"name", t.str(v.name)}, {"namespace", t.str(v.ns)}});
    } else if (resource == "uids") {
      re.type = kPrincipalUID;
      re.id = v.name;
    } else if (resource == "users") {
      re.type = kUser;
      SV nm = v.name;
      if (sv_starts(v.name, "system:node:") && std::count(v.name.begin(), v.name.end(), ':') == 2) {
        re.type = kNode;
        nm = colon_field(v.name, 2);
      }
      re.attrs = t.rec({{"name", t.str(nm)}});
      re.id = v.name;
    } else if (resource == "groups") {
      re.type = kGroup;
      re.id = v.name;
      re.attrs = t.rec({{"name", t.str(v.name)}});
    } else if (resource == "userextras") {
      re.type = kExtra;
      re.id = v.subresource;
      std::vector<std::pair<SV, uint32_t>> f{{"key", t.str(v.subresource)}};
      if (!v.name.empty()) f.emplace_back("value", t.str(v.name));
      re.attrs = t.rec(f);
    }
  } else {
    re.type = kResource;
    {  // resource_request_to_path
      std::string path = v.group.empty() ? std::string("/api") : "/apis/" + std::string(v.group);
      path += '/';
      path += v.version;
      if (!v.ns.empty()) { path += "/namespaces/"; path += v.ns; }
      path += '/';
      path += v.resource;
      if (!v.name.empty()) { path += '/'; path += v.name; }
      if (!v.subresource.empty()) { path += '/'; path += v.subresource; }
      arena.push_back(std::move(path));
      re.id = arena.back();
    }
    std::vector<std::pair<SV, uint32_t>> f{{"apiGroup", t.str(v.group)}, {"resource", t.str(v.resource)}};
    if (!v.name.empty()) f.emplace_back("name", t.str(v.name));
    if (!v.subresource.empty()) f.emplace_back("subresource", t.str(v.subresource));
    if (!v.ns.empty()) f.emplace_back("namespace", t.str(v.ns));
    std::vector<uint32_t> ls;
    for (auto& r : v.lsel) {  // attributes_from_sar's labelSelector filter
      if (!r.is_obj) continue;
      SV op;
      if (r.op == "In") op = "in";
      else if (r.op == "NotIn") op = "notin";
      else if (r.op == "Exists") op = "exists";
      else if (r.op == "DoesNotExist") op = "!";
      else continue;
      if (!valid_label_key(std::string(r.key))) continue;
      if ((op == "in" || op == "notin") && r.values.empty()) continue;
      if ((op == "exists" || op == "!") && !r.values.empty()) continue;
      bool ok = true;
      for (SV x : r.values) if (!valid_label_value(std::string(x))) ok = false;
      if (!ok) continue;
      ls.push_back(t.rec({{"key", t.str(r.key)}, {"operator", t.str(op)}, {"values", t.str_set(r.values)}}));
    }
    if (!ls.empty()) f.emplace_back("labelSelector", t.set(ls));
    std::vector<uint32_t> fs;
    for (auto& r : v.fsel) {
      if (!r.is_obj || r.values.size() > 1) continue;
      SV op;
      if (r.op == "In" && r.values.size() == 1) op = "=";
      else if (r.op == "NotIn" && r.values.size() == 1) op = "!=";
      else continue;
      fs.push_back(t.rec({{"field", t.str(r.key)}, {"operator", t.str(op)}, {"value", t.str(r.values[0])}}));
    }
    if (!fs.empty()) f.emplace_back("fieldSelector", t.set(fs));
    re.attrs = t.rec(f);
  }
  const std::pair<SV, SV> ru{re.type, re.id};
  ents.push_back(std::move(re));
  const std::pair<SV, SV> pu{ptype, v.uid}, au{kAction, verb};
  encode_impl(img, LSrc{t, ents, pu, au, ru}, out);
  return 1;
}

}  // namespace cg
