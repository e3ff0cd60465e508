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
#include <cctype>

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
  for (auto& g : groups) {
    EntityIn ge;
    ge.type = kGroup;
    ge.id = g;
    ge.attrs = rec({{"name", HVal::Str(g)}});
    ents.push_back(std::move(ge));
    if (std::find(parents.begin(), parents.end(), std::make_pair(std::string(kGroup), g)) == parents.end())
      parents.emplace_back(kGroup, g);
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

}  // namespace cg
