// Admission webhook model: AdmissionReview request -> (EntityMap, Request), the C++ restatement of
//   cedarHandler.Handle / review                        internal/server/admission/handler.go:43-167
//   CedarPrincipalEntitesFromAdmissionRequest           internal/server/entities/admission.go:56-60
//   cedarResourceEntityFromAdmissionRequest             admission.go:123-158
//   UnstructuredToRecord / walkObject                   admission.go:160-369
//   AdmissionActionEntities / CedarActionEntity...      admission.go:40-53, 62-77
//   UserInfoWrapper.GetUID (uid defaults to username)   internal/server/entities/user.go:19-25
//
// Where the reference depends on Go map iteration order (the order of key/value set elements, and
// which entries precede the first non-string value that stops a key/value map), this walks the
// object in document order; JSON objects with a repeated key keep the last value, as Go's
// decoder does. A null inside a list (cedar.NewSet over a nil Value in the reference) is reported
// as an error here.
#include <algorithm>

#include "admission.h"

namespace cg {

namespace {

const char* kAdmAction = "k8s::admission::Action";

// knownKeyValueStringMapAttributes (admission.go:197-236): group -> version -> kind -> keys
struct KV { const char *g, *v, *k; std::vector<const char*> keys; };
const std::vector<KV>& kv_string_maps() {
  static const std::vector<KV> t = {
      {"core", "v1", "ConfigMap", {"data", "binaryData"}},
      {"core", "v1", "CSIPersistentVolumeSource", {"volumeAttributes"}},
      {"core", "v1", "CSIVolumeSource", {"volumeAttributes"}},
      {"core", "v1", "FlexPersistentVolumeSource", {"options"}},
      {"core", "v1", "FlexVolumeSource", {"options"}},
      {"core", "v1", "PersistentVolumeClaimStatus", {"allocatedResourceStatuses"}},
      {"core", "v1", "Pod", {"nodeSelector"}},
      {"core", "v1", "ReplicationController", {"selector"}},
      {"core", "v1", "Secret", {"data", "stringData"}},
      {"core", "v1", "Service", {"selector"}},
      {"discovery", "v1", "Endpoint", {"deprecatedTopology"}},
      {"node", "v1", "Scheduling", {"nodeSelectors"}},
      {"storage", "v1", "StorageClass", {"parameters"}},
      {"storage", "v1", "VolumeAttachmentStatus", {"attachmentMetadata"}},
      {"meta", "v1", "LabelSelector", {"matchLabels"}},
      {"meta", "v1", "ObjectMeta", {"annotations", "labels"}},
  };
  return t;
}
// knownKeyValueStringSliceMapAttributes (admission.go:266-283)
const std::vector<KV>& kv_slice_maps() {
  static const std::vector<KV> t = {
      {"authentication", "v1", "UserInfo", {"extra"}},
      {"authorization", "v1", "SubjectAccessReview", {"extra"}},
      {"certificates", "v1", "CertificateSigningRequest", {"extra"}},
  };
  return t;
}
bool kv_match(const std::vector<KV>& t, const std::string& g, const std::string& v, const std::string& k,
              const std::string& key) {
  for (auto& e : t)
    if (g == e.g && v == e.v && k == e.k)
      for (auto* n : e.keys)
        if (key == n) return true;
  return false;
}

struct WalkError : std::exception {
  std::string m;
  explicit WalkError(std::string s) : m(std::move(s)) {}
  const char* what() const noexcept override { return m.c_str(); }
};

// (key, value) entries of a JSON object with Go's last-wins for repeated keys, in the order of
// each key's first appearance
std::vector<const std::pair<std::string, JVal>*> entries(const JVal& o) {
  std::vector<const std::pair<std::string, JVal>*> out;
  out.reserve(o.obj.size());
  for (auto& kv : o.obj) {
    bool dup = false;
    for (auto*& e : out)
      if (e->first == kv.first) { e = &kv; dup = true; break; }
    if (!dup) out.push_back(&kv);
  }
  return out;
}

HVal kv_record(const std::string& k, HVal v, const char* vname) {
  HVal r;
  r.k = VK::Rec;
  r.fields.emplace_back("key", HVal::Str(k));
  r.fields.emplace_back(vname, std::move(v));
  return r;
}

// string key/value map -> Set<{key, value}>; stops at the first non-string value (admission.go:215)
HVal kv_string_set(const JVal& o) {
  if (o.t != JVal::Obj) throw WalkError("key/value map attribute is not an object");
  HVal s;
  s.k = VK::Set;
  for (auto* e : entries(o)) {
    if (e->second.t != JVal::Str) break;
    s.elems.push_back(kv_record(e->first, HVal::Str(e->second.s), "value"));
  }
  return s;
}

const char* go_type(const JVal& v) {
  switch (v.t) {
    case JVal::Num: return "float64";
    case JVal::Str: return "string";
    default: return "unknown";
  }
}

// walkObject (admission.go:184-369). Returns false for the reference's nil (skipped) value.
bool walk(int depth, const std::string& g, const std::string& ver, const std::string& kind, const std::string& key,
          const JVal& o, HVal& out) {
  if (depth == 0) throw WalkError("max depth reached");
  if (o.t == JVal::Null) return false;
  if (kv_match(kv_string_maps(), g, ver, kind, key)) { out = kv_string_set(o); return true; }
  if (kv_match(kv_slice_maps(), g, ver, kind, key)) {
    // the reference asserts each value to []string, which a decoded JSON array ([]interface{})
    // never is: the loop stops at the first entry, leaving an empty set
    if (o.t != JVal::Obj) throw WalkError("key/value slice map attribute is not an object");
    out = HVal();
    out.k = VK::Set;
    return true;
  }
  if (o.t == JVal::Obj && (key == "labels" || key == "annotations")) { out = kv_string_set(o); return true; }
  switch (o.t) {
    case JVal::Obj: {
      HVal r;
      r.k = VK::Rec;
      for (auto* e : entries(o)) {
        HVal v;
        if (walk(depth - 1, g, ver, kind, e->first, e->second, v)) r.fields.emplace_back(e->first, std::move(v));
      }
      if (r.fields.empty()) return false;  // empty records are skipped
      out = std::move(r);
      return true;
    }
    case JVal::Arr: {
      HVal s;
      s.k = VK::Set;
      for (auto& x : o.arr) {
        HVal v;
        if (!walk(depth - 1, g, ver, kind, key, x, v)) throw WalkError("unsupported nil value in a list");
        s.elems.push_back(std::move(v));
      }
      out = std::move(s);
      return true;
    }
    case JVal::Str: {
      static const char* ip_keys[] = {"podIP", "clusterIP", "loadBalancerIP", "hostIP", "ip", "podIPs", "hostIPs"};
      for (auto* k : ip_keys)
        if (key == k) {
          IpVal ip;
          if (parse_ip(o.s, &ip)) {
            out = HVal();
            out.k = VK::Ip;
            out.ip = ip;
            return true;
          }
          break;
        }
      out = HVal::Str(o.s);
      return true;
    }
    case JVal::Int: out = HVal::Long(o.i); return true;
    case JVal::Bool: out = HVal::Bool(o.b); return true;
    default: throw WalkError(std::string("unsupported type ") + go_type(o));
  }
}

std::string str_of(const JVal* o, const char* key) { return o ? o->str_or(key) : std::string(); }

struct ResourceError : std::exception {
  std::string m;
  explicit ResourceError(std::string s) : m(std::move(s)) {}
  const char* what() const noexcept override { return m.c_str(); }
};

}  // namespace

AdmissionRequest admission_request_from_json(const JVal& v) {
  const JVal* r = v.get("request");
  const JVal& q = (r && r->t == JVal::Obj) ? *r : v;
  if (q.t != JVal::Obj) throw CedarError("admission review without a request object");
  AdmissionRequest a;
  a.uid = q.str_or("uid");
  a.operation = q.str_or("operation");
  a.name = q.str_or("name");
  a.ns = q.str_or("namespace");
  a.sub_resource = q.str_or("subResource");
  const JVal* kind = q.get("kind");
  a.kind_group = str_of(kind, "group");
  a.kind_version = str_of(kind, "version");
  a.kind = str_of(kind, "kind");
  const JVal* res = q.get("resource");
  a.res_group = str_of(res, "group");
  a.res_version = str_of(res, "version");
  a.resource = str_of(res, "resource");
  if (const JVal* u = q.get("userInfo"); u && u->t == JVal::Obj) {
    a.username = u->str_or("username");
    a.user_uid = u->str_or("uid");
    if (const JVal* g = u->get("groups"))
      for (auto& x : g->arr)
        if (x.t == JVal::Str) a.groups.push_back(x.s);
    if (const JVal* ex = u->get("extra"); ex && ex->t == JVal::Obj)
      for (auto* e : entries(*ex)) {
        std::vector<std::string> vs;
        for (auto& x : e->second.arr)
          if (x.t == JVal::Str) vs.push_back(x.s);
        a.extra.emplace_back(e->first, std::move(vs));
      }
  }
  const JVal* ob = q.get("object");
  const JVal* old = q.get("oldObject");
  a.has_object = ob && ob->t != JVal::Null;
  a.has_old = old && old->t != JVal::Null;
  if (a.has_object) a.object = *ob;
  if (a.has_old) a.old_object = *old;
  return a;
}

int admission_to_cedar(const AdmissionRequest& a, std::vector<EntityIn>& ents, RequestIn& req, std::string& err) {
  ents.clear();
  // Handle: skipped namespaces answer allowed without evaluation (handler.go:44-47)
  if (a.ns == "kube-system" || a.ns == "cedar-k8s-authz-system") return ADM_SKIP;
  // principal entities (UserInfoWrapper: uid defaults to the username)
  user_to_cedar(a.username, a.user_uid.empty() ? a.username : a.user_uid, a.groups, a.extra, ents, req.principal);
  const std::string group = a.res_group.empty() ? std::string("core") : a.res_group;
  const std::string rtype = group + "::" + a.kind_version + "::" + a.kind;
  Attributes at;  // AdmissionRequestToAuthorizerAttribute -> ResourceRequestToPath
  at.api_group = a.res_group;
  at.api_version = a.res_version;
  at.ns = a.ns;
  at.resource = a.resource;
  at.name = a.name;
  at.subresource = a.sub_resource;
  const std::string rid = resource_request_to_path(at);
  auto entity = [&](bool present, const JVal& raw) {
    if (!present) throw ResourceError("error getting unstructured resource " + a.name + ": unstructured data is nil");
    if (raw.t != JVal::Obj)
      throw ResourceError("error getting unstructured resource " + a.name + ": error decoding generator resource: not an object");
    const JVal* kd = raw.get("kind");
    if (!kd || kd->t != JVal::Str || kd->s.empty())
      throw ResourceError("error getting unstructured resource " + a.name + ": Object 'Kind' is missing");
    EntityIn e;
    e.type = rtype;
    e.id = rid;
    e.attrs.k = VK::Rec;
    try {
      for (auto* kv : entries(raw)) {  // UnstructuredToRecord (admission.go:160-182)
        if (kv->second.t == JVal::Null) continue;
        HVal v;
        if (walk(32, group, a.kind_version, a.kind, kv->first, kv->second, v)) e.attrs.fields.emplace_back(kv->first, std::move(v));
      }
    } catch (const WalkError& w) {
      throw ResourceError(std::string("error converting unstructured object to Cedar entity: ") + w.what());
    }
    return e;
  };
  EntityIn res, old;
  bool have_old = false;
  try {
    if (a.operation == "DELETE") {
      try {
        res = entity(a.has_old, a.old_object);
      } catch (const ResourceError& e) {
        err = std::string("error converting oldObject to Cedar entity: ") + e.what();
        return ADM_ERROR;
      }
    } else {
      try {
        res = entity(a.has_object, a.object);
      } catch (const ResourceError& e) {
        err = std::string("error converting request to Cedar resource entity: ") + e.what();
        return ADM_ERROR;
      }
    }
    if (a.has_old && a.operation != "DELETE") {
      try {
        old = entity(true, a.old_object);
      } catch (const ResourceError& e) {
        err = std::string("error converting oldObject to Cedar entity: ") + e.what();
        return ADM_ERROR;
      }
      old.id = a.uid;  // handler.go:114-119
      HVal ref = HVal::Ent(old.type, old.id);
      bool set = false;
      for (auto& f : res.attrs.fields)
        if (f.first == "oldObject") { f.second = ref; set = true; }
      if (!set) res.attrs.fields.emplace_back("oldObject", ref);
      have_old = true;
    }
  } catch (const ResourceError& e) {
    err = e.what();
    return ADM_ERROR;
  }
  std::string op;
  if (a.operation == "CONNECT") op = "connect";
  else if (a.operation == "CREATE") op = "create";
  else if (a.operation == "UPDATE") op = "update";
  else if (a.operation == "DELETE") op = "delete";
  else {
    err = "error converting request to Cedar action entity: unsupported operation " + a.operation;
    return ADM_ERROR;
  }
  HVal old_attrs;
  if (have_old) {
    old_attrs = old.attrs;
    ents.push_back(std::move(old));
  }
  req.resource = {res.type, res.id};
  ents.push_back(std::move(res));
  // AdmissionActionEntities (IDs are the whole quoted UID string: a reference quirk)
  const std::string all = std::string(kAdmAction) + "::\"all\"";
  EntityIn ae;
  ae.type = kAdmAction;
  ae.id = all;
  ae.attrs.k = VK::Rec;
  ents.push_back(ae);
  for (const char* x : {"connect", "create", "update", "delete"}) {
    EntityIn e;
    e.type = kAdmAction;
    e.id = std::string(kAdmAction) + "::\"" + x + "\"";
    e.attrs.k = VK::Rec;
    e.parents.emplace_back(kAdmAction, all);
    ents.push_back(std::move(e));
  }
  req.action = {kAdmAction, op};
  req.context = HVal();
  req.context.k = VK::Rec;
  if (have_old) req.context.fields.emplace_back("oldObject", std::move(old_attrs));
  return ADM_EVAL;
}

}  // namespace cg
