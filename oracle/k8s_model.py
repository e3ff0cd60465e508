"""CPU restatement of the reference's Kubernetes -> Cedar request model — TEST INFRASTRUCTURE ONLY.

Restates (file:line in /root/reference):
* `GetAuthorizerAttributes` / `convertExtraForAuthorizerAttributes` — internal/server/server.go:163-214
* `RecordToCedarResource` — internal/server/authorizer/authorizer.go:89-111
* `ActionEntities`, `ImpersonatedResourceToCedarEntity`, `NonResourceToCedarEntity`,
  `ResourceToCedarEntity` — internal/server/authorizer/entitiy_builders.go:13-143
* `UserToCedarEntity` — internal/server/entities/user.go:35-100
* `ResourceRequestToPath` — internal/server/entities/authorization.go:13-30
* `cedarWebhookAuthorizer.Authorize` + `diagnosticToReason` — authorizer.go:36-85,113-124
* `UnstructuredToRecord` / `walkObject` — internal/server/entities/admission.go:160-369
* admission `review` / `Handle` — internal/server/admission/handler.go:43-167
"""
from __future__ import annotations

import ipaddress
import re
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import cedar_oracle as _co
from cedar_oracle import (CSet, Diagnostic, Entity, EntityMap, EntityUID, IPAddr, Long, PolicySet, Record,
                          Request, parse_policies, tiered_is_authorized)

# schema constants (internal/schema/authorization.go:9-19, user_entities.go:7-20, admission_actions.go:7-15)
ACTION_TYPE = "k8s::Action"
PRINCIPAL_UID_TYPE = "k8s::PrincipalUID"
NON_RESOURCE_URL_TYPE = "k8s::NonResourceURL"
RESOURCE_TYPE = "k8s::Resource"
USER_TYPE = "k8s::User"
GROUP_TYPE = "k8s::Group"
EXTRA_TYPE = "k8s::Extra"
SA_TYPE = "k8s::ServiceAccount"
NODE_TYPE = "k8s::Node"
ADMISSION_ACTION_TYPE = "k8s::admission::Action"
CEDAR_AUTHORIZER_IDENTITY = "system:authorizer:cedar-authorizer"  # options.go:15

DECISION_DENY, DECISION_ALLOW, DECISION_NO_OPINION = 0, 1, 2  # k8s authorizer.Decision values


@dataclass
class UserInfo:
    name: str = ""
    uid: str = ""
    groups: List[str] = field(default_factory=list)
    extra: Dict[str, List[str]] = field(default_factory=dict)


@dataclass
class LabelRequirement:
    key: str
    operator: str
    values: List[str]


@dataclass
class FieldRequirement:
    field: str
    operator: str
    value: str


@dataclass
class Attributes:
    """k8s.io/apiserver authorizer.AttributesRecord subset used by the webhook."""
    user: UserInfo = field(default_factory=UserInfo)
    verb: str = ""
    namespace: str = ""
    api_group: str = ""
    api_version: str = ""
    resource: str = ""
    subresource: str = ""
    name: str = ""
    resource_request: bool = False
    path: str = ""
    label_selector: List[LabelRequirement] = field(default_factory=list)
    field_selector: List[FieldRequirement] = field(default_factory=list)

    def is_read_only(self) -> bool:
        return self.verb in ("get", "list", "watch")


def resource_request_to_path(a: Attributes) -> str:
    """entities/authorization.go:13-30"""
    base = "/api"
    if a.api_group != "":
        base = "/apis/" + a.api_group
    ns = ""
    if a.namespace != "":
        ns = "/namespaces/" + a.namespace
    resp = f"{base}/{a.api_version}{ns}/{a.resource}"
    if a.name != "":
        resp += "/" + a.name
    if a.subresource != "":
        resp += "/" + a.subresource
    return resp


def user_to_cedar_entity(u: UserInfo) -> Tuple[EntityUID, EntityMap]:
    """entities/user.go:35-100"""
    resp: EntityMap = {}
    group_uids = []
    for g in u.groups:
        guid = EntityUID(GROUP_TYPE, g)
        resp[guid] = Entity(guid, Record({"name": g}), ())
        group_uids.append(guid)
    attrs = {"name": u.name}
    ptype = USER_TYPE
    if u.name.startswith("system:node:") and u.name.count(":") == 2:
        ptype = NODE_TYPE
        attrs["name"] = u.name.split(":")[2]
    if u.name.startswith("system:serviceaccount:") and u.name.count(":") == 3:
        ptype = SA_TYPE
        parts = u.name.split(":")
        attrs["namespace"] = parts[2]
        attrs["name"] = parts[3]
    extra_vals = []
    for k, vs in u.extra.items():
        extra_vals.append(Record({"key": k, "values": CSet(list(vs))}))
    if extra_vals:
        attrs["extra"] = CSet(extra_vals)
    puid = EntityUID(ptype, u.uid)
    # Parents is a set: duplicates collapse, order irrelevant
    parents = tuple(dict.fromkeys(group_uids))
    resp[puid] = Entity(puid, Record(attrs), parents)
    return puid, resp


def impersonated_resource_to_entity(a: Attributes) -> Entity:
    """entitiy_builders.go:25-76"""
    attrs: Dict[str, object] = {}
    uid = EntityUID("", "")
    r = a.resource
    if r == "serviceaccounts":
        uid = EntityUID(SA_TYPE, "system:serviceaccount:" + a.namespace + ":" + a.name)
        attrs["name"] = a.name
        attrs["namespace"] = a.namespace
    elif r == "uids":
        uid = EntityUID(PRINCIPAL_UID_TYPE, a.name)
    elif r == "users":
        t = USER_TYPE
        attrs["name"] = a.name
        if a.name.startswith("system:node:") and a.name.count(":") == 2:
            t = NODE_TYPE
            attrs["name"] = a.name.split(":")[2]
        uid = EntityUID(t, a.name)
    elif r == "groups":
        uid = EntityUID(GROUP_TYPE, a.name)
        attrs["name"] = a.name
    elif r == "userextras":
        uid = EntityUID(EXTRA_TYPE, a.subresource)
        attrs["key"] = a.subresource
        if a.name != "":
            attrs["value"] = a.name
    return Entity(uid, Record(attrs), ())


def non_resource_to_entity(a: Attributes) -> Entity:
    """entitiy_builders.go:78-88"""
    return Entity(EntityUID(NON_RESOURCE_URL_TYPE, a.path), Record({"path": a.path}), ())


def resource_to_entity(a: Attributes) -> Entity:
    """entitiy_builders.go:90-143"""
    attrs: Dict[str, object] = {"apiGroup": a.api_group, "resource": a.resource}
    if a.name != "":
        attrs["name"] = a.name
    if a.subresource != "":
        attrs["subresource"] = a.subresource
    if a.namespace != "":
        attrs["namespace"] = a.namespace
    if a.label_selector:
        attrs["labelSelector"] = CSet([Record({"key": s.key, "operator": s.operator, "values": CSet(list(s.values))})
                                       for s in a.label_selector])
    if a.field_selector:
        attrs["fieldSelector"] = CSet([Record({"field": s.field, "operator": s.operator, "value": s.value})
                                       for s in a.field_selector])
    return Entity(EntityUID(RESOURCE_TYPE, resource_request_to_path(a)), Record(attrs), ())


def record_to_cedar_resource(a: Attributes) -> Tuple[EntityMap, Request]:
    """authorizer.go:89-111"""
    action = EntityUID(ACTION_TYPE, a.verb)
    puid, em = user_to_cedar_entity(a.user)
    if a.resource_request:
        ent = impersonated_resource_to_entity(a) if a.verb == "impersonate" else resource_to_entity(a)
    else:
        ent = non_resource_to_entity(a)
    em = dict(em)
    em[ent.uid] = ent
    return em, Request(puid, action, ent.uid, Record({}))


def diagnostic_to_reason(d: Diagnostic) -> str:
    """authorizer.go:113-124"""
    if not d.reasons:
        return ""
    return d.to_go_json()


def authorize(tiers: List[PolicySet], a: Attributes, stores_loaded: bool = True, static=None) -> Tuple[int, str]:
    """cedarWebhookAuthorizer.Authorize (authorizer.go:36-85). Returns (decision, reason).
    `static`: an EntityMap of static entities merged into the request's (merge_static_entities)."""
    name = a.user.name
    if name == CEDAR_AUTHORIZER_IDENTITY and a.is_read_only() and a.api_group == "cedar.k8s.aws" and a.resource == "policies":
        return DECISION_ALLOW, "cedar authorizer is always allowed to access policies"
    if name == CEDAR_AUTHORIZER_IDENTITY and a.is_read_only() and a.api_group == "rbac.authorization.k8s.io":
        return DECISION_ALLOW, "cedar authorizer is always allowed to read RBAC policies"
    if name.startswith("system:") and not name.startswith("system:serviceaccount:") and not name.startswith("system:node:"):
        return DECISION_NO_OPINION, ""
    if not stores_loaded:
        return DECISION_NO_OPINION, ""
    em, req = record_to_cedar_resource(a)
    ok, diag, _ = tiered_is_authorized(tiers, _co.merge_static_entities(em, static), req)
    if ok:
        return DECISION_ALLOW, diagnostic_to_reason(diag)
    if diag.reasons:
        return DECISION_DENY, diagnostic_to_reason(diag)
    return DECISION_NO_OPINION, ""


def attributes_from_sar(sar: dict) -> Attributes:
    """GetAuthorizerAttributes (server.go:163-214) over a SubjectAccessReview JSON object."""
    spec = sar.get("spec", {})
    extra = None
    if spec.get("extra") is not None:
        extra = {k.lower(): list(v) for k, v in spec["extra"].items()}
    a = Attributes(user=UserInfo(spec.get("user", ""), spec.get("uid", ""), list(spec.get("groups") or []), extra or {}))
    ra = spec.get("resourceAttributes")
    if ra is not None:
        a.verb = ra.get("verb", "")
        a.namespace = ra.get("namespace", "")
        a.api_group = ra.get("group", "")
        a.api_version = ra.get("version", "")
        a.resource = ra.get("resource", "")
        a.subresource = ra.get("subresource", "")
        a.name = ra.get("name", "")
        a.resource_request = True
        fs = (ra.get("fieldSelector") or {}).get("requirements")
        if fs:  # fieldSelectorAsSelector (server.go:262-300): invalid requirements are dropped
            for r in fs:
                vals = list(r.get("values") or [])
                if len(vals) > 1:
                    continue
                if r.get("operator") == "In" and len(vals) == 1:
                    a.field_selector.append(FieldRequirement(r.get("key", ""), "=", vals[0]))
                elif r.get("operator") == "NotIn" and len(vals) == 1:
                    a.field_selector.append(FieldRequirement(r.get("key", ""), "!=", vals[0]))
        ls = (ra.get("labelSelector") or {}).get("requirements")
        if ls:  # labelSelectorAsSelector (server.go:228-260) + labels.NewRequirement validation
            for r in ls:
                op = _sel_op(r.get("operator", ""))
                key = r.get("key", "")
                vals = list(r.get("values") or [])
                if op not in ("in", "notin", "exists", "!") or not _valid_label_key(key):
                    continue
                if op in ("in", "notin") and not vals:
                    continue
                if op in ("exists", "!") and vals:
                    continue
                if not all(_valid_label_value(v) for v in vals):
                    continue
                a.label_selector.append(LabelRequirement(key, op, vals))
    nra = spec.get("nonResourceAttributes")
    if nra is not None:
        a.path = nra.get("path", "")
        a.resource_request = False
        a.verb = nra.get("verb", "")
    return a


def _sel_op(op: str) -> str:
    # metav1 LabelSelectorOperator -> selection.Operator strings
    return {"In": "in", "NotIn": "notin", "Exists": "exists", "DoesNotExist": "!"}.get(op, "?")


_NAME63 = re.compile(r"^[A-Za-z0-9]([-A-Za-z0-9_.]*[A-Za-z0-9])?$")
_DNS_LABEL = re.compile(r"^[a-z0-9]([-a-z0-9]*[a-z0-9])?$")


def _valid_label_value(v: str) -> bool:
    return v == "" or (len(v) <= 63 and bool(_NAME63.match(v)))


def _valid_label_key(k: str) -> bool:
    """k8s.io/apimachinery IsQualifiedName."""
    parts = k.split("/")
    if len(parts) == 1:
        return len(k) <= 63 and bool(_NAME63.match(k))
    if len(parts) != 2:
        return False
    prefix, name = parts
    if not prefix or len(prefix) > 253 or not all(_DNS_LABEL.match(x) and len(x) <= 63 for x in prefix.split(".")):
        return False
    return len(name) <= 63 and bool(_NAME63.match(name))


# ---------------------------------------------------------------------------------------------
# Admission (entities/admission.go, admission/handler.go)
# ---------------------------------------------------------------------------------------------

ADMISSION_ACTION_IDS = [f'{ADMISSION_ACTION_TYPE}::"{x}"' for x in ("connect", "create", "update", "delete")]

_KV_STRING_MAP = {
    "core": {"v1": {"ConfigMap": ["data", "binaryData"], "CSIPersistentVolumeSource": ["volumeAttributes"],
                    "CSIVolumeSource": ["volumeAttributes"], "FlexPersistentVolumeSource": ["options"],
                    "FlexVolumeSource": ["options"], "PersistentVolumeClaimStatus": ["allocatedResourceStatuses"],
                    "Pod": ["nodeSelector"], "ReplicationController": ["selector"],
                    "Secret": ["data", "stringData"], "Service": ["selector"]}},
    "discovery": {"v1": {"Endpoint": ["deprecatedTopology"]}},
    "node": {"v1": {"Scheduling": ["nodeSelectors"]}},
    "storage": {"v1": {"StorageClass": ["parameters"], "VolumeAttachmentStatus": ["attachmentMetadata"]}},
    "meta": {"v1": {"LabelSelector": ["matchLabels"], "ObjectMeta": ["annotations", "labels"]}},
}
_IP_KEYS = ("podIP", "clusterIP", "loadBalancerIP", "hostIP", "ip", "podIPs", "hostIPs")
# knownKeyValueStringSliceMapAttributes (admission.go:266-283): the reference asserts each value
# to []string, which a decoded JSON array never is, so the walk stops at once: an empty set
_KV_SLICE_MAP = {
    "authentication": {"v1": {"UserInfo": ["extra"]}},
    "authorization": {"v1": {"SubjectAccessReview": ["extra"]}},
    "certificates": {"v1": {"CertificateSigningRequest": ["extra"]}},
}


class WalkError(Exception):
    pass


def _kv_set(obj: dict):
    if not isinstance(obj, dict):
        raise WalkError("key/value map attribute is not an object")  # a Go type-assertion panic
    out = []
    for kk, vv in obj.items():
        if not isinstance(vv, str):
            break  # reference logs and breaks (admission.go:235-239)
        out.append(Record({"key": kk, "value": vv}))
    return CSet(out)


def walk_object(depth: int, group: str, version: str, kind: str, key: str, obj):
    """admission.go:184-369"""
    if depth == 0:
        raise WalkError("max depth reached")
    if obj is None:
        return None
    names = _KV_STRING_MAP.get(group, {}).get(version, {}).get(kind)
    if names and key in names:
        return _kv_set(obj)
    names = _KV_SLICE_MAP.get(group, {}).get(version, {}).get(kind)
    if names and key in names:
        if not isinstance(obj, dict):
            raise WalkError("key/value slice map attribute is not an object")
        return CSet([])
    if isinstance(obj, dict) and key in ("labels", "annotations"):
        return _kv_set(obj)
    if isinstance(obj, dict):
        rec = {}
        for kk, vv in obj.items():
            v = walk_object(depth - 1, group, version, kind, kk, vv)
            if v is None:
                continue
            rec[kk] = v
        if not rec:
            return None
        return Record(rec)
    if isinstance(obj, list):
        items = [walk_object(depth - 1, group, version, kind, key, x) for x in obj]
        if any(x is None for x in items):
            # the reference builds cedar.NewSet over a nil Value here; reported as an error
            raise WalkError("unsupported nil value in a list")
        return CSet(items)
    if isinstance(obj, bool):
        return obj
    if isinstance(obj, str):
        if key in _IP_KEYS:
            try:
                return IPAddr(ipaddress.ip_interface(obj))
            except ValueError:
                return obj
        return obj
    if isinstance(obj, int):
        return Long(obj)
    raise WalkError(f"unsupported type {type(obj).__name__}")


def unstructured_to_record(obj: dict, group: str, version: str, kind: str) -> Record:
    """admission.go:160-182"""
    attrs = {}
    for k, v in obj.items():
        if v is None:
            continue
        val = walk_object(32, group, version, kind, k, v)
        if val is None:
            continue
        attrs[k] = val
    return Record(attrs)


def admission_action_entities() -> List[Entity]:
    """admission.go:40-53 (note: IDs are the whole quoted string — reference quirk)."""
    all_uid = EntityUID(ADMISSION_ACTION_TYPE, f'{ADMISSION_ACTION_TYPE}::"all"')
    out = [Entity(all_uid, Record(), ())]
    for aid in ADMISSION_ACTION_IDS:
        out.append(Entity(EntityUID(ADMISSION_ACTION_TYPE, aid), Record(), (all_uid,)))
    return out


@dataclass
class AdmissionRequest:
    uid: str
    operation: str  # CREATE UPDATE DELETE CONNECT
    user: UserInfo
    group: str
    version: str
    resource: str
    kind: str
    namespace: str = ""
    name: str = ""
    subresource: str = ""
    object: Optional[dict] = None
    old_object: Optional[dict] = None
    kind_version: Optional[str] = None  # req.Kind.Version when it differs from req.Resource.Version


def _admission_path(req: AdmissionRequest) -> str:
    a = Attributes(namespace=req.namespace, api_group=req.group, api_version=req.version, resource=req.resource,
                   subresource=req.subresource, name=req.name)
    return resource_request_to_path(a)


def _admission_resource_entity(req: AdmissionRequest, raw: Optional[dict]) -> Entity:
    if raw is None:
        raise WalkError("unstructured data is nil")
    if not isinstance(raw, dict) or not isinstance(raw.get("kind"), str) or not raw.get("kind"):
        raise WalkError("Object 'Kind' is missing")  # unstructured decoding requires kind
    group = req.group or "core"
    kver = req.kind_version if req.kind_version is not None else req.version
    attrs = unstructured_to_record(raw, group, kver, req.kind)
    return Entity(EntityUID(f"{group}::{kver}::{req.kind}", _admission_path(req)), attrs, ())


def admission_request_from_review(review: dict) -> AdmissionRequest:
    """An AdmissionReview ({"request": {...}}) as controller-runtime's admission.Request."""
    q = review.get("request", review)
    u = q.get("userInfo") or {}
    extra = {k: [x for x in v if isinstance(x, str)] for k, v in (u.get("extra") or {}).items()}
    return AdmissionRequest(
        uid=q.get("uid", ""), operation=q.get("operation", ""),
        user=UserInfo(u.get("username", ""), u.get("uid", ""), [g for g in u.get("groups") or [] if isinstance(g, str)],
                      extra),
        group=(q.get("resource") or {}).get("group", ""), version=(q.get("resource") or {}).get("version", ""),
        resource=(q.get("resource") or {}).get("resource", ""), kind=(q.get("kind") or {}).get("kind", ""),
        namespace=q.get("namespace", ""), name=q.get("name", ""), subresource=q.get("subResource", ""),
        object=q.get("object"), old_object=q.get("oldObject"),
        kind_version=(q.get("kind") or {}).get("version", ""))


def admission_to_cedar(req: AdmissionRequest) -> Tuple[EntityMap, Request]:
    """handler.go:82-153 (entity + request construction)."""
    user = UserInfo(req.user.name, req.user.uid or req.user.name, req.user.groups, req.user.extra)  # user.go:19-25
    puid, em = user_to_cedar_entity(user)
    em = dict(em)
    if req.operation == "DELETE":
        res = _admission_resource_entity(req, req.old_object)
    else:
        res = _admission_resource_entity(req, req.object)
    old = None
    if req.old_object is not None and req.operation != "DELETE":
        old = _admission_resource_entity(req, req.old_object)
        old = Entity(EntityUID(old.uid.type, req.uid), old.attrs, ())
        m = dict(res.attrs.m)
        m["oldObject"] = old.uid
        res = Entity(res.uid, Record(m), ())
        em[old.uid] = old
    em[res.uid] = res
    op = {"CONNECT": "connect", "CREATE": "create", "UPDATE": "update", "DELETE": "delete"}[req.operation]
    action = EntityUID(ADMISSION_ACTION_TYPE, op)
    for e in admission_action_entities():
        em[e.uid] = e
    ctx = {}
    if old is not None:
        ctx["oldObject"] = old.attrs
    return em, Request(puid, action, res.uid, Record(ctx))


ALLOW_ALL_ADMISSION_POLICY = (
    'permit (principal, action in [k8s::admission::Action::"create", k8s::admission::Action::"update", '
    'k8s::admission::Action::"delete", k8s::admission::Action::"connect"], resource);')


def allow_all_admission_store() -> PolicySet:
    """admit_all_policy.go:10-19 + main.go:111-116 (policy ID `allow-all-admission`)."""
    ps = PolicySet()
    p = parse_policies(ALLOW_ALL_ADMISSION_POLICY, "")[0]
    # NewPolicyFromAST carries a zero Position
    p.offset, p.line, p.col = 0, 0, 0
    ps.add("allow-all-admission", p)
    return ps


def admission_handle(tiers: List[PolicySet], req: AdmissionRequest, stores_ready: bool = True) -> Tuple[bool, str]:
    """handler.go:43-80 — returns (allowed, message). `tiers` must already include the trailing
    allow-all store (main.go:111-116)."""
    if req.namespace in ("kube-system", "cedar-k8s-authz-system"):
        return True, ""
    if not stores_ready:
        return True, ""
    em, creq = admission_to_cedar(req)
    ok, diag, _ = tiered_is_authorized(tiers, em, creq)
    if not ok:
        return False, diag.reasons_json() if diag.reasons else ""
    return True, ""
