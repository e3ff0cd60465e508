"""Generates tests/golden/reference_vectors.json and tests/golden/reference_corpus.json.

reference_vectors.json is a hand transcription (as data) of the reference's own pinned test vectors:
  * TestAuthorize            internal/server/authorizer/authorizer_test.go:462-920 (13 cases)
  * TestTieredIsAuthorized   internal/server/store/store_test.go:21-188 (3 cases)
  * TestRecordToCedarResource internal/server/authorizer/authorizer_test.go:31-460 (6 cases)
  * TestResourceRequestToPath internal/server/entities/authorization_test.go:10-57 (3 cases)
  * TestUnstructuredToEntity internal/server/entities/admission_test.go:15-90 (1 case)
reference_corpus.json bundles the reference's Cedar policy texts used as parser/compiler fixtures:
  * the 13 converter golden files internal/convert/testdata/*.cedar
  * every Policy `spec.content` in demo/authorization-policy.yaml and demo/admission-policy.yaml
The corpus step reads /root/reference and is run only in the build container; the GPU box uses the
committed JSON. Run: python tests/golden/make_reference_fixtures.py
"""
import glob
import json
import os

import yaml

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"

U_DEFAULT = {"name": "test-user", "uid": "1234567890", "groups": ["test-group"], "extra": {"attr1": ["value1"]}}

# ---------------------------------------------------------------- TestAuthorize (authorizer_test.go:462-920)
AUTH_CASES = [
    ("Allow", '''
permit (
	principal,
	action in [k8s::Action::"get", k8s::Action::"list", k8s::Action::"watch"],
	resource is k8s::Resource
) when {
	principal.name == "test-user" &&
	resource.resource == "pods"
};''', dict(user=U_DEFAULT, verb="get", namespace="default", api_version="v1", resource="pods", name="test-pod",
            resource_request=True), True, 1,
     '{"reasons":[{"policy":"policy0","position":{"filename":"Allow","offset":1,"line":2,"column":1}}]}'),
    ("Allow Impersonate UID", '''
permit (
	principal,
	action == k8s::Action::"impersonate",
	resource == k8s::PrincipalUID::"1234"
) when {
	principal.name == "test-user"
};''', dict(user=U_DEFAULT, verb="impersonate", resource="uids", name="1234", resource_request=True), True, 1,
     '{"reasons":[{"policy":"policy0","position":{"filename":"Allow Impersonate UID","offset":1,"line":2,"column":1}}]}'),
    ("Allow Impersonate serviceaccount", '''
permit (
	principal,
	action == k8s::Action::"impersonate",
	resource is k8s::ServiceAccount
) when {
	principal.name == "test-user" &&
	resource.name == "default" &&
	resource.namespace == "kube-system"
};''', dict(user=U_DEFAULT, verb="impersonate", namespace="kube-system", resource="serviceaccounts", name="default",
            resource_request=True), True, 1,
     '{"reasons":[{"policy":"policy0","position":{"filename":"Allow Impersonate serviceaccount","offset":1,"line":2,"column":1}}]}'),
    ("Allow Impersonate serviceaccount id", '''
permit (
	principal,
	action == k8s::Action::"impersonate",
	resource == k8s::ServiceAccount::"system:serviceaccount:kube-system:default"
) when {
	principal.name == "test-user"
};''', dict(user=U_DEFAULT, verb="impersonate", namespace="kube-system", resource="serviceaccounts", name="default",
            resource_request=True), True, 1,
     '{"reasons":[{"policy":"policy0","position":{"filename":"Allow Impersonate serviceaccount id","offset":1,"line":2,"column":1}}]}'),
    ("Allow Impersonate node", '''
permit (
	principal,
	action == k8s::Action::"impersonate",
	resource is k8s::Node
) when {
	principal.name == "test-user" &&
	resource.name == "ip-10-24-34-0.us-west-2.compute.internal"
};''', dict(user=U_DEFAULT, verb="impersonate", resource="users",
            name="system:node:ip-10-24-34-0.us-west-2.compute.internal", resource_request=True), True, 1,
     '{"reasons":[{"policy":"policy0","position":{"filename":"Allow Impersonate node","offset":1,"line":2,"column":1}}]}'),
    ("Allow Impersonate user", '''
permit (
	principal,
	action == k8s::Action::"impersonate",
	resource is k8s::User
) when {
	principal.name == "test-user" &&
	resource.name == "test-impersonated"
};''', dict(user=U_DEFAULT, verb="impersonate", resource="users", name="test-impersonated", resource_request=True),
     True, 1,
     '{"reasons":[{"policy":"policy0","position":{"filename":"Allow Impersonate user","offset":1,"line":2,"column":1}}]}'),
    ("Allow Impersonate group", '''
permit (
	principal,
	action == k8s::Action::"impersonate",
	resource is k8s::Group
) when {
	principal.name == "test-user" &&
	resource.name == "test-impersonated-group"
};''', dict(user=U_DEFAULT, verb="impersonate", resource="groups", name="test-impersonated-group",
            resource_request=True), True, 1,
     '{"reasons":[{"policy":"policy0","position":{"filename":"Allow Impersonate group","offset":1,"line":2,"column":1}}]}'),
    ("Allow Impersonate extra", '''
permit (
	principal is k8s::User,
	action == k8s::Action::"impersonate",
	resource is k8s::Extra
) when {
	principal.name == "test-user" &&
	resource.key == "test-key" &&
	resource has value &&
	resource.value == "test-value"
};''', dict(user=U_DEFAULT, verb="impersonate", resource="userextras", subresource="test-key", name="test-value",
            resource_request=True), True, 1,
     '{"reasons":[{"policy":"policy0","position":{"filename":"Allow Impersonate extra","offset":1,"line":2,"column":1}}]}'),
    ("Explicit Deny", '''
forbid (
	principal,
	action in [k8s::Action::"get", k8s::Action::"list", k8s::Action::"watch"],
	resource is k8s::Resource
) when {
	principal.name == "test-user" &&
	resource.resource == "pods"
};''', dict(user=U_DEFAULT, verb="get", namespace="default", api_version="v1", resource="pods", name="test-pod",
            resource_request=True), True, 0,
     '{"reasons":[{"policy":"policy0","position":{"filename":"Explicit Deny","offset":1,"line":2,"column":1}}]}'),
    ("No Opinion", '''
forbid (
	principal,
	action in [k8s::Action::"get", k8s::Action::"list", k8s::Action::"watch"],
	resource is k8s::Resource
) when {
	principal.name == "test-user" &&
	resource.resource == "nodes"
};''', dict(user=U_DEFAULT, verb="get", namespace="default", api_version="v1", resource="pods", name="test-pod",
            resource_request=True), True, 2, ""),
    ("system identity: No Opinion", '''
forbid (
	principal,
	action in [k8s::Action::"get", k8s::Action::"list", k8s::Action::"watch"],
	resource is k8s::Resource
) when {
	principal.name == "test-user" &&
	resource.resource == "nodes"
};''', dict(user={"name": "system:kube-apiserver", "uid": "1234567890", "groups": ["system:masters"], "extra": {}},
            verb="get", namespace="default", api_version="v1", resource="pods", name="test-pod",
            resource_request=True), True, 2, ""),
    ("store incomplete: No Opinion", '''
forbid (
	principal,
	action in [k8s::Action::"get", k8s::Action::"list", k8s::Action::"watch"],
	resource is k8s::Resource
) when {
	principal.name == "test-user" &&
	resource.resource == "nodes"
};''', dict(user={"name": "test-user", "uid": "1234567890", "groups": ["test-group"], "extra": {}},
            verb="get", namespace="default", api_version="v1", resource="pods", name="test-pod",
            resource_request=True), False, 2, ""),
    ("allow self", '''
forbid (
	principal,
	action in [k8s::Action::"get", k8s::Action::"list", k8s::Action::"watch"],
	resource is k8s::Resource
) when {
	principal.name == "test-user" &&
	resource.resource == "nodes"
};''', dict(user={"name": "system:authorizer:cedar-authorizer", "uid": "1234567890", "groups": [], "extra": {}},
            verb="list", api_group="cedar.k8s.aws", api_version="v1", resource="policies", resource_request=True),
     True, 1, "cedar authorizer is always allowed to access policies"),
]

# ---------------------------------------------------------------- TestTieredIsAuthorized (store_test.go:21-188)
TIER_ENTITIES = [
    {"uid": {"type": "k8s::User", "id": "alice"}, "attrs": {"name": "alice"},
     "parents": [{"type": "k8s::Group", "id": "admin"}]},
    {"uid": {"type": "k8s::Group", "id": "admin"}, "attrs": {"name": "admin"}, "parents": []},
    {"uid": {"type": "k8s::Resource", "id": "/api/v1/namespaces/default/configmaps/cm1"},
     "attrs": {"name": "cm1", "namespace": "default", "apiGroup": "", "resource": "configmaps"}, "parents": []},
]
TIER_REQ = {"principal": {"type": "k8s::User", "id": "alice"}, "action": {"type": "k8s::Action", "id": "get"},
            "resource": {"type": "k8s::Resource", "id": "/api/v1/namespaces/default/configmaps/cm1"}, "context": {}}
TIER_REASON0 = {"reasons": [{"policy": "policy0", "position": {"filename": "in-memory-test-store.cedar", "offset": 0,
                                                                "line": 1, "column": 1}}]}
TIER_CASES = [
    ("tiered policies allow over deny",
     ['permit(principal in k8s::Group::"admin", action, resource);',
      'forbid(principal in k8s::Group::"admin", action, resource);'], True, TIER_REASON0),
    ("tiered default deny",
     ['forbid(principal, action == k8s::Action::"list", resource);',
      'forbid(principal in k8s::Group::"read-only", action, resource);'], False, {}),
    ("tiered default allow",
     ['forbid(principal, action == k8s::Action::"list", resource);',
      'forbid(principal in k8s::Group::"read-only", action, resource);',
      'permit(principal, action, resource);'], True, TIER_REASON0),
]

# ---------------------------------------------------------------- TestRecordToCedarResource (authorizer_test.go:31-460)
def _user_ent(ptype, extra_attrs=None, groups=("test-group",)):
    attrs = {"name": "test-user", "extra": [{"key": "attr1", "values": ["value1"]}]}
    if extra_attrs:
        attrs.update(extra_attrs)
    return {"uid": {"type": ptype, "id": "1234567890"}, "attrs": attrs,
            "parents": [{"type": "k8s::Group", "id": g} for g in groups]}


def _group_ent(g):
    return {"uid": {"type": "k8s::Group", "id": g}, "attrs": {"name": g}, "parents": []}


def _res(t, i, attrs):
    return {"uid": {"type": t, "id": i}, "attrs": attrs, "parents": []}


def _req(ptype, verb, rtype, rid):
    return {"principal": {"type": ptype, "id": "1234567890"}, "action": {"type": "k8s::Action", "id": verb},
            "resource": {"type": rtype, "id": rid}, "context": {}}


RECORD_CASES = [
    ("Resource with namespace",
     dict(user=U_DEFAULT, verb="get", namespace="default", api_version="v1", resource="pods", name="test-pod",
          resource_request=True),
     [_user_ent("k8s::User"), _group_ent("test-group"),
      _res("k8s::Resource", "/api/v1/namespaces/default/pods/test-pod",
           {"apiGroup": "", "namespace": "default", "resource": "pods", "name": "test-pod"})],
     _req("k8s::User", "get", "k8s::Resource", "/api/v1/namespaces/default/pods/test-pod")),
    ("k8s::Resource",
     dict(user=U_DEFAULT, verb="list", api_version="v1", resource="pods", resource_request=True),
     [_user_ent("k8s::User"), _group_ent("test-group"),
      _res("k8s::Resource", "/api/v1/pods", {"apiGroup": "", "resource": "pods"})],
     _req("k8s::User", "list", "k8s::Resource", "/api/v1/pods")),
    ("NonResourceURL",
     dict(user=U_DEFAULT, verb="get", resource_request=False, path="/metrics"),
     [_user_ent("k8s::User"), _group_ent("test-group"),
      _res("k8s::NonResourceURL", "/metrics", {"path": "/metrics"})],
     _req("k8s::User", "get", "k8s::NonResourceURL", "/metrics")),
    ("apigroup subresource",
     dict(user=U_DEFAULT, verb="patch", namespace="default", api_group="apps", api_version="v1",
          resource="deployments", subresource="scale", name="nginx", resource_request=True),
     [_user_ent("k8s::User"), _group_ent("test-group"),
      _res("k8s::Resource", "/apis/apps/v1/namespaces/default/deployments/nginx/scale",
           {"apiGroup": "apps", "namespace": "default", "resource": "deployments", "name": "nginx",
            "subresource": "scale"})],
     _req("k8s::User", "patch", "k8s::Resource", "/apis/apps/v1/namespaces/default/deployments/nginx/scale")),
    ("ServiceAccount principal",
     dict(user={"name": "system:serviceaccount:foo:bar", "uid": "1234567890",
                "groups": ["system:serviceaccounts", "system:serviceaccounts:default", "system:authenticated"],
                "extra": {"attr1": ["value1"]}},
          verb="get", namespace="default", api_version="v1", resource="pods", name="test-pod", resource_request=True),
     [{"uid": {"type": "k8s::ServiceAccount", "id": "1234567890"},
       "attrs": {"name": "bar", "namespace": "foo", "extra": [{"key": "attr1", "values": ["value1"]}]},
       "parents": [{"type": "k8s::Group", "id": g} for g in
                   ("system:serviceaccounts", "system:serviceaccounts:default", "system:authenticated")]},
      _group_ent("system:serviceaccounts"), _group_ent("system:serviceaccounts:default"),
      _group_ent("system:authenticated"),
      _res("k8s::Resource", "/api/v1/namespaces/default/pods/test-pod",
           {"apiGroup": "", "namespace": "default", "resource": "pods", "name": "test-pod"})],
     _req("k8s::ServiceAccount", "get", "k8s::Resource", "/api/v1/namespaces/default/pods/test-pod")),
    ("labelSelector & fieldSelector",
     dict(user=U_DEFAULT, verb="list", namespace="default", api_version="v1", resource="pods", resource_request=True,
          label_selector=[{"key": "owner", "operator": "=", "values": ["test-user"]}],
          field_selector=[{"field": ".spec.nodeName", "operator": "=", "value": "test-node"}]),
     [_user_ent("k8s::User"), _group_ent("test-group"),
      _res("k8s::Resource", "/api/v1/namespaces/default/pods",
           {"apiGroup": "", "namespace": "default", "resource": "pods",
            "labelSelector": [{"key": "owner", "operator": "=", "values": ["test-user"]}],
            "fieldSelector": [{"field": ".spec.nodeName", "operator": "=", "value": "test-node"}]})],
     _req("k8s::User", "list", "k8s::Resource", "/api/v1/namespaces/default/pods")),
]

# ---------------------------------------------------------------- TestResourceRequestToPath (authorization_test.go:10-57)
PATH_CASES = [
    (dict(api_version="v1", resource="pods"), "/api/v1/pods"),
    (dict(api_group="apps", api_version="v1", namespace="kube-system", resource="deployments", name="coredns"),
     "/apis/apps/v1/namespaces/kube-system/deployments/coredns"),
    (dict(api_version="v1", namespace="default", resource="pods", name="mypod", subresource="logs"),
     "/api/v1/namespaces/default/pods/mypod/logs"),
]

# ---------------------------------------------------------------- TestUnstructuredToEntity (admission_test.go:15-90)
# The unstructured form of the typed Pod (runtime.DefaultUnstructuredConverter drops zero values,
# keeps creationTimestamp: null and the empty resources/status maps).
POD_UNSTRUCTURED = {
    "apiVersion": "v1", "kind": "Pod",
    "metadata": {"name": "test-pod", "namespace": "default", "creationTimestamp": None},
    "spec": {"containers": [{"name": "test-container", "image": "test-image", "resources": {}}],
             "nodeName": "test-node", "hostNetwork": True, "shareProcessNamespace": False},
    "status": {"phase": "Running", "podIP": "10.10.1.4"},
}
POD_EXPECTED = {
    "apiVersion": "v1", "kind": "Pod",
    "metadata": {"name": "test-pod", "namespace": "default"},
    "spec": {"containers": [{"name": "test-container", "image": "test-image"}], "nodeName": "test-node",
             "hostNetwork": True, "shareProcessNamespace": False},
    "status": {"phase": "Running", "podIP": {"__extn": {"fn": "ip", "arg": "10.10.1.4/32"}}},
}


def vectors():
    return {
        "authorize": [dict(name=n, policy=p, attributes=a, store_complete=c, want_decision=d, want_reason=r)
                      for (n, p, a, c, d, r) in AUTH_CASES],
        "tiers": {"entities": TIER_ENTITIES, "request": TIER_REQ,
                  "cases": [dict(name=n, stores=s, want=w, want_diag=dg) for (n, s, w, dg) in TIER_CASES]},
        "record_to_cedar": [dict(name=n, attributes=a, want_entities=e, want_request=r)
                            for (n, a, e, r) in RECORD_CASES],
        "paths": [dict(attributes=a, want=w) for (a, w) in PATH_CASES],
        "unstructured": [dict(name="valid pod", group="core", version="v1", kind="Pod", input=POD_UNSTRUCTURED,
                              want=POD_EXPECTED)],
    }


def corpus():
    out = {"converter": {}, "demo": {}}
    for f in sorted(glob.glob(os.path.join(REF, "internal/convert/testdata/*.cedar"))):
        out["converter"][os.path.basename(f)] = open(f).read()
    for f in ("demo/authorization-policy.yaml", "demo/admission-policy.yaml"):
        for doc in yaml.safe_load_all(open(os.path.join(REF, f))):
            if doc and doc.get("kind") == "Policy":
                out["demo"][f"{os.path.basename(f)}:{doc['metadata']['name']}"] = doc["spec"]["content"]
    return out


if __name__ == "__main__":
    with open(os.path.join(HERE, "reference_vectors.json"), "w") as fh:
        json.dump(vectors(), fh, indent=1, sort_keys=True)
    if os.path.isdir(REF):
        with open(os.path.join(HERE, "reference_corpus.json"), "w") as fh:
            json.dump(corpus(), fh, indent=1, sort_keys=True)
    print("ok")
