"""Seeded synthetic workloads for the benchmark configs (SURVEY §8d / BASELINE.json configs).

  C1  demo/authorization-policy.yaml policies x synthetic SubjectAccessReviews
  C2  RBAC-converted policies (shaped exactly like internal/convert/converter.go:31-165 output)
  C3  ABAC policies over k8s::Group membership (namespace / resource / apiGroup / name / labelSelector)
  C4  admission policies over ConfigMap / Secret objects (like, label sets, has)

SubjectAccessReviews follow the SURVEY §8(d) mix: Zipf users (85% User, 12% ServiceAccount,
3% Node; no `system:` bypass identities), 1+Binomial(7, 0.35) groups, K8s verb mix, ~80 resources,
200 namespaces, names 60%, subresources 10%, non-resource URLs 5%, impersonation 1%,
label selectors 3%. Everything is driven by numpy PCG64 with fixed seeds.
"""
from __future__ import annotations

import json
from typing import Dict, List, Optional, Tuple

import numpy as np

VERBS = ["get", "list", "watch", "create", "update", "patch", "delete", "deletecollection", "use", "bind", "escalate",
         "approve", "sign", "attest", "put", "post", "head", "options"]
_VERB_P = np.array([35, 20, 15, 7, 6, 6, 6, 1, 0.5, 0.5, 0.5, 0.5, 0.5, 0.5, 0.25, 0.25, 0.25, 0.25])
_VERB_P = _VERB_P / _VERB_P.sum()

BUILTIN = [("", "v1", r) for r in ("pods", "services", "configmaps", "secrets", "nodes", "namespaces", "endpoints",
                                   "events", "persistentvolumeclaims", "persistentvolumes", "serviceaccounts",
                                   "replicationcontrollers", "limitranges", "resourcequotas", "podtemplates",
                                   "componentstatuses", "bindings")]
BUILTIN += [("apps", "v1", r) for r in ("deployments", "replicasets", "statefulsets", "daemonsets", "controllerrevisions")]
BUILTIN += [("batch", "v1", r) for r in ("jobs", "cronjobs")]
BUILTIN += [("rbac.authorization.k8s.io", "v1", r) for r in ("roles", "rolebindings", "clusterroles", "clusterrolebindings")]
BUILTIN += [("networking.k8s.io", "v1", r) for r in ("ingresses", "networkpolicies", "ingressclasses")]
BUILTIN += [("policy", "v1", r) for r in ("poddisruptionbudgets",)]
BUILTIN += [("storage.k8s.io", "v1", r) for r in ("storageclasses", "volumeattachments", "csidrivers", "csinodes")]
BUILTIN += [("autoscaling", "v2", r) for r in ("horizontalpodautoscalers",)]
BUILTIN += [("coordination.k8s.io", "v1", r) for r in ("leases",)]
BUILTIN += [("discovery.k8s.io", "v1", r) for r in ("endpointslices",)]
BUILTIN += [("certificates.k8s.io", "v1", r) for r in ("certificatesigningrequests",)]
BUILTIN += [("admissionregistration.k8s.io", "v1", r) for r in ("mutatingwebhookconfigurations",
                                                               "validatingwebhookconfigurations")]
BUILTIN += [("apiextensions.k8s.io", "v1", r) for r in ("customresourcedefinitions",)]
BUILTIN += [("scheduling.k8s.io", "v1", r) for r in ("priorityclasses",)]
BUILTIN += [("node.k8s.io", "v1", r) for r in ("runtimeclasses",)]
BUILTIN += [("cedar.k8s.aws", "v1alpha1", "policies")]
CRDS = [(f"example{i % 5}.acme.io", "v1", f"widgets{i}") for i in range(20)]
RESOURCES = BUILTIN + CRDS
SUBRESOURCES = ["status", "scale", "log", "exec", "portforward", "proxy", "token", "eviction"]
NONRES_PATHS = ["/healthz", "/livez", "/readyz", "/version", "/version/", "/metrics", "/openapi/v2", "/openapi/v3",
                "/openapi/v3/apis/apps/v1", "/healthz/ping", "/readyz/etcd", "/api", "/apis", "/logs/kube-apiserver.log"]


def _zipf_idx(rng, n: int, size: int, s: float = 1.1) -> np.ndarray:
    ranks = np.arange(1, n + 1, dtype=np.float64)
    p = ranks ** (-s)
    p /= p.sum()
    return rng.choice(n, size=size, p=p)


class Population:
    """Users, service accounts, nodes and their group memberships; with `dag_depth`, a static
    k8s::Group hierarchy of at most that many levels (C3).

    The hierarchy ranks groups by popularity (group-00000 is the most used, in memberships and in
    policies) and puts the popular ones near the roots: level L holds ~8 * 1.8^L groups. A group at
    level L > 0 has one parent on level L - 1 and, one time in four, a second one on level L - 1 or
    L - 2, so a group's transitive ancestors number up to ~2L. The reference's SAR entities give
    groups no parents (internal/server/entities/user.go:40-54): the hierarchy reaches evaluation as
    the image's static entities (`static_entities()`, cg_compiler_set_entities)."""

    def __init__(self, seed: int = 7, n_users: int = 50_000, n_groups: int = 5_000, n_namespaces: int = 200,
                 dag_depth: int = 0):
        rng = np.random.Generator(np.random.PCG64(seed))
        self.n_users = n_users
        self.groups = [f"group-{i:05d}" for i in range(n_groups)]
        self.namespaces = [f"ns-{i:03d}" for i in range(n_namespaces)]
        kind = rng.choice(3, size=n_users, p=[0.85, 0.12, 0.03])
        self.names = []
        for i in range(n_users):
            if kind[i] == 0:
                self.names.append(f"user-{i:05d}")
            elif kind[i] == 1:
                self.names.append(f"system:serviceaccount:{self.namespaces[i % n_namespaces]}:sa-{i:05d}")
            else:
                self.names.append(f"system:node:node-{i:05d}")
        ng = 1 + rng.binomial(7, 0.35, size=n_users)
        gidx = _zipf_idx(rng, n_groups, int(ng.sum()), s=0.9)
        self.user_groups: List[List[str]] = []
        o = 0
        for i in range(n_users):
            gs = [self.groups[g] for g in gidx[o:o + ng[i]]]
            o += ng[i]
            gs.append("system:authenticated")
            if kind[i] == 1:
                gs += ["system:serviceaccounts", f"system:serviceaccounts:{self.names[i].split(':')[2]}"]
            self.user_groups.append(list(dict.fromkeys(gs)))
        self.group_parents: Dict[str, List[str]] = {}
        if dag_depth > 0:
            drng = np.random.Generator(np.random.PCG64(seed + 0x5A6))  # memberships above are unchanged
            level = [min(dag_depth - 1, int(np.log1p(i / 8.0) / np.log(1.8))) for i in range(n_groups)]
            by_level: Dict[int, List[int]] = {}
            for i, lv in enumerate(level):
                by_level.setdefault(lv, []).append(i)
            for i, lv in enumerate(level):
                if lv == 0:
                    continue
                up = by_level[lv - 1]
                par = [up[int(drng.integers(len(up)))]]
                if drng.random() < 0.25:
                    alt = by_level[max(0, lv - 2)] if drng.random() < 0.5 else up
                    par.append(alt[int(drng.integers(len(alt)))])
                self.group_parents[self.groups[i]] = [self.groups[p] for p in dict.fromkeys(par)]

    def static_entities(self) -> List[dict]:
        """The group hierarchy as Cedar JSON entities, shaped like UserToCedarEntity's group
        entities (entities/user.go:40-54: attrs {name}) plus their parents."""
        if not self.group_parents:
            return []
        return [{"uid": {"type": "k8s::Group", "id": g}, "attrs": {"name": g},
                 "parents": [{"type": "k8s::Group", "id": p} for p in self.group_parents.get(g, [])]}
                for g in self.groups]


def make_sar(user: str, uid: str, groups: List[str], verb: str, ns: str = "", group: str = "", version: str = "v1",
             resource: str = "", subresource: str = "", name: str = "", path: Optional[str] = None,
             extra: Optional[Dict[str, List[str]]] = None, label_selector: Optional[List[dict]] = None) -> dict:
    spec = {"user": user, "uid": uid, "groups": groups}
    if extra:
        spec["extra"] = extra
    if path is not None:
        spec["nonResourceAttributes"] = {"path": path, "verb": verb}
    else:
        ra = {"verb": verb, "namespace": ns, "group": group, "version": version, "resource": resource,
              "subresource": subresource, "name": name}
        if label_selector:
            ra["labelSelector"] = {"requirements": label_selector}
        spec["resourceAttributes"] = ra
    return {"apiVersion": "authorization.k8s.io/v1", "kind": "SubjectAccessReview", "spec": spec}


def random_sars(n: int, seed: int = 11, pop: Optional[Population] = None) -> List[dict]:
    pop = pop or Population()
    rng = np.random.Generator(np.random.PCG64(seed))
    users = _zipf_idx(rng, pop.n_users, n)
    verbs = rng.choice(len(VERBS), size=n, p=_VERB_P)
    res = rng.integers(0, len(RESOURCES), size=n)
    nss = rng.integers(0, len(pop.namespaces), size=n)
    u = rng.random((n, 6))
    out = []
    for i in range(n):
        ui = int(users[i])
        user, groups = pop.names[ui], pop.user_groups[ui]
        uid = f"uid-{ui:05d}"
        verb = VERBS[verbs[i]]
        if u[i, 0] < 0.05:
            out.append(make_sar(user, uid, groups, verb if verb in ("get", "post", "put", "head", "options") else "get",
                                path=NONRES_PATHS[int(u[i, 1] * len(NONRES_PATHS))]))
            continue
        if u[i, 0] < 0.06:
            kind = ["users", "groups", "serviceaccounts", "uids", "userextras"][int(u[i, 1] * 5)]
            tgt = pop.names[int(u[i, 2] * pop.n_users)]
            if kind == "groups":
                tgt = pop.groups[int(u[i, 2] * len(pop.groups))]
            sub = "scopes" if kind == "userextras" else ""
            ns = pop.namespaces[nss[i]] if kind == "serviceaccounts" else ""
            out.append(make_sar(user, uid, groups, "impersonate", ns=ns, group="", version="v1", resource=kind,
                                subresource=sub, name=tgt.split(":")[-1] if kind == "serviceaccounts" else tgt))
            continue
        g, v, r = RESOURCES[int(res[i])]
        cluster = r in ("nodes", "namespaces", "persistentvolumes", "clusterroles", "clusterrolebindings",
                        "storageclasses", "customresourcedefinitions", "priorityclasses")
        ns = "" if cluster else pop.namespaces[nss[i]]
        name = f"{r[:-1]}-{int(u[i, 2] * 1000)}" if (u[i, 3] < 0.6 and verb not in ("list", "watch", "create")) else ""
        if name and u[i, 4] < 0.15:
            name = "prod-" + name
        sub = SUBRESOURCES[int(u[i, 5] * len(SUBRESOURCES))] if (name and u[i, 5] < 0.1) else ""
        ls = None
        if verb in ("list", "watch") and u[i, 4] < 0.15:
            ls = [{"key": "owner", "operator": "In", "values": [user.split(":")[-1]]}]
        out.append(make_sar(user, uid, groups, verb, ns=ns, group=g, version=v, resource=r, subresource=sub, name=name,
                            label_selector=ls))
    return out


# -------------------------------------------------------------------------------------------------
# Policy generators
# -------------------------------------------------------------------------------------------------

def _set(xs):
    return "[" + ", ".join(json.dumps(x) for x in xs) + "]"


def _actions(vs):
    if len(vs) == 1:
        return f'action == k8s::Action::{json.dumps(vs[0])}'
    return "action in [" + ", ".join(f"k8s::Action::{json.dumps(v)}" for v in vs) + "]"


def rbac_policies(n: int, seed: int = 21, pop: Optional[Population] = None) -> str:
    """C2: policies shaped like the RBAC converter's output (converter.go:31-165)."""
    pop = pop or Population()
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    read = ["get", "list", "watch"]
    write = ["create", "update", "patch", "delete"]
    for i in range(n):
        kind = rng.choice(3, p=[0.45, 0.35, 0.20])
        ann = f'@clusterRoleBinding("binding-{i // 4}")\n@clusterRole("role-{i // 4}")\n@policyRule("{i % 4:02d}")\n'
        when = []
        if kind == 0:
            principal = f'principal in k8s::Group::{json.dumps(pop.groups[int(rng.integers(len(pop.groups)))])}'
        elif kind == 1:
            principal = "principal is k8s::User"
            when.append(f'principal.name == {json.dumps(pop.names[int(rng.integers(pop.n_users))].split(":")[-1])}')
        else:
            principal = "principal is k8s::ServiceAccount"
            ns = pop.namespaces[int(rng.integers(len(pop.namespaces)))]
            when.append(f'principal.namespace == {json.dumps(ns)} && principal.name == "sa-{int(rng.integers(50000)):05d}"')
        verbs = read if rng.random() < 0.6 else (read + write if rng.random() < 0.5 else write)
        if rng.random() < 0.15:
            verbs = [VERBS[int(rng.integers(0, 7))]]
        nres = 1 + int(rng.integers(0, 3))
        picks = [RESOURCES[int(x)] for x in rng.integers(0, len(RESOURCES), size=nres)]
        groups = sorted({p[0] for p in picks})
        ress = sorted({p[2] for p in picks})
        when.append(f'resource.apiGroup == {json.dumps(groups[0])}' if len(groups) == 1
                    else f'{_set(groups)}.contains(resource.apiGroup)')
        when.append(f'resource.resource == {json.dumps(ress[0])}' if len(ress) == 1
                    else f'{_set(ress)}.contains(resource.resource)')
        if rng.random() < 0.2:
            when.append(f'resource has name && resource.name == "{ress[0][:-1]}-{int(rng.integers(1000))}"')
        if rng.random() < 0.5:
            when.append(f'resource has namespace && resource.namespace == {json.dumps(pop.namespaces[int(rng.integers(len(pop.namespaces)))])}')
        pol = (f"{ann}permit (\n  {principal},\n  {_actions(verbs)},\n  resource is k8s::Resource\n)\n"
               f"when {{ {' && '.join(when)} }}\nunless {{ resource has subresource }};\n")
        out.append(pol)
    return "\n".join(out)


def abac_policies(n: int, seed: int = 31, pop: Optional[Population] = None, variant: str = "full") -> str:
    """C3: attribute-based policies keyed on group membership.

    variant (shape studies of the evaluator; `full` is the benchmark workload):
      full        group-scoped policies with when-clauses
      scope-only  the same scopes, conditions dropped
      no-group    the same conditions, principal scope `principal is k8s::User` instead of `in Group`
    """
    text = _abac(n, seed, pop)
    if variant == "scope-only":
        import re
        text = re.sub(r"\)\nwhen \{.*?\};\n", ");\n", text, flags=re.S)
    elif variant == "no-group":
        import re
        text = re.sub(r'principal in k8s::Group::"[^"]*"', "principal is k8s::User", text)
    elif variant == "atomic-only":  # drop the runtime-record (bytecode) template
        text = "\n".join(p for p in text.split("\n\n") if "containsAny" not in p)
    elif variant != "full":
        raise ValueError(variant)
    return text


def _abac(n: int, seed: int, pop: Optional[Population]) -> str:
    pop = pop or Population()
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    for i in range(n):
        g = pop.groups[int(_zipf_idx(rng, len(pop.groups), 1, s=0.9)[0])]
        ns = pop.namespaces[int(rng.integers(len(pop.namespaces)))]
        grp, ver, res = RESOURCES[int(rng.integers(len(RESOURCES)))]
        t = rng.random()
        if t < 0.55:
            verbs = ["get", "list", "watch"] if rng.random() < 0.6 else ["create", "update", "patch", "delete"]
            pol = (f'permit (\n  principal in k8s::Group::{json.dumps(g)},\n  {_actions(verbs)},\n  resource is k8s::Resource\n)\n'
                   f'when {{ resource has namespace && resource.namespace == {json.dumps(ns)} && '
                   f'resource.apiGroup == {json.dumps(grp)} }};\n')
        elif t < 0.75:
            pol = (f'permit (\n  principal in k8s::Group::{json.dumps(g)},\n  action,\n  resource is k8s::Resource\n)\n'
                   f'when {{ resource.resource == {json.dumps(res)} && resource has labelSelector && '
                   f'resource.labelSelector.containsAny([{{"key": "owner", "operator": "in", "values": [principal.name]}}]) }};\n')
        elif t < 0.9:
            pol = (f'forbid (\n  principal in k8s::Group::{json.dumps(g)},\n  action in [k8s::Action::"delete", k8s::Action::"update"],\n'
                   f'  resource is k8s::Resource\n)\nwhen {{ resource has name && resource.name like "prod-*" }};\n')
        else:
            pol = (f'permit (\n  principal in k8s::Group::{json.dumps(g)},\n  action == k8s::Action::"get",\n  resource is k8s::NonResourceURL\n)\n'
                   f'when {{ resource.path like "/healthz*" || ["/version", "/version/"].contains(resource.path) }};\n')
        out.append(pol)
    return "\n".join(out)


def sars_json(sars: List[dict]) -> str:
    return json.dumps(sars, separators=(",", ":"))


def admission_objects(n: int, seed: int = 41) -> List[Tuple[str, dict]]:
    """C4 object corpus: (kind, unstructured object) for ConfigMaps and Secrets."""
    rng = np.random.Generator(np.random.PCG64(seed))
    out = []
    for i in range(n):
        kind = "ConfigMap" if rng.random() < 0.6 else "Secret"
        nl = int(rng.integers(0, 17))
        labels = {f"label-{int(x)}": f"v{int(y)}" for x, y in zip(rng.integers(0, 40, nl), rng.integers(0, 5, nl))}
        if rng.random() < 0.7:
            labels["owner"] = f"user-{int(rng.integers(0, 200)):05d}"
        nd = int(rng.integers(0, 9))
        data = {f"key{j}": f"value{int(rng.integers(0, 100))}" for j in range(nd)}
        name = ("prod-" if rng.random() < 0.2 else "") + f"{kind.lower()}-{i}"
        obj = {"apiVersion": "v1", "kind": kind, "metadata": {"name": name, "namespace": f"ns-{i % 20:03d}",
                                                               "labels": labels}, "data": data}
        out.append((kind, obj))
    return out


def admission_reviews(n: int, seed: int = 43, objects: Optional[List[Tuple[str, dict]]] = None) -> List[dict]:
    """C4 AdmissionReview requests (admission.k8s.io/v1) over ConfigMap / Secret objects, as the
    reference's /v1/admit handler receives them: CREATE / UPDATE / DELETE with object / oldObject,
    users with groups."""
    rng = np.random.Generator(np.random.PCG64(seed))
    objs = objects or admission_objects(max(n, 2), seed=seed)
    out = []
    for i in range(n):
        kind, obj = objs[i % len(objs)]
        op = ["CREATE", "UPDATE", "DELETE"][int(rng.integers(0, 3))]
        old = objs[(i + 1) % len(objs)][1]
        user = {"username": ["test-user", "sample-user", f"user-{int(rng.integers(0, 200)):05d}"][i % 3], "uid": "",
                "groups": ["requires-labels"] if rng.random() < 0.5 else ["viewers", "system:authenticated"]}
        req = {"uid": f"req-{i}", "kind": {"group": "", "version": "v1", "kind": kind},
               "resource": {"group": "", "version": "v1", "resource": kind.lower() + "s"},
               "name": obj["metadata"]["name"], "namespace": obj["metadata"]["namespace"], "operation": op,
               "userInfo": user,
               "object": obj if op != "DELETE" else None,
               "oldObject": (obj if op == "DELETE" else old) if op != "CREATE" else None}
        out.append({"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "request": req})
    return out


def admission_policies(n: int, seed: int = 3) -> str:
    """C4: admission forbids on ConfigMap / Secret objects (name prefix globs, label and data
    key/value contains, has-guards, oldObject comparisons), the shapes of demo/admission-policy.yaml."""
    rng = np.random.Generator(np.random.PCG64(seed))
    acts = ['k8s::admission::Action::"create"', 'k8s::admission::Action::"update"', 'k8s::admission::Action::"delete"']
    out = []
    for i in range(n):
        kind = "ConfigMap" if rng.random() < 0.6 else "Secret"
        user = ["test-user", "sample-user", f"user-{int(rng.integers(0, 200)):05d}"][int(rng.integers(0, 3))]
        t = rng.random()
        if t < 0.3:
            out.append(f'forbid (\n  principal is k8s::User,\n  action in [{acts[0]}, {acts[1]}],\n  resource is core::v1::{kind}\n)\n'
                       f'when {{ principal.name == {json.dumps(user)} && resource.metadata.name like "prod-*" }};\n')
        elif t < 0.55:
            out.append(f'forbid (\n  principal is k8s::User in k8s::Group::"requires-labels",\n  action in [{", ".join(acts)}],\n'
                       f'  resource is core::v1::{kind}\n)\nunless {{ resource has metadata && resource.metadata has labels && '
                       f'resource.metadata.labels.contains({{"key": "owner", "value": principal.name}}) }};\n')
        elif t < 0.8:
            ns = f"ns-{int(rng.integers(0, 20)):03d}"
            lab = f"label-{int(rng.integers(0, 40))}"
            out.append(f'forbid (\n  principal,\n  action == {acts[1]},\n  resource is core::v1::{kind}\n)\n'
                       f'when {{ resource.metadata.namespace == {json.dumps(ns)} && resource has oldObject && '
                       f'resource.oldObject.metadata has labels && '
                       f'resource.oldObject.metadata.labels.contains({{"key": {json.dumps(lab)}, "value": "v{int(rng.integers(0, 5))}"}}) }};\n')
        else:
            out.append(f'forbid (\n  principal,\n  action in [{acts[0]}, {acts[1]}],\n  resource is core::v1::{kind}\n)\n'
                       f'when {{ resource has data && resource.data.contains({{"key": "key{int(rng.integers(0, 9))}", '
                       f'"value": "value{int(rng.integers(0, 100))}"}}) }};\n')
    return "\n".join(out)


def multitenant_policies(n: int, seed: int = 51, pop: Optional[Population] = None) -> List[Tuple[str, str, str]]:
    """C5: `n` policies across the population's namespaces as tenants, one Policy CRD document per
    tenant ((name, uid, text) for CRDStore): group-scoped permits on the tenant's namespace and
    resource, and production-name forbids."""
    pop = pop or Population(seed=7, n_namespaces=1000)
    rng = np.random.Generator(np.random.PCG64(seed))
    per = max(1, n // len(pop.namespaces))
    gi = _zipf_idx(rng, len(pop.groups), n, s=0.9)
    ri = rng.integers(len(RESOURCES), size=n)
    u = rng.random((n, 2))
    docs = []
    k = 0
    for t, ns in enumerate(pop.namespaces):
        out = []
        for i in range(per if t < len(pop.namespaces) - 1 else n - per * (len(pop.namespaces) - 1)):
            g = pop.groups[int(gi[k])]
            grp, ver, res = RESOURCES[int(ri[k])]
            if u[k, 0] < 0.85:
                verbs = ["get", "list", "watch"] if u[k, 1] < 0.6 else ["create", "update", "patch", "delete"]
                out.append(f'permit (\n  principal in k8s::Group::{json.dumps(g)},\n  {_actions(verbs)},\n'
                           f'  resource is k8s::Resource\n)\nwhen {{ resource has namespace && resource.namespace == '
                           f'{json.dumps(ns)} && resource.resource == {json.dumps(res)} }};\n')
            else:
                out.append(f'forbid (\n  principal,\n  action in [k8s::Action::"delete", k8s::Action::"update"],\n'
                           f'  resource is k8s::Resource\n)\nwhen {{ resource has namespace && resource.namespace == '
                           f'{json.dumps(ns)} && resource has name && resource.name like "prod-*" }};\n')
            k += 1
        docs.append((f"tenant-{t:04d}", f"uid-{t:04d}", "\n".join(out)))
    return docs
