"""Admission entity build (admission.cpp: cedarHandler.review, UnstructuredToRecord / walkObject,
UserToCedarEntity, the oldObject linkage and the admission action entities) against the oracle's
restatement (oracle/k8s_model.py admission_to_cedar), as Cedar JSON. Host only.

The oracle is pinned to the reference's own admission record case (entities/admission_test.go,
tests/test_oracle_golden.py). Set element order is compared as a set (Cedar sets are unordered and
the reference iterates Go maps); error texts are parity unpinned (no reference test holds them),
so an error is compared as an error."""
import copy
import ipaddress
import json

import pytest

import cedar_oracle as co
import k8s_model as km

import cedargpu
from cedargpu import synth


def _canon(v):
    if isinstance(v, dict):
        if set(v) == {"__extn"} and v["__extn"].get("fn") == "ip":  # IPv6 text forms differ, values not
            return {"ip": str(ipaddress.ip_interface(v["__extn"]["arg"]))}
        return {k: _canon(x) for k, x in v.items()}
    if isinstance(v, list):
        return sorted((_canon(x) for x in v), key=lambda x: json.dumps(x, sort_keys=True))
    return v


def _entity_map(ents):
    m = {}
    for e in ents:  # EntityMap semantics: a repeated UID replaces the earlier entity
        m[(e["uid"]["type"], e["uid"]["id"])] = {"attrs": _canon(e["attrs"]), "parents": _canon(e["parents"])}
    return m


def _oracle(review):
    req = km.admission_request_from_review(review)
    if req.namespace in ("kube-system", "cedar-k8s-authz-system"):
        return {"skip": True}
    try:
        em, r = km.admission_to_cedar(req)
    except (km.WalkError, KeyError):
        return {"error": True}
    return {"entities": co.entities_to_json(em), "request": co.request_to_json(r)}


def check(review):
    ours = cedargpu.admission_to_cedar_json(review)
    want = _oracle(review)
    if "skip" in want or "error" in want:
        assert set(ours) == set(want), (ours, review)
        return ours
    assert "entities" in ours, (ours, review)
    assert _entity_map(ours["entities"]) == _entity_map(want["entities"]), review
    assert _canon(ours["request"]) == _canon(want["request"]), review
    return ours


def test_synthetic_reviews_match_oracle():
    for r in synth.admission_reviews(400, seed=7):
        check(r)


def _base(kind="Pod", op="UPDATE", ns="default", group=""):
    obj = {"apiVersion": "v1", "kind": kind, "metadata": {"name": "x", "namespace": ns, "labels": {"app": "web"},
                                                         "annotations": {"a": "b"}}}
    return {"request": {"uid": "rid", "kind": {"group": group, "version": "v1", "kind": kind},
                        "resource": {"group": group, "version": "v1", "resource": kind.lower() + "s"},
                        "name": "x", "namespace": ns, "operation": op,
                        "userInfo": {"username": "alice", "uid": "", "groups": ["g1", "g1", "g2"],
                                     "extra": {"Scopes": ["s1", "s1", "s2"]}},
                        "object": obj, "oldObject": copy.deepcopy(obj)}}


def _variants():
    out = []
    for user in ("alice", "system:node:n1", "system:node:a:b", "system:serviceaccount:ns:sa",
                 "system:serviceaccount:a:b:c", ""):
        r = _base()
        r["request"]["userInfo"]["username"] = user
        out.append(r)
    for op in ("CREATE", "UPDATE", "DELETE", "CONNECT", "PATCH"):
        r = _base(op=op)
        if op == "CREATE":
            r["request"]["oldObject"] = None
        if op == "DELETE":
            r["request"]["object"] = None
        out.append(r)
    for ns in ("kube-system", "cedar-k8s-authz-system", ""):
        out.append(_base(ns=ns))
    r = _base()
    r["request"]["object"]["spec"] = {"nodeSelector": {"k": "v", "n": 3, "z": "after"},
                                      "containers": [{"name": "c", "ports": [{"containerPort": 80, "hostIP": "10.1.2.3"}]}],
                                      "hostNetwork": False, "empty": {}, "emptyList": [], "nested": {"a": {"b": {}}}}
    r["request"]["object"]["status"] = {"podIP": "10.0.0.1", "podIPs": ["10.0.0.1", "fd00::1"], "hostIP": "not-an-ip",
                                        "ip": "192.168.0.0/16", "phase": None}
    out.append(r)
    for kind, key in (("Secret", "data"), ("Secret", "stringData"), ("ConfigMap", "binaryData"), ("Service", "selector"),
                      ("ReplicationController", "selector")):
        r = _base(kind=kind)
        r["request"]["object"][key] = {"a": "1", "b": "2"}
        out.append(r)
    r = _base(kind="UserInfo", group="authentication")
    r["request"]["object"]["extra"] = {"k": ["v"]}
    out.append(r)
    r = _base(kind="UserInfo", group="authentication")
    r["request"]["object"]["extra"] = "not-a-map"
    out.append(r)
    errs = []
    r = _base(); r["request"]["object"]["spec"] = {"replicas": 1.5}; errs.append(r)
    r = _base(); r["request"]["object"]["items"] = [None, "x"]; errs.append(r)
    r = _base(); r["request"]["object"]["items"] = [{}, "x"]; errs.append(r)
    r = _base(); del r["request"]["object"]["kind"]; errs.append(r)
    r = _base(op="CREATE"); r["request"]["object"] = None; errs.append(r)
    r = _base(kind="Secret"); r["request"]["object"]["data"] = ["not", "a", "map"]; errs.append(r)
    deep = {}
    cur = deep
    for _ in range(40):
        cur["d"] = {}
        cur = cur["d"]
    cur["leaf"] = 1
    r = _base(); r["request"]["object"]["deep"] = deep; errs.append(r)
    return out, errs


def test_variant_reviews_match_oracle():
    out, errs = _variants()
    for r in out:
        check(r)
    for r in errs:
        assert "error" in check(r), r


def test_duplicate_keys_keep_the_last_value():
    text = ('{"request":{"uid":"u","kind":{"group":"","version":"v1","kind":"ConfigMap"},'
            '"resource":{"group":"","version":"v1","resource":"configmaps"},"name":"c","namespace":"d",'
            '"operation":"CREATE","userInfo":{"username":"bob"},'
            '"object":{"apiVersion":"v1","kind":"ConfigMap","metadata":{"name":"c","labels":{"a":"1","a":"2"}},'
            '"data":{"k":"x"},"data":{"k":"y"}}}}')
    ours = cedargpu.admission_to_cedar_json(json.loads(text))  # Python keeps the last value too
    want = _oracle(json.loads(text))
    assert _entity_map(ours["entities"]) == _entity_map(want["entities"])
    b = text.encode()
    import ctypes
    from cedargpu._lib import lib
    buf = ctypes.create_string_buffer(1 << 16)
    need = ctypes.c_size_t()
    assert lib.cg_admission_to_cedar_json(b, len(b), buf, 1 << 16, ctypes.byref(need)) == 0
    raw = json.loads(buf.value.decode())
    assert _entity_map(raw["entities"]) == _entity_map(want["entities"])
