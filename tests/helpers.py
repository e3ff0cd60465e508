"""Shared test helpers: conversions between the oracle's model and the product's JSON inputs."""
import ctypes
import json

import cedar_oracle as co
import k8s_model as km


def attrs_from(d):
    d = dict(d)
    u = d.pop("user", {})
    ls = [km.LabelRequirement(**x) for x in d.pop("label_selector", [])]
    fs = [km.FieldRequirement(**x) for x in d.pop("field_selector", [])]
    return km.Attributes(user=km.UserInfo(**u), label_selector=ls, field_selector=fs, **d)


def sar_from_attrs(a: dict) -> dict:
    """Reference-test Attributes -> SubjectAccessReview JSON (inverse of server.go:163-203)."""
    u = a.get("user", {})
    spec = {"user": u.get("name", ""), "uid": u.get("uid", ""), "groups": list(u.get("groups", []))}
    if u.get("extra"):
        spec["extra"] = u["extra"]
    if a.get("resource_request"):
        ra = {"verb": a.get("verb", ""), "namespace": a.get("namespace", ""), "group": a.get("api_group", ""),
              "version": a.get("api_version", ""), "resource": a.get("resource", ""),
              "subresource": a.get("subresource", ""), "name": a.get("name", "")}
        spec["resourceAttributes"] = ra
    else:
        spec["nonResourceAttributes"] = {"path": a.get("path", ""), "verb": a.get("verb", "")}
    return {"spec": spec}


def cxx_sar_to_cedar(sar: dict) -> dict:
    import cedargpu
    lib = cedargpu.lib
    b = json.dumps(sar).encode()
    need = ctypes.c_size_t(0)
    rc = lib.cg_sar_to_cedar_json(b, len(b), None, 0, ctypes.byref(need))
    buf = ctypes.create_string_buffer(need.value)
    rc = lib.cg_sar_to_cedar_json(b, len(b), buf, need.value, ctypes.byref(need))
    assert rc == 0, rc
    return json.loads(buf.value.decode())


def norm_entities(arr):
    out = {}
    for e in arr:
        k = (e["uid"]["type"], e["uid"]["id"])
        out[k] = (co.value_from_json(e["attrs"]), frozenset((p["type"], p["id"]) for p in e["parents"]))
    return out


def oracle_item(em, req):
    return co.entities_to_json(em), co.request_to_json(req)
