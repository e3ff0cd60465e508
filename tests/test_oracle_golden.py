"""Pins the CPU oracle against the reference's own test vectors."""
import json
import os

import pytest

import cedar_oracle as co
import k8s_model as km
from conftest import GOLDEN

V = json.load(open(os.path.join(GOLDEN, "reference_vectors.json")))
CORPUS = json.load(open(os.path.join(GOLDEN, "reference_corpus.json")))


def attrs_from(d):
    d = dict(d)
    u = d.pop("user", {})
    ls = [km.LabelRequirement(**x) for x in d.pop("label_selector", [])]
    fs = [km.FieldRequirement(**x) for x in d.pop("field_selector", [])]
    return km.Attributes(user=km.UserInfo(**u), label_selector=ls, field_selector=fs, **d)


@pytest.mark.parametrize("case", V["authorize"], ids=lambda c: c["name"])
def test_authorize_vectors(case):
    """authorizer_test.go:462-920 — decision and exact reason string."""
    ps = co.PolicySet.from_bytes(case["name"], case["policy"])
    dec, reason = km.authorize([ps], attrs_from(case["attributes"]), stores_loaded=case["store_complete"])
    assert dec == case["want_decision"]
    assert reason == case["want_reason"]


@pytest.mark.parametrize("case", V["tiers"]["cases"], ids=lambda c: c["name"])
def test_tier_vectors(case):
    """store_test.go:21-188 — tier semantics + MarshalIndent of the Diagnostic."""
    em = co.entities_from_json(V["tiers"]["entities"])
    req = co.request_from_json(V["tiers"]["request"])
    tiers = [co.PolicySet.from_bytes("in-memory-test-store.cedar", s) for s in case["stores"]]
    ok, diag, _ = co.tiered_is_authorized(tiers, em, req)
    assert ok == case["want"]
    assert json.loads(diag.to_go_json()) == case["want_diag"]


def _norm_entities(arr):
    out = {}
    for e in arr:
        k = (e["uid"]["type"], e["uid"]["id"])
        out[k] = (co.value_from_json(e["attrs"]), frozenset((p["type"], p["id"]) for p in e["parents"]))
    return out


@pytest.mark.parametrize("case", V["record_to_cedar"], ids=lambda c: c["name"])
def test_record_to_cedar_vectors(case):
    """authorizer_test.go:31-460 — exact EntityMap + Request construction."""
    em, req = km.record_to_cedar_resource(attrs_from(case["attributes"]))
    got = _norm_entities(co.entities_to_json(em))
    assert got == _norm_entities(case["want_entities"])
    assert co.request_to_json(req) == case["want_request"]


@pytest.mark.parametrize("case", V["paths"])
def test_path_vectors(case):
    """entities/authorization_test.go:10-57"""
    assert km.resource_request_to_path(attrs_from(case["attributes"])) == case["want"]


def test_unstructured_vector():
    """entities/admission_test.go:15-90"""
    c = V["unstructured"][0]
    rec = km.unstructured_to_record(c["input"], c["group"], c["version"], c["kind"])
    assert rec == co.value_from_json(c["want"])


@pytest.mark.parametrize("name", sorted(CORPUS["converter"]) + sorted(CORPUS["demo"]))
def test_corpus_parses(name):
    """Converter goldens (internal/convert/testdata) and demo policies are valid Cedar."""
    src = CORPUS["converter"].get(name) or CORPUS["demo"][name]
    ps = co.parse_policies(src, name)
    # invalid-service-account.cedar is empty by design: the converter skips the bad subject
    assert len(ps) >= (0 if name == "invalid-service-account.cedar" else 1)
    for p in ps:
        assert p.effect in ("permit", "forbid")


def test_converter_policy_counts():
    counts = {k: len(co.parse_policies(v, k)) for k, v in CORPUS["converter"].items()}
    assert counts["non-resource-url.cedar"] == 7
    assert counts["invalid-service-account.cedar"] == 0
    assert sum(counts.values()) > 40


def test_position_first_token_with_annotation():
    src = "\n\n@id(\"x\")\npermit(principal, action, resource);"
    p = co.parse_policies(src, "f")[0]
    assert (p.offset, p.line, p.col) == (2, 3, 1)
    assert p.annotations == {"id": "x"}


def test_go_json_html_escape():
    d = co.Diagnostic([co.DiagReason("a<b>&", "f", 0, 1, 1)], [])
    assert d.to_go_json() == '{"reasons":[{"policy":"a\\u003cb\\u003e\\u0026","position":{"filename":"f","offset":0,"line":1,"column":1}}]}'
