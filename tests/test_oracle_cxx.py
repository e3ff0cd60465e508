"""Pins the C++ oracle (oracle/cedar_ref.cpp) to the Python oracle and to the reference's vectors.

The C++ restatement is what large GPU parity runs and bench.py's CPU baseline use, so it must agree
with the readable Python restatement (itself pinned to the reference's TestAuthorize /
TestTieredIsAuthorized vectors, tests/test_oracle_golden.py) bit for bit: decision, deciding tier,
the full json.Marshal(Diagnostic) string and the admission reasons string."""
import json
import os

import pytest

import cedar_oracle as co
import k8s_model as km
from cedar_ref import RefPolicySet, items_json
from conftest import GOLDEN
from randgen import Gen

V = json.load(open(os.path.join(GOLDEN, "reference_vectors.json")))
CORPUS = json.load(open(os.path.join(GOLDEN, "reference_corpus.json")))


def _py_tiers(docs_per_tier):
    out = []
    for docs in docs_per_tier:
        ps = co.PolicySet()
        for fname, text in docs:
            for i, p in enumerate(co.parse_policies(text, fname)):
                ps.add(f"policy{i}", p)
        out.append(ps)
    return out


def _ref(docs_per_tier, statics=None):
    r = RefPolicySet()
    if statics:
        r.set_entities(json.dumps(statics))
    for docs in docs_per_tier:
        r.add_tier()
        for fname, text in docs:
            r.add_document(fname, text, "policy", "")
    return r


def _compare(docs_per_tier, items, threads=4, statics=None):
    py = _py_tiers(docs_per_tier)
    ref = _ref(docs_per_tier, statics)
    sem = co.entities_from_json(statics) if statics else None
    assert ref.load_items(items_json(items)) == len(items)
    got = ref.evaluate(threads)
    for (ents, req), (ok, tier, diag, reasons) in zip(items, got):
        em = co.merge_static_entities(co.entities_from_json(ents), sem)
        want_ok, want_diag, want_tier = co.tiered_is_authorized(py, em, co.request_from_json(req))
        assert (ok, tier) == (want_ok, want_tier), req
        assert diag == want_diag.to_go_json(), req
        assert reasons == want_diag.reasons_json(), req
    ref.close()


@pytest.mark.parametrize("case", V["tiers"]["cases"], ids=lambda c: c["name"])
def test_cxx_tier_vectors(case):
    """store_test.go:21-188 through the C++ oracle."""
    r = _ref([[("in-memory-test-store.cedar", s)] for s in case["stores"]])
    r.load_items(items_json([(V["tiers"]["entities"], V["tiers"]["request"])]))
    (ok, tier, diag, _), = r.evaluate(1)
    assert ok == case["want"]
    assert json.loads(diag) == case["want_diag"]


@pytest.mark.parametrize("case", V["authorize"], ids=lambda c: c["name"])
def test_cxx_authorize_vectors(case):
    """authorizer_test.go:462-920: the Cedar decision + Diagnostic the reason string is made from."""
    a = km.Attributes(**{k: v for k, v in case["attributes"].items() if k not in ("user", "label_selector", "field_selector")},
                      user=km.UserInfo(**case["attributes"].get("user", {})),
                      label_selector=[km.LabelRequirement(**x) for x in case["attributes"].get("label_selector", [])],
                      field_selector=[km.FieldRequirement(**x) for x in case["attributes"].get("field_selector", [])])
    em, req = km.record_to_cedar_resource(a)
    ps = co.PolicySet.from_bytes(case["name"], case["policy"])
    want_ok, want_diag, _ = co.tiered_is_authorized([ps], em, req)
    r = _ref([[(case["name"], case["policy"])]])
    r.load_items(items_json([(co.entities_to_json(em), co.request_to_json(req))]))
    (ok, _, diag, _), = r.evaluate(1)
    assert ok == want_ok and diag == want_diag.to_go_json()
    if case["store_complete"] and case["want_decision"] in (0, 1) and "system:" not in str(case["attributes"]):
        assert diag == case["want_reason"] or case["want_reason"] == ""


@pytest.mark.parametrize("seed", range(6))
def test_cxx_random_general_policies(seed):
    g = Gen(seed)
    tiers = [[("t%d.cedar" % t, g.policies(40))] for t in range(1 + seed % 3)]
    items = [g.item() for _ in range(60)]
    _compare(tiers, items)


@pytest.mark.parametrize("seed", range(4))
def test_cxx_random_atomic_policies(seed):
    g = Gen(100 + seed)
    tiers = [[("a%d.cedar" % t, g.atomic_policies(50))] for t in range(1 + seed % 2)]
    items = [g.item() for _ in range(60)]
    _compare(tiers, items)


@pytest.mark.parametrize("seed", range(4))
def test_cxx_static_entities(seed):
    """Static entities (an image-level hierarchy) merged into every EntityMap: the C++ oracle's
    lookup fallback against the Python oracle's merge_static_entities."""
    g = Gen(300 + seed, static=True)
    statics = g.static_entities()
    tiers = [[("s%d.cedar" % t, g.policies(40) if seed % 2 else g.atomic_policies(50))] for t in range(1 + seed % 2)]
    items = [g.item() for _ in range(80)]
    _compare(tiers, items, statics=statics)


def test_merge_static_entities_semantics():
    """A UID in both maps keeps the request's attributes and unites the parents; a UID only in the
    static map is added; the request's other entities are untouched."""
    req = co.entities_from_json([{"uid": {"type": "G", "id": "a"}, "attrs": {"n": 1}, "parents": [{"type": "G", "id": "x"}]},
                                 {"uid": {"type": "U", "id": "u"}, "attrs": {}, "parents": [{"type": "G", "id": "a"}]}])
    st = co.entities_from_json([{"uid": {"type": "G", "id": "a"}, "attrs": {"n": 2}, "parents": [{"type": "G", "id": "b"}]},
                                {"uid": {"type": "G", "id": "b"}, "attrs": {}, "parents": [{"type": "G", "id": "c"}]}])
    m = co.merge_static_entities(req, st)
    a = m[co.EntityUID("G", "a")]
    assert a.attrs == co.Record({"n": co.Long(1)}) and set(a.parents) == {co.EntityUID("G", "x"), co.EntityUID("G", "b")}
    assert co.EntityUID("G", "b") in m and co.entity_in(m, co.EntityUID("U", "u"), co.EntityUID("G", "c"))


def test_cxx_demo_and_converter_corpus():
    from cedargpu import synth
    docs = [(k, v) for k, v in sorted(CORPUS["converter"].items())]
    demo = [(k, v) for k, v in sorted(CORPUS["demo"].items())]
    sars = synth.random_sars(150, seed=3, pop=synth.Population(seed=3, n_users=300, n_groups=40))
    items = []
    for s in sars:
        em, req = km.record_to_cedar_resource(km.attributes_from_sar(s))
        items.append((co.entities_to_json(em), co.request_to_json(req)))
    _compare([docs], items)
    _compare([demo, docs], items)


def test_cxx_parse_error_reported():
    r = RefPolicySet()
    with pytest.raises(Exception):
        r.add_document("bad.cedar", "permit(principal, action, resource) when { ;", "policy", "")


def test_cxx_bench_runs():
    g = Gen(7)
    r = _ref([[("b.cedar", g.policies(20))]])
    r.load_items(items_json([g.item() for _ in range(16)]))
    n, wall = r.bench(2, 0.05)
    assert n > 0 and wall > 0
