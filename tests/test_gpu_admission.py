"""Admission webhook end to end on the GPU (cg_batch_add_admission_json + cg_batch_admit: the C++
AdmissionReview model, the device evaluation over the policy tiers plus the static allow-all tier)
against the oracle's cedarHandler (oracle/k8s_model.py admission_handle, handler.go:43-80)."""
import json
import os

import pytest

import cedar_oracle as co
import k8s_model as km
from conftest import GOLDEN
from test_admission_encoder import _variants

import cedargpu
from cedargpu import synth

pytestmark = pytest.mark.gpu

CORPUS = json.load(open(os.path.join(GOLDEN, "reference_corpus.json")))


@pytest.fixture(scope="module")
def ctx():
    assert cedargpu.device_count() >= 1, "GPU tests need a GPU"
    c = cedargpu.Context(0)
    yield c
    c.close()


def _stores(text):
    return [cedargpu.MemoryStore("adm.cedar", text), cedargpu.ALLOW_ALL_ADMISSION]


def _oracle_tiers(text):
    ps = co.PolicySet()
    for d in cedargpu.MemoryStore("adm.cedar", text).documents():
        _, fname, body, pre, suf = d
        for i, p in enumerate(co.parse_policies(body, fname)):
            ps.add(f"{pre}{i}{suf}", p)
    return [ps, km.allow_all_admission_store()]


def _check(ctx, text, reviews):
    h = cedargpu.AdmissionHandler(_stores(text), ctx=ctx)
    got = h.handle_batch(reviews)
    tiers = _oracle_tiers(text)
    n_deny = 0
    for r, (allowed, code, msg) in zip(reviews, got):
        req = km.admission_request_from_review(r)
        try:
            want = km.admission_handle(tiers, req)
        except (km.WalkError, KeyError):
            assert (allowed, code) == (False, 500), r
            continue
        assert (allowed, msg) == want and code == 200, (r, allowed, msg, want)
        n_deny += not allowed
    return n_deny


def test_demo_admission_policies(ctx):
    """C4 at test scale: the demo admission policies over synthetic ConfigMap / Secret reviews."""
    text = "\n".join(v for k, v in sorted(CORPUS["demo"].items()) if k.startswith("admission"))
    assert _check(ctx, text, synth.admission_reviews(1500, seed=11)) > 0


def test_c4_admission_forbids(ctx):
    """C4 policy shapes: name prefix globs, label contains, has-guards, oldObject comparisons."""
    text = synth.admission_policies(200, seed=3)
    assert _check(ctx, text, synth.admission_reviews(1500, seed=12)) > 0


def test_c4_bench_size_vs_cpp_oracle(ctx):
    """C4 at its bench configuration (BENCH configs.c4_admission_1k): 1,000 admission forbids plus
    the allow-all tier over 4,096 ConfigMap / Secret reviews of the bench's generator, where about
    half of the requests collect more hits than the first pass holds and finish in the large stage.
    Every review's (allowed, code, message) against the C++ oracle (oracle/cedar_ref.cpp) through
    handler.go:43-80's mapping (km.admission_handle)."""
    from cedar_ref import RefPolicySet, items_json
    text = synth.admission_policies(1000, seed=3)
    reviews = synth.admission_reviews(4096, seed=4000)
    h = cedargpu.AdmissionHandler(_stores(text), ctx=ctx)
    got = h.handle_batch(reviews)
    want, items, idx = {}, [], []
    for i, r in enumerate(reviews):
        req = km.admission_request_from_review(r)
        if req.namespace in ("kube-system", "cedar-k8s-authz-system"):
            want[i] = (True, 200, "")
            continue
        try:
            em, creq = km.admission_to_cedar(req)
        except (km.WalkError, KeyError):
            want[i] = (False, 500, None)
            continue
        items.append((co.entities_to_json(em), co.request_to_json(creq)))
        idx.append(i)
    ref = RefPolicySet.from_stores(_stores(text))
    ref.load_items(items_json(items))
    for i, (ok, _, _, reasons) in zip(idx, ref.evaluate(16)):
        want[i] = (ok, 200, reasons if not ok and reasons not in ("", "[]", "null") else "")
    ref.close()
    n_deny = n_long = 0
    for i, g in enumerate(got):
        w = want[i]
        if w[1] == 500:
            assert g[:2] == (False, 500), (i, g)
            continue
        assert tuple(g) == w, (i, reviews[i], g, w)
        n_deny += not g[0]
        n_long += not g[0] and g[2].count('"policy"') > 64  # more reasons than the first pass holds
    assert n_deny > 1000 and n_long > 0, (n_deny, n_long)


def test_admission_variants(ctx):
    text = "\n".join(v for k, v in sorted(CORPUS["demo"].items()) if k.startswith("admission"))
    out, errs = _variants()
    _check(ctx, text, out + errs)
