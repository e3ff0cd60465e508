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


def test_admission_variants(ctx):
    text = "\n".join(v for k, v in sorted(CORPUS["demo"].items()) if k.startswith("admission"))
    out, errs = _variants()
    _check(ctx, text, out + errs)
