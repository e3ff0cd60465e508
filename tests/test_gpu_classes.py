"""GPU parity of duplicate classes reported whole (image.h RS_CLASS): policies whose records agree
word for word are filed once, and the candidate pass records a holding class in one hit slot under
its representative; the host lists the members in policy order (Batch::reason_ids). Classes larger
than the first pass's hit slots (admission's `requires-labels` forbids: ~150 members), classes
interleaved by index with single policies and with each other, classes that err (every member
recorded with the error), permits and forbids over two tiers, on the split first pass of a large
batch and on the one-launch small-batch kernel, against the oracle."""
import pytest

import cedargpu
from cedargpu import synth

from test_gpu_parity import check_items, check_items_ref, ctx  # noqa: F401  (module fixture)

pytestmark = pytest.mark.gpu


def _policies(seed):
    import random
    r = random.Random(seed)
    out = []
    shapes = [
        'forbid (principal, action == A::"w", resource) when {{ resource.owner != principal.name }};',
        'permit (principal, action in [A::"r", A::"w"], resource) when {{ resource.team == "t{k}" }};',
        'permit (principal, action == A::"r", resource) when {{ resource.level > {k} }};',
        'forbid (principal, action == A::"r", resource) when {{ resource.secret }};',  # errs without `has`
        'permit (principal, action == A::"x", resource);',
    ]
    for i in range(900):
        s = r.random()
        if s < 0.25:
            out.append(shapes[0].format())  # one class of ~225 forbids
        elif s < 0.45:
            out.append(shapes[1].format(k=r.randint(0, 2)))  # three classes
        elif s < 0.6:
            out.append(shapes[2].format(k=r.randint(0, 40)))  # small classes and singles
        elif s < 0.7:
            out.append(shapes[3].format())  # an erroring class
        elif s < 0.8:
            out.append(shapes[4].format())
        else:  # singles
            out.append(f'permit (principal == U::"u{i % 7}", action == A::"r", resource) when {{ resource.level == {i} }};')
    return "\n".join(out)


def _items(n, seed):
    import random
    r = random.Random(seed)
    items = []
    for i in range(n):
        u = f"u{r.randint(0, 9)}"
        attrs = {"owner": u if r.random() < 0.5 else "other", "team": f"t{r.randint(0, 3)}", "level": r.randint(0, 60)}
        if r.random() < 0.6:
            attrs["secret"] = r.random() < 0.3
        ents = [{"uid": {"type": "U", "id": u}, "attrs": {"name": u}, "parents": []},
                {"uid": {"type": "R", "id": f"r{i}"}, "attrs": attrs, "parents": []}]
        req = {"principal": {"type": "U", "id": u}, "action": {"type": "A", "id": r.choice("rwx")},
               "resource": {"type": "R", "id": f"r{i}"}, "context": {}}
        items.append((ents, req))
    return items


@pytest.mark.parametrize("small_n", [None, "0"])
def test_classes_whole(ctx, small_n, monkeypatch):  # noqa: F811
    if small_n is not None:
        monkeypatch.setenv("CEDARGPU_SMALL_N", small_n)
    stores = [cedargpu.MemoryStore("a.cedar", _policies(1)), cedargpu.MemoryStore("b.cedar", _policies(2))]
    img = cedargpu.build_image(stores)
    assert cedargpu.image_stats(img)["indexed"]
    items = _items(1200, 3)
    check_items_ref(ctx, stores, items)
    check_items(ctx, stores, items[:300])


@pytest.mark.parametrize("small_n", [None, "0"])
def test_admission_classes(ctx, small_n, monkeypatch):  # noqa: F811
    """C4's shape: 1k admission forbids (two ~125-member `requires-labels` classes) plus the
    allow-all tier over synthetic AdmissionReviews, reasons included, vs the oracle."""
    import cedar_oracle as co
    import k8s_model as km
    from cedar_ref import RefPolicySet, items_json
    if small_n is not None:
        monkeypatch.setenv("CEDARGPU_SMALL_N", small_n)
    stores = [cedargpu.MemoryStore("adm.cedar", synth.admission_policies(1000, seed=3)), cedargpu.ALLOW_ALL_ADMISSION]
    reviews = synth.admission_reviews(3000, seed=4000)
    items = []
    for rv in reviews:
        em, req = km.admission_to_cedar(km.admission_request_from_review(rv))
        items.append((co.entities_to_json(em), co.request_to_json(req)))
    tiers = cedargpu.TieredPolicyStores(stores, ctx=ctx)
    got = tiers.is_authorized_batch(items)
    ref = RefPolicySet.from_stores(stores)
    ref.load_items(items_json(items))
    want = ref.evaluate(8)
    ref.close()
    long_lists = 0
    for k, ((ok, diag), (wok, _, wdiag, _)) in enumerate(zip(got, want)):
        assert (ok, diag) == (wok, wdiag), k
        long_lists += diag.count('"policy"') > 64
    assert long_lists > 100  # the class-sized deciding lists this test is about
