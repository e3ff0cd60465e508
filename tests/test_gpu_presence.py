"""Presence masks and equality filters (image.h): the scan lists a bucket from the scope bitsets
only when the request has every attribute its policies' `has` atoms require, where those atoms
come before anything that can raise (and, in a bucket of a key's value, after the key atom), and
when no equality after the key atom that all its policies share is false for the request. Policies
with `has` before, after and instead of their key atom, on a false path, and behind atoms that
raise, against SubjectAccessReviews with and without those attributes: every decision and
diagnostic equal to the C++ oracle's (oracle/cedar_ref.cpp), on the split first pass (the bitset
path) and on the one-launch small path."""
import pytest

import cedar_oracle as co
import k8s_model as km

import cedargpu
from cedargpu import synth
from test_gpu_parity import check_items_ref, ctx  # noqa: F401 (the module's GPU context fixture)

pytestmark = pytest.mark.gpu


def _policies(groups):
    sel = '[{"key": "owner", "operator": "In", "values": [principal.name]}]'
    out = []
    for g in groups:
        scope = f'principal in k8s::Group::"{g}",\n  action,\n  resource is k8s::Resource'
        out += [
            # has after the key atom (the value bucket's mask: labelSelector)
            f'permit (\n  {scope}\n)\nwhen {{ resource.resource == "pods" && resource has labelSelector && '
            f'resource.labelSelector.containsAny({sel}) }};',
            # has before a prefix key
            f'permit (\n  {scope}\n)\nwhen {{ resource has name && resource.name like "prod-*" }};',
            # has after the key, then an equality on the guarded attribute
            f'forbid (\n  {scope}\n)\nwhen {{ resource.apiGroup == "apps" && resource has subresource && '
            f'resource.subresource == "status" }};',
            # an unguarded key that raises on cluster-scoped requests (its MISSING bucket: no mask)
            f'permit (\n  {scope}\n)\nwhen {{ resource.namespace == "ns-001" && resource has name }};',
            # has on the false path: requires the attribute to be absent
            f'permit (\n  {scope}\n)\nwhen {{ !(resource has name) && resource.resource == "secrets" }};',
            # unkeyed: the level-1 bucket's mask
            f'permit (\n  {scope}\n)\nwhen {{ resource has labelSelector }};',
            # a selector read with no guard: raises without one (never masked)
            f'permit (\n  {scope}\n)\nwhen {{ resource.resource == "deployments" && '
            f'resource.labelSelector.containsAny({sel}) }};',
            # equality filters: an equality after the key on an attribute a request may lack (the
            # atom raises: never skipped) ...
            f'permit (\n  {scope}\n)\nwhen {{ resource.resource == "configmaps" && resource.name == "configmap-5" }};',
            # ... and buckets whose policies agree on the filter or do not
            f'permit (\n  {scope}\n)\nwhen {{ resource.namespace == "ns-002" && resource.apiGroup == "apps" }};',
        ]
        if int(g[-1]) % 2 == 0:
            out.append(f'forbid (\n  {scope}\n)\nwhen {{ resource.namespace == "ns-002" && resource.apiGroup == "" }};')
    return "\n".join(out)


def _items(n, seed, pop):
    out = []
    for s in synth.random_sars(n, seed=seed, pop=pop):
        a = km.attributes_from_sar(s)
        if km.authorize([], a)[0] != km.DECISION_NO_OPINION:
            continue
        em, r = km.record_to_cedar_resource(a)
        out.append((co.entities_to_json(em), co.request_to_json(r)))
    return out


@pytest.mark.parametrize("small_n", [None, "0"])
def test_presence_masks_vs_oracle(ctx, small_n, monkeypatch):  # noqa: F811
    if small_n is not None:
        monkeypatch.setenv("CEDARGPU_SMALL_N", small_n)
    pop = synth.Population(seed=13, n_users=400, n_groups=12)
    stores = [cedargpu.MemoryStore("presence.cedar", _policies(pop.groups))]
    img = cedargpu.build_image(stores)
    assert cedargpu.image_stats(img)["indexed"]
    items = _items(2500, 17, pop)
    assert len(items) > 1500
    check_items_ref(ctx, stores, items, want_indexed=True)
