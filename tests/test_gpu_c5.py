"""C5 under -m gpu: the 100k-policy multi-tenant image (1,000 tenant Policy CRDs) and a hot reload
while a batch bound to the old epoch is still in flight (crd.go:45-118 mutates the
policy set per CRD event while requests keep being served).

The reload's new epoch carries three CRD events at once: one tenant's permits turned into forbids
(update), one tenant's CRD replaced by text that does not parse (skipped, crd.go:51-55,91-95 — its
old policies are removed, the others' edits still apply) and one tenant deleted. The in-flight
batch must finish on the epoch it was submitted against; the next batch must see every edit. Both
are checked against the C++ oracle (oracle/cedar_ref.cpp) built from the matching store snapshot."""
import json
import random
import re

import pytest

import cedargpu
from cedargpu import synth
from cedar_ref import RefPolicySet, items_json
import cedar_oracle as co
import k8s_model as km

pytestmark = pytest.mark.gpu

N_REQ = 600


@pytest.fixture(scope="module")
def ctx():
    assert cedargpu.device_count() >= 1, "GPU tests need a GPU"
    c = cedargpu.Context(0)
    yield c
    c.close()


def _items(sars):
    out = []
    for s in sars:
        a = km.attributes_from_sar(s)
        em, req = km.record_to_cedar_resource(a)
        out.append((co.entities_to_json(em), co.request_to_json(req)))
    return out


_PERMIT = re.compile(r'principal in k8s::Group::"([^"]+)",\s*action in \[([^\]]*)\],.*?resource\.namespace == "([^"]+)" '
                     r'&& resource\.resource == "([^"]+)"', re.S)


def _targeted(docs, tenants, n_each, seed):
    """SARs that a tenant's permits (and, for delete / update of prod-* names, its forbids) decide."""
    r = random.Random(seed)
    api = {res: (grp, ver) for grp, ver, res in synth.RESOURCES}
    out = []
    for t in tenants:
        pols = _PERMIT.findall(docs[t][2])
        for k in range(n_each):
            g, acts, ns, res = r.choice(pols)
            verb = r.choice(re.findall(r'"([^"]+)"', acts))
            grp, ver = api[res]
            name = r.choice(["", "web-1", "prod-db"])
            out.append(synth.make_sar(f"user-{t}-{k}", f"uid-{k}", [g, "system:authenticated"], verb, ns=ns, group=grp,
                                      version=ver, resource=res, name=name))
    return out


def _want(docs, items):
    ref = RefPolicySet.from_stores([cedargpu.CRDStore(docs)])
    ref.load_items(items_json(items))
    got = ref.evaluate(16)
    ref.close()
    return [(ok, diag) for ok, _, diag, _ in got]


def _batch(ctx, items):
    b = ctx.batch()
    b.add_json(json.dumps([{"entities": e, "request": r} for e, r in items]))
    return b


def _results(b):
    return [(b.decision(i)[0], b.diagnostic(i)) for i in range(len(b))]


def test_c5_100k_reload_with_batch_in_flight(ctx):
    pop = synth.Population(seed=7, n_namespaces=1000)
    docs = synth.multitenant_policies(100_000, seed=51, pop=pop)
    # requests aimed at a few tenants, the edited ones among them, plus random traffic
    sars = synth.random_sars(N_REQ // 2, seed=5001, pop=pop) + _targeted(docs, (3, 500, 501, 502, 777), N_REQ // 10, 9)
    items = _items(sars)

    comp = cedargpu.Compiler()
    img1 = comp.build([cedargpu.CRDStore(docs)], epoch=1)
    assert cedargpu.image_stats(img1)["policies"] == 100_000
    ctx.load(img1, 1)

    docs2 = list(docs)
    name, uid, text = docs2[500]
    docs2[500] = (name, uid, text.replace("permit", "forbid"))                  # update
    docs2[501] = (docs2[501][0], docs2[501][1], "permit (principal, action, resource) when { 1 + };")  # broken
    del docs2[502]                                                              # delete

    # batch A is submitted against epoch 1; epoch 2 is compiled and activated while A runs
    a = _batch(ctx, items)
    a.submit()
    img2 = comp.build([cedargpu.CRDStore(docs2)], epoch=2)
    errs = comp.doc_errors()
    assert [e["filename"] for e in errs] == [docs2[501][0]], errs
    st = comp.cache_stats()
    assert st["hits"] >= 997, st  # only the edited documents were parsed again
    lb = comp.last_build()
    assert lb["incremental"] and lb["lowered"] <= 300, lb  # ... and lowered again
    comp.close()
    ctx.load(img2, 2)
    b = _batch(ctx, items)
    b.submit()
    a.wait()
    b.wait()
    got_a, got_b = _results(a), _results(b)
    a.close()
    b.close()

    want_a, want_b = _want(docs, items), _want(docs2, items)
    assert got_a == want_a
    assert got_b == want_b
    # the edits are visible: some decision changed between the epochs
    assert sum(1 for x, y in zip(want_a, want_b) if x != y) > 0


def test_incremental_image_decides_like_a_fresh_build(ctx):
    """An incremental rebuild (only the changed CRDs lowered, the rest copied from the previous
    build) decides every request exactly as a full build of the same stores: decision and the
    full diagnostic for 4,096 SARs over the ABAC corpus on a static group DAG, and both agree with
    the C++ oracle on a sample."""
    pop = synth.Population(seed=12, n_users=800, n_groups=300, dag_depth=6)
    ents = pop.static_entities()
    pols = [p for p in synth.abac_policies(2000, seed=13, pop=pop).split("\n\n") if p.strip()]
    docs = [(f"team-{i:03d}", f"uid-{i}", "\n\n".join(pols[i * 50:(i + 1) * 50])) for i in range(40)]
    comp = cedargpu.Compiler()
    comp.build([cedargpu.CRDStore(docs)], epoch=11, entities=ents)
    docs2 = list(docs)
    docs2[3] = (docs2[3][0], docs2[3][1], docs2[3][2].replace("permit", "forbid"))  # update
    del docs2[17]                                                                    # delete
    docs2.append(("team-new", "uid-new", "\n\n".join(pols[50:80])))                 # add
    inc = comp.build([cedargpu.CRDStore(docs2)], epoch=12, entities=ents)
    assert comp.last_build()["incremental"], comp.last_build()
    comp.close()
    fresh = cedargpu.Compiler(incremental=False).build([cedargpu.CRDStore(docs2)], epoch=13, entities=ents)
    assert inc != fresh
    sars = synth.random_sars(4096, seed=14, pop=pop)
    got = []
    for img, ep in ((inc, 12), (fresh, 13)):
        ctx.load(img, ep)
        b = ctx.batch()
        b.add_sar_json(synth.sars_json(sars))
        b.submit()
        b.wait()
        got.append([b.authz(i) for i in range(len(b))])
        b.close()
    assert got[0] == got[1]
    assert sum(1 for d, _ in got[0] if d == 1) > 100  # the corpus decides many requests
    # (SARs the authorizer answers before evaluation, authorizer.go:38-57, are left out)
    idx = [i for i, s in enumerate(sars[:400]) if not (s["spec"]["user"].startswith("system:") and not (
        s["spec"]["user"].startswith("system:serviceaccount:") or s["spec"]["user"].startswith("system:node:")))]
    items = _items([sars[i] for i in idx])
    ref = RefPolicySet.from_stores([cedargpu.CRDStore(docs2)], entities=ents)
    ref.load_items(items_json(items))
    want = ref.evaluate(16)
    ref.close()
    for (ok, _, diag, _), g in zip(want, [got[0][i] for i in idx]):
        wd = 1 if ok else (0 if diag.startswith('{"reasons"') else 2)
        assert g == (wd, diag if wd != 2 else "")


def test_delta_reload_decides_like_a_full_load(ctx):
    """§8 f2 delta images: CRD events (update, delete, add) compiled incrementally, shipped as a
    delta against the loaded epoch and rebuilt on the GPU (cg_image_load_delta) decide exactly as
    the full image loaded the ordinary way, and as the C++ oracle over the new store snapshot; a
    delta-loaded image serves as the base of the next delta; bad deltas are refused."""
    pop = synth.Population(seed=7, n_namespaces=200)
    docs = synth.multitenant_policies(20_000, seed=52, pop=pop)
    comp = cedargpu.Compiler()
    img1 = comp.build([cedargpu.CRDStore(docs)], epoch=21)
    ctx.load(img1, 21, activate=False)
    docs2 = list(docs)
    docs2[40] = (docs2[40][0], docs2[40][1], docs2[40][2].replace("permit", "forbid"))  # update
    del docs2[77]                                                                      # delete
    docs2.append(("tenant-new", "uid-new", docs[5][2]))                                # add
    img2 = comp.build([cedargpu.CRDStore(docs2)], epoch=22)
    docs3 = list(docs2)
    docs3[120] = (docs3[120][0], docs3[120][1], docs3[120][2].replace("permit", "forbid"))
    img3 = comp.build([cedargpu.CRDStore(docs3)], epoch=23)
    comp.close()
    d12, d23 = cedargpu.image_delta(img1, img2), cedargpu.image_delta(img2, img3)
    assert len(d23) < len(img3) // 100  # an update alone: a small delta
    ctx.load_delta(21, d12, 22, activate=False)
    ctx.load_delta(22, d23, 23, activate=False)  # the delta-loaded epoch as the next base
    ctx.load(img3, 24, activate=False)             # the same image, loaded in full
    sars = (synth.random_sars(1500, seed=5002, pop=pop) + _targeted(docs3, (40, 120, len(docs3) - 1), 60, 10))
    items = _items(sars)
    got = {}
    for ep in (23, 24):
        ctx.activate(ep)
        b = _batch(ctx, items)
        b.submit()
        b.wait()
        got[ep] = _results(b)
        b.close()
    assert got[23] == got[24]
    want = _want(docs3, items)
    assert got[23] == want
    # refusals: no such base, another base, a corrupted literal / operation
    with pytest.raises(cedargpu.CedarGPUError):
        ctx.load_delta(999, d12, 30)
    with pytest.raises(cedargpu.CedarGPUError):
        ctx.load_delta(23, d12, 31)
    bad = bytearray(d23)
    bad[-1] ^= 0xFF
    with pytest.raises(cedargpu.CedarGPUError):
        ctx.load_delta(22, bytes(bad), 32)
    ctx.activate(23)
