"""Serving queue (cg_queue_*): concurrent blocking per-request calls batched onto the GPU must give
the same (authorizer.Decision, reason) as the oracle's Authorize (authorizer.go:36-86) for every
request, whichever batch it lands in."""
import json
import os
import threading

import pytest

import cedar_oracle as co
import k8s_model as km
from conftest import GOLDEN

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


def _oracle_tiers(text):
    """The oracle's policy set for MemoryStore("demo.cedar", text), IDs as the store assigns them."""
    ps = co.PolicySet()
    for d in cedargpu.MemoryStore("demo.cedar", text).documents():
        _, fname, body, pre, suf = d
        for i, p in enumerate(co.parse_policies(body, fname)):
            ps.add(f"{pre}{i}{suf}", p)
    return [ps]


def _demo():
    return "\n".join(v for k, v in sorted(CORPUS["demo"].items()))


def _load(ctx, stores, epoch):
    ctx.load(cedargpu.build_image(stores, epoch=epoch), epoch)


@pytest.mark.parametrize("max_batch,delay_us,threads", [(4096, 0, 32), (7, 0, 16), (64, 2000, 24)])
def test_queue_threads_match_oracle(ctx, max_batch, delay_us, threads):
    text = _demo()
    _load(ctx, [cedargpu.MemoryStore("demo.cedar", text)], 101)
    sars = synth.random_sars(1200, seed=23, pop=synth.Population(seed=23, n_users=800, n_groups=80))
    sars.append(synth.make_sar("system:authorizer:cedar-authorizer", "", [], "get", group="rbac.authorization.k8s.io",
                               resource="roles"))
    otiers = _oracle_tiers(text)
    want = [km.authorize(otiers, km.attributes_from_sar(s)) for s in sars]
    got = [None] * len(sars)
    q = cedargpu.Queue(ctx, max_batch=max_batch, max_delay_us=delay_us)
    errors = []

    def work(t):
        try:
            for i in range(t, len(sars), threads):
                got[i] = q.authorize(sars[i])
        except Exception as e:  # surfaced below
            errors.append(e)

    ws = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for w in ws:
        w.start()
    for w in ws:
        w.join(120)
    st = q.stats()
    q.close()
    assert not errors, errors[0]
    for s, g, w in zip(sars, got, want):
        assert g == w, s
    assert st["requests"] + st["fast"] == len(sars)
    assert st["max_batch"] <= max_batch
    assert st["batches"] >= (st["requests"] + max_batch - 1) // max_batch


def test_queue_is_authorized_json(ctx):
    text = _demo()
    stores = [cedargpu.MemoryStore("demo.cedar", text)]
    _load(ctx, stores, 102)
    sars = synth.random_sars(300, seed=29, pop=synth.Population(seed=29, n_users=300, n_groups=40))
    items = []
    for s in sars:
        a = km.attributes_from_sar(s)
        em, r = km.record_to_cedar_resource(a)
        items.append((co.entities_to_json(em), co.request_to_json(r)))
    otiers = _oracle_tiers(text)
    q = cedargpu.Queue(ctx, max_batch=50)
    got = [None] * len(items)

    def work(t):
        for i in range(t, len(items), 8):
            got[i] = q.is_authorized(*items[i])

    ws = [threading.Thread(target=work, args=(t,)) for t in range(8)]
    for w in ws:
        w.start()
    for w in ws:
        w.join(120)
    q.close()
    for (ents, req), (ok, diag) in zip(items, got):
        want_ok, want_diag, _ = co.tiered_is_authorized(otiers, co.entities_from_json(ents), co.request_from_json(req))
        assert ok == want_ok and diag == want_diag.to_go_json(), req


def test_queue_loadgen_counts_match_batch(ctx):
    """The native load generator's decision counts equal one plain batch over the same SARs."""
    pop = synth.Population(seed=5, n_users=2000, n_groups=60)
    _load(ctx, [cedargpu.MemoryStore("c3.cedar", synth.abac_policies(1500, seed=5, pop=pop))], 103)
    sars = synth.random_sars(2000, seed=41, pop=pop)
    b = ctx.batch()
    b.add_sar_json(synth.sars_json(sars))
    b.submit()
    b.wait()
    want = [0, 0, 0]
    for i in range(len(b)):
        want[b.authz(i)[0]] += 1
    b.close()
    q = cedargpu.Queue(ctx, max_batch=512)
    r = q.loadgen([json.dumps(s) for s in sars], threads=32, total=2 * len(sars))
    st = q.stats()
    m = q.metrics()
    q.close()
    assert [r["deny"], r["allow"], r["no_opinion"]] == [2 * w for w in want]
    assert st["batches"] >= 8 and st["max_batch"] <= 512
    # metrics (cg_queue_metrics_get): request_total by decision = the loadgen's counts, every call in
    # exactly one latency bucket, batches in the size histogram, the active epoch
    assert [m["requests"][k] for k in ("deny", "allow", "no_opinion")] == [2 * w for w in want]
    assert m["requests"]["error"] == 0
    for k in ("deny", "allow", "no_opinion"):
        assert sum(m["latency"][k]) == m["requests"][k]
        assert m["latency_sum_ns"][k] > 0 or m["requests"][k] == 0
    assert sum(m["batch_size"]) == m["batches"] == st["batches"]
    assert sum(m["batch_size"][10:]) == 0  # max_batch 512 = 2^9
    assert sum(m["batch_latency"]) == m["batches"] and m["batch_latency_sum_ns"] > 0
    assert m["active_epoch"] == 103 and m["activations"] >= 1


@pytest.mark.parametrize("per_call", [1, 3, 16])
def test_queue_authorize_many_matches_oracle(ctx, per_call):
    """cg_queue_authorize_sar_n (a host-side batcher's entry point): groups of SARs per call from
    several threads, fast paths mixed in, every (decision, reason) equal to the oracle's Authorize;
    the native load generator's batched mode counts the same decisions as per-request calls."""
    text = _demo()
    _load(ctx, [cedargpu.MemoryStore("demo.cedar", text)], 105)
    sars = synth.random_sars(600, seed=31, pop=synth.Population(seed=31, n_users=500, n_groups=60))
    sars.insert(7, synth.make_sar("system:authorizer:cedar-authorizer", "", [], "get", group="rbac.authorization.k8s.io",
                                  resource="roles"))
    otiers = _oracle_tiers(text)
    want = [km.authorize(otiers, km.attributes_from_sar(s)) for s in sars]
    got = [None] * len(sars)
    q = cedargpu.Queue(ctx, max_batch=64)
    errors = []
    groups = [list(range(i, min(i + per_call, len(sars)))) for i in range(0, len(sars), per_call)]

    def work(t):
        try:
            for g in groups[t::6]:
                for i, r in zip(g, q.authorize_many([sars[i] for i in g])):
                    got[i] = r
        except Exception as e:  # surfaced below
            errors.append(e)

    ws = [threading.Thread(target=work, args=(t,)) for t in range(6)]
    for w in ws:
        w.start()
    for w in ws:
        w.join(120)
    assert not errors, errors[0]
    for s, g, w in zip(sars, got, want):
        assert g == w, s
    one = q.loadgen([json.dumps(s) for s in sars], threads=8, total=len(sars))
    many = q.loadgen([json.dumps(s) for s in sars], threads=8, total=len(sars), per_call=per_call)
    q.close()
    assert [many[k] for k in ("deny", "allow", "no_opinion")] == [one[k] for k in ("deny", "allow", "no_opinion")]
    assert [one[k] for k in ("deny", "allow", "no_opinion")] == [sum(1 for d, _ in want if d == k) for k in (0, 1, 2)]


def test_queue_errors(ctx):
    q = cedargpu.Queue(ctx, max_batch=16)
    with pytest.raises(cedargpu.CedarGPUError):
        q.authorize("{not json")
    # a bad request does not poison the batch it would have joined
    _load(ctx, [cedargpu.MemoryStore("demo.cedar", _demo())], 104)
    dec, _ = q.authorize(synth.make_sar("alice", "", ["viewers"], "get", resource="pods", ns="default"))
    assert dec in (0, 1, 2)
    q.close()


def test_multi_context_queue_peer_reload_matches_oracle(ctx):
    """cg_queue_create_multi over two contexts (here both on GPU 0; one per GPU in production):
    the image reaches the second context by cg_image_load_peer (device-to-device copy, host tables
    shared), batches are dealt to both, and a reload (load + activate on the first context, peer
    load on the second) while callers run changes no result against the oracle of the epoch each
    request was encoded against."""
    text = _demo()
    extra = '\nforbid (principal, action == k8s::Action::"get", resource) when { resource has namespace && ' \
            'resource.namespace == "kube-system" };'
    c2 = cedargpu.Context(0)
    try:
        _load(ctx, [cedargpu.MemoryStore("demo.cedar", text)], 301)
        c2.load_peer(ctx, 301)
        q = cedargpu.Queue([ctx, c2], max_batch=48, max_delay_us=100)
        pop = synth.Population(seed=29, n_users=600, n_groups=60)
        sars = synth.random_sars(3000, seed=29, pop=pop)
        for k in range(0, len(sars), 5):
            ra = sars[k]["spec"].get("resourceAttributes")
            if ra is not None:
                ra["namespace"], ra["verb"] = "kube-system", "get"
        want1 = [km.authorize(_oracle_tiers(text), km.attributes_from_sar(s)) for s in sars]
        want2 = [km.authorize(_oracle_tiers(text + extra), km.attributes_from_sar(s)) for s in sars]
        assert want1 != want2
        got = [None] * len(sars)
        errors = []
        half, reloaded = threading.Barrier(17), threading.Barrier(17)

        def work(t):
            try:
                for n, i in enumerate(range(t, len(sars), 16)):
                    if n == 20:
                        half.wait(60)      # every caller has had 20 answers on epoch 301
                        reloaded.wait(60)  # and continues once epoch 302 is active
                    got[i] = q.authorize(sars[i])
            except Exception as e:  # surfaced below
                errors.append(e)

        ws = [threading.Thread(target=work, args=(t,)) for t in range(16)]
        for w in ws:
            w.start()
        half.wait(60)
        _load(ctx, [cedargpu.MemoryStore("demo.cedar", text + extra)], 302)
        c2.load_peer(ctx, 302)
        reloaded.wait(60)
        for w in ws:
            w.join(120)
        per_gpu = q.gpu_stats()
        q.close()
        assert not errors, errors[0]
        for s, g, w1, w2 in zip(sars, got, want1, want2):
            assert g in (w1, w2), s  # either epoch, depending on when the request was encoded
        # requests issued after the reload see the new epoch
        late = [i for t in range(16) for n, i in enumerate(range(t, len(sars), 16)) if n >= 20]
        assert all(got[i] == want2[i] for i in late)
        assert all(p["batches"] > 0 for p in per_gpu), per_gpu
    finally:
        c2.close()
