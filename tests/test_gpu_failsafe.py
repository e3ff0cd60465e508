"""§8(b) fail-safe contract through the C-ABI: deadlines (CG_E_TIMEOUT) and device errors
(CG_E_DEVICE) on the batch and queue paths, driven by the gameday fault injector
(cg_ctx_inject_fault). Authorization fails safe to NoOpinion (authorizer.go:80-84; the apiserver's
failurePolicy NoOpinion, mount/authorization-config.yaml:11,16), admission to allow
(cmd/cedar-webhook/main.go:116 allowOnError; manifests/admission-webhook.yaml:11 Ignore)."""
import json
import os
import time

import pytest

import cedar_oracle as co
import k8s_model as km
from conftest import GOLDEN

import cedargpu
from cedargpu import synth

pytestmark = pytest.mark.gpu

CORPUS = json.load(open(os.path.join(GOLDEN, "reference_corpus.json")))
DEMO_AUTHZ = "\n".join(v for k, v in sorted(CORPUS["demo"].items()) if k.startswith("authorization"))
DEMO_ADM = "\n".join(v for k, v in sorted(CORPUS["demo"].items()) if k.startswith("admission"))


@pytest.fixture()
def ctx():
    assert cedargpu.device_count() >= 1, "GPU tests need a GPU"
    c = cedargpu.Context(0)
    yield c
    c.inject_fault(cedargpu.FAULT_NONE)
    c.close()


def _sars():
    sars = synth.random_sars(200, seed=71, pop=synth.Population(seed=71, n_users=300, n_groups=30))
    sars.append(synth.make_sar("system:authorizer:cedar-authorizer", "", [], "get", group="rbac.authorization.k8s.io",
                               resource="roles"))  # self-allow fast path (authorizer.go:44-49)
    sars.append(synth.make_sar("system:kube-scheduler", "", [], "get", resource="pods"))  # system: bypass
    sars.append(synth.make_sar("test-user", "1", ["viewers"], "get", ns="default", resource="pods", name="p"))
    return sars


def _oracle(text, sars):
    tiers = [co.PolicySet.from_bytes("demo.cedar", text)]
    return [km.authorize(tiers, km.attributes_from_sar(s)) for s in sars]


def test_device_error_authz_answers_noopinion(ctx):
    authz = cedargpu.Authorizer([cedargpu.MemoryStore("demo.cedar", DEMO_AUTHZ)], ctx=ctx)
    sars = _sars()
    want = _oracle(DEMO_AUTHZ, sars)
    ctx.inject_fault(cedargpu.FAULT_DEVICE_ERROR, 1)
    got = authz.authorize_batch(sars)
    for s, g, w in zip(sars, got, want):
        name = s["spec"]["user"]
        fast = name.startswith("system:") and not name.startswith(("system:serviceaccount:", "system:node:"))
        fast = fast or (name == "system:authorizer:cedar-authorizer")
        assert g == (w if fast else (cedargpu.Authorizer.NO_OPINION, "")), s
    assert authz.authorize_batch(sars) == want  # the injected error was consumed


def test_device_error_admission_allows(ctx):
    handler = cedargpu.AdmissionHandler([cedargpu.MemoryStore("adm.cedar", DEMO_ADM), cedargpu.ALLOW_ALL_ADMISSION],
                                        ctx=ctx)
    reviews = synth.admission_reviews(64, seed=9)
    normal = handler.handle_batch(reviews)
    assert any(not ok for ok, _, _ in normal), "the workload must hold denials for the test to mean anything"
    ctx.inject_fault(cedargpu.FAULT_DEVICE_ERROR, 1)
    assert handler.handle_batch(reviews) == [(True, 200, "")] * len(reviews)
    assert handler.handle_batch(reviews) == normal


def test_batch_wait_deadline_then_completes(ctx):
    tiers = cedargpu.TieredPolicyStores([cedargpu.MemoryStore("demo.cedar", DEMO_AUTHZ)], ctx=ctx)
    assert tiers.ready()
    sars = _sars()
    ctx.inject_fault(cedargpu.FAULT_STALL, 300_000)
    b = ctx.batch()
    b.add_sar_json(json.dumps(sars))
    b.submit()
    t0 = time.perf_counter()
    with pytest.raises(cedargpu.DeadlineError):
        b.wait(timeout=0.02)
    assert time.perf_counter() - t0 < 0.2
    b.wait()  # the batch stayed in flight and completes
    assert [b.authz(i) for i in range(len(b))] == _oracle(DEMO_AUTHZ, sars)
    b.close()
    # a timed-out batch destroyed while in flight: destroy returns at once (its blocks go back to
    # the pool once the stream has passed them, dev_batch_retire)
    b = ctx.batch()
    b.add_sar_json(json.dumps(sars[:10]))
    b.submit()
    with pytest.raises(cedargpu.DeadlineError):
        b.wait(timeout=0.01)
    t0 = time.perf_counter()
    b.close()
    assert time.perf_counter() - t0 < 0.1
    ctx.inject_fault(cedargpu.FAULT_NONE)
    b = ctx.batch()
    b.add_sar_json(json.dumps(sars))
    b.submit()
    b.wait(timeout=5.0)
    assert [b.authz(i) for i in range(len(b))] == _oracle(DEMO_AUTHZ, sars)
    b.close()


def test_queue_deadline_and_failsafe(ctx):
    cedargpu.TieredPolicyStores([cedargpu.MemoryStore("demo.cedar", DEMO_AUTHZ)], ctx=ctx)
    sars = _sars()
    want = _oracle(DEMO_AUTHZ, sars)
    q = cedargpu.Queue(ctx, max_batch=256, max_delay_us=0)
    try:
        ctx.inject_fault(cedargpu.FAULT_STALL, 400_000)
        t0 = time.perf_counter()
        with pytest.raises(cedargpu.DeadlineError):
            q.authorize(sars[-1], timeout=0.05)
        assert time.perf_counter() - t0 < 0.3
        assert q.authorize_failsafe(sars[-1], timeout=0.05) == (cedargpu.Authorizer.NO_OPINION, "")
        em, r = km.record_to_cedar_resource(km.attributes_from_sar(sars[-1]))
        with pytest.raises(cedargpu.DeadlineError):
            q.is_authorized(co.entities_to_json(em), co.request_to_json(r), timeout=0.05)
        # fast paths answer on the caller's thread, inside any deadline
        assert q.authorize(sars[-3], timeout=0.0) == want[-3]
        # two batches now hold the stalled device (one running, one queued); requests behind them
        # wait in the backlog, time out there and are dropped unevaluated (Ticket T_ABANDONED)
        slow = [s for s in sars if not s["spec"]["user"].startswith("system:")][:6]
        for s in slow:
            with pytest.raises(cedargpu.DeadlineError):
                q.authorize(s, timeout=0.02)
        ctx.inject_fault(cedargpu.FAULT_NONE)
        time.sleep(1.5)  # the stalled batches drain
        assert [q.authorize(s, timeout=5.0) for s in sars] == want
        assert q.stats()["dropped"] >= 1
        ctx.inject_fault(cedargpu.FAULT_DEVICE_ERROR, 1)
        got = q.authorize_failsafe(sars[-1], timeout=5.0)
        assert got == (cedargpu.Authorizer.NO_OPINION, "")
        assert q.authorize(sars[-1], timeout=5.0) == want[-1]
    finally:
        ctx.inject_fault(cedargpu.FAULT_NONE)
        q.close()


def test_authorizer_deadline_under_stall(ctx):
    """Authorizer(timeout=...) answers NoOpinion within its deadline while the device stalls, and
    AdmissionHandler allows: the timed-out batch is retired without waiting for the stream (ADVICE
    r02: close() used to drain it). Blocks of the retired batches return to the pool afterwards."""
    authz = cedargpu.Authorizer([cedargpu.MemoryStore("demo.cedar", DEMO_AUTHZ)], ctx=ctx, timeout=0.05)
    sars = _sars()
    want = _oracle(DEMO_AUTHZ, sars)
    assert authz.authorize_batch(sars) == want
    ctx.inject_fault(cedargpu.FAULT_STALL, 400_000)
    t0 = time.perf_counter()
    got = authz.authorize_batch(sars)
    assert time.perf_counter() - t0 < 0.2
    for s, g, w in zip(sars, got, want):
        name = s["spec"]["user"]
        fast = name.startswith("system:") and not name.startswith(("system:serviceaccount:", "system:node:"))
        assert g == (w if fast else (cedargpu.Authorizer.NO_OPINION, "")), s
    ctx.inject_fault(cedargpu.FAULT_NONE)
    time.sleep(0.6)  # the stalled batch drains; its blocks are reaped by the next batch
    authz.timeout = 5.0
    assert authz.authorize_batch(sars) == want
    # admission on its own context (a handler's tiers activate their image on the context they use)
    actx = cedargpu.Context(0)
    try:
        handler = cedargpu.AdmissionHandler([cedargpu.MemoryStore("adm.cedar", DEMO_ADM), cedargpu.ALLOW_ALL_ADMISSION],
                                            ctx=actx, timeout=0.05)
        reviews = synth.admission_reviews(16, seed=9)
        normal = handler.handle_batch(reviews)
        actx.inject_fault(cedargpu.FAULT_STALL, 400_000)
        t0 = time.perf_counter()
        assert handler.handle_batch(reviews) == [(True, 200, "")] * len(reviews)
        assert time.perf_counter() - t0 < 0.2
        actx.inject_fault(cedargpu.FAULT_NONE)
        time.sleep(0.6)
        handler.timeout = 5.0
        assert handler.handle_batch(reviews) == normal
    finally:
        actx.inject_fault(cedargpu.FAULT_NONE)
        actx.close()


def test_queue_close_bounded_on_a_stalled_device(ctx):
    """cg_queue_destroy over a device that does not finish: a submitter already waiting
    on its in-flight batch polls the download in slices, so the close returns after the grace
    (CEDARGPU_QUEUE_STOP_GRACE_MS) and the batch's caller gets an error instead of hanging."""
    import threading
    cedargpu.TieredPolicyStores([cedargpu.MemoryStore("demo.cedar", DEMO_AUTHZ)], ctx=ctx)
    sars = _sars()
    q = cedargpu.Queue(ctx, max_batch=256, max_delay_us=0)
    got = []
    old = os.environ.get("CEDARGPU_QUEUE_STOP_GRACE_MS")
    try:
        assert q.authorize(sars[-1], timeout=5.0)  # warm
        ctx.inject_fault(cedargpu.FAULT_STALL, 1_500_000)
        th = threading.Thread(target=lambda: got.append(q.authorize_failsafe(sars[-1])))
        th.start()
        time.sleep(0.2)  # the submitter is now waiting on the stalled batch
        os.environ["CEDARGPU_QUEUE_STOP_GRACE_MS"] = "200"
        t0 = time.perf_counter()
        q.close()
        dt = time.perf_counter() - t0
        th.join(timeout=5.0)
        assert not th.is_alive()
        assert dt < 0.8, dt                                   # the grace, not the 1.5 s stall
        assert got == [(cedargpu.Authorizer.NO_OPINION, "")]  # the caller failed safe
    finally:
        if old is None:
            os.environ.pop("CEDARGPU_QUEUE_STOP_GRACE_MS", None)
        else:
            os.environ["CEDARGPU_QUEUE_STOP_GRACE_MS"] = old
        ctx.inject_fault(cedargpu.FAULT_NONE)
        q.close()
        time.sleep(1.6)  # the stalled batch drains before the context goes


def test_bad_key_entity_indices_fail_the_batch(ctx):
    """a key-entity index outside the image's (a batch encoded for another
    image) used to read as "bit not set" in the scan's bitset pass, dropping the key without a
    signal. The scan now counts such requests (and enumerates their keys exactly), and the batch
    fails with CG_E_DEVICE, so the webhook answers fail safe instead of trusting the batch."""
    pop = synth.Population(seed=17, n_users=400, n_groups=60, dag_depth=5)
    text = synth.abac_policies(400, seed=17, pop=pop)
    ents = pop.static_entities()
    tiers = cedargpu.TieredPolicyStores([cedargpu.MemoryStore("c3.cedar", text)], ctx=ctx, entities=ents)
    assert tiers.ready()
    assert cedargpu.index_stats(tiers.image)["contexts"] > 0, "the workload must use the scope bitsets"
    sars = synth.random_sars(2600, seed=18, pop=pop)  # past dev_small_n(): the scan's bitset pass runs
    payload = json.dumps(sars)
    b = ctx.batch()
    b.add_sar_json(payload)
    b.submit()
    b.wait()
    normal = [b.authz(i) for i in range(len(b))]
    b.close()
    ctx.inject_fault(cedargpu.FAULT_BAD_KIDX, 1)
    b = ctx.batch()
    try:
        b.add_sar_json(payload)
        b.submit()
        with pytest.raises(cedargpu.DeviceError):
            b.wait()
    finally:
        b.close()
    b = ctx.batch()  # the fault was consumed: the next batch decides as before
    b.add_sar_json(payload)
    b.submit()
    b.wait()
    assert [b.authz(i) for i in range(len(b))] == normal
    b.close()


def test_closed_in_flight_batch_keeps_its_pinned_arrays(ctx):
    """A small batch whose heap went to the device straight from a pinned block (engine.h PinVec,
    dev_batch_upload's direct copy), closed while in flight: its arrays go with the retired batch
    until the stream drains (cg_batch's destructor, DevBatch::keep), and the batches after it, which
    take the same pinned blocks again, decide as before."""
    pop = synth.Population(seed=7, dag_depth=6)
    img = cedargpu.build_image([cedargpu.MemoryStore("c3.cedar", synth.abac_policies(2000, seed=31, pop=pop))], epoch=1,
                               entities=pop.static_entities())
    ctx.load(img, 1)
    payload = synth.sars_json(synth.random_sars(2048, seed=5, pop=pop)).encode()
    b = ctx.batch()
    b.add_sar_json(payload)
    assert b.bytes()[2] >= 64 << 10  # a heap the upload copies straight from its pinned block
    b.submit()
    b.wait()
    want = [b.authz(i) for i in range(len(b))]
    b.close()
    ctx.inject_fault(cedargpu.FAULT_STALL, 200_000)
    kept0 = cedargpu.pinned_stats()["kept_batches"]
    for _ in range(3):
        b = ctx.batch()
        b.add_sar_json(payload)
        b.submit()
        b.close()  # in flight: retired, never waited
    # the mechanism itself: each closed in-flight batch handed its pinned arrays to the retired batch
    # (a batch whose DevBatch::direct never reached cg_batch would return them to the pool at once)
    assert cedargpu.pinned_stats()["kept_batches"] - kept0 == 3
    ctx.inject_fault(cedargpu.FAULT_NONE)
    for _ in range(3):
        b = ctx.batch()
        b.add_sar_json(payload)
        b.submit()
        b.wait(timeout=5.0)
        assert [b.authz(i) for i in range(len(b))] == want
        b.close()
