"""Benchmark: authz decisions/sec at 10k policies on MI355X (BASELINE.json metric).

One step = one evaluation pass of the GPU hot path (TieredPolicyStores.IsAuthorized for every
request of a device-resident batch) over a batch of synthetic SubjectAccessReviews.
Workload (config C3 of BASELINE.json, single-GPU shard): 10,000 ABAC policies keyed on
k8s::Group membership with when-clauses over namespace / apiGroup / resource / name (like) /
labelSelector (containsAny), x `--batch` SARs per GPU, Zipf users with 1+Binomial(7,0.35) groups.
Multi-GPU: one process per GPU (torchrun), the compiled image is replicated, requests are sharded
(weak scaling: fixed batch per GPU), no collective on the decision path.

Prints ONE JSON line (rank 0) with roofline and cpu_baseline objects; see DESIGN.md §Measurement.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "cedar-access-control-for-k8s_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def algorithmic_bytes(sars, n_reasons, has_like):
    """B_dec = 64 + 4G + 8S + A + 16 + 4 n_reasons per decision."""
    total = 0
    for s, nr in zip(sars, n_reasons):
        sp = s["spec"]
        g = len(sp.get("groups") or [])
        ra = sp.get("resourceAttributes") or {}
        S = len((ra.get("labelSelector") or {}).get("requirements") or []) + len(sp.get("extra") or {})
        A = 0
        if has_like:
            A = len(ra.get("name", "")) if ra else len((sp.get("nonResourceAttributes") or {}).get("path", ""))
        total += 64 + 4 * g + 8 * S + A + 16 + 4 * nr
    return total


def oracle_items(sars):
    """(EntityMap, Request) JSON items of the SARs that reach evaluation (the fast paths of
    authorizer.go:38-57 never do), built by the oracle's k8s model (test infrastructure)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cedar_oracle as co
    import k8s_model as km
    items, idx = [], []
    for i, s in enumerate(sars):
        a = km.attributes_from_sar(s)
        n = a.user.name
        if n.startswith("system:") and not (n.startswith("system:serviceaccount:") or n.startswith("system:node:")):
            continue
        em, req = km.record_to_cedar_resource(a)
        items.append((co.entities_to_json(em), co.request_to_json(req)))
        idx.append(i)
    return items, idx


def host_cpus():
    """The host cores this process may run on: the affinity mask, bounded by the cgroup CPU
    quota (cgroup v2 cpu.max or v1 cfs_quota/period) when one is set; plus the CPU model."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = float(q) / float(p)
    except (OSError, ValueError):
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = q / p
        except (OSError, ValueError):
            pass
    usable = affinity if quota is None else max(1, min(affinity, int(quota + 0.5)))
    # the GPU pool declares each box's host-core share in OMP_NUM_THREADS (16 per GPU); nproc there
    # counts the whole machine, so the share bounds the worker count too
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        usable = min(usable, int(share))
    model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return usable, {"affinity_cpus": affinity, "cgroup_quota_cpus": quota, "os_cpu_count": os.cpu_count(),
                    "omp_num_threads": share, "cpu_model": model}


def cpu_baseline(policies_text, items, seconds, threads, cpu_info, entities=None):
    """C++ oracle (`port`: oracle/cedar_ref.cpp, the restatement of cedar-go's per-request linear
    scan with a tree-walking evaluator) on `threads` host threads (one per usable core, SURVEY
    §8(d) GOMAXPROCS = nproc) over pre-built EntityMaps. Runs before any GPU initialisation."""
    from cedar_ref import RefPolicySet, items_json
    ref = RefPolicySet()
    if entities:
        ref.set_entities(json.dumps(entities))
    ref.add_tier()
    ref.add_document("c3.cedar", policies_text)
    ref.load_items(items_json(items))
    n, wall = ref.bench(threads, seconds)
    ref.close()
    return {"value": n / wall, "unit": "decisions/s", "cores": threads, "kind": "port", **cpu_info,
            "sample": f"{n} decisions in {wall:.1f} s: {len(items)} pre-built (EntityMap, Request) items from the "
                      f"benchmark's SubjectAccessReviews x {policies_text.count(';')} policies through "
                      f"oracle/cedar_ref.cpp (C++ restatement of cedar-go IsAuthorized, linear scan; not cedar-go), "
                      f"{threads} threads = the usable host cores (affinity {cpu_info['affinity_cpus']}, cgroup "
                      f"quota {cpu_info['cgroup_quota_cpus']}, declared share OMP_NUM_THREADS="
                      f"{cpu_info['omp_num_threads']}) on {cpu_info['cpu_model'] or 'unknown CPU'}"}


def parity_sample(policies_text, items, idx, gpu_batch, threads, entities=None):
    """GPU authorizer answers vs the C++ oracle on a sample of the timed batch (decision + exact
    reason string, authorizer.go:75-84 mapping; the static group hierarchy merged into every
    EntityMap)."""
    from cedar_ref import RefPolicySet, items_json
    ref = RefPolicySet()
    if entities:
        ref.set_entities(json.dumps(entities))
    ref.add_tier()
    ref.add_document("c3.cedar", policies_text)
    ref.load_items(items_json(items))
    want = ref.evaluate(threads)
    ref.close()
    bad = 0
    for (ok, _, diag, _), i in zip(want, idx):
        wd = 1 if ok else (0 if diag.startswith('{"reasons"') else 2)
        wr = diag if wd != 2 else ""
        if gpu_batch.authz(i) != (wd, wr):
            bad += 1
    return {"requests": len(items), "mismatches": bad, "oracle": "oracle/cedar_ref.cpp"}


def secondary_configs(ctx, n_req, threads, sample=512):
    """The other single-GPU BASELINE configs, run after the timed region (not part of `value`):
    C2 = 1k RBAC-converted policies x SubjectAccessReviews, C4 = 1k admission forbids plus the
    static allow-all tier x AdmissionReviews on ConfigMaps / Secrets. Per config: device
    decisions/s (HIP events over 5 launches of the resident batch), host encode rate (the C++ SAR
    / admission models), and a parity sample against the C++ oracle."""
    import cedargpu
    from cedargpu import synth
    from cedar_ref import RefPolicySet, items_json
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cedar_oracle as co
    import k8s_model as km
    out = {}

    def run(name, stores, payload, add, result, want_of, items, idx, what):
        image = cedargpu.build_image(stores, epoch=100 + len(out))
        ctx.load(image, 100 + len(out))
        b = ctx.batch()
        t0 = time.perf_counter()
        add(b, payload)
        enc_s = time.perf_counter() - t0
        b.submit()
        b.wait()
        n_req_b = len(b)
        ref = RefPolicySet.from_stores(stores)
        ref.load_items(items_json(items))
        want = ref.evaluate(threads)
        ref.close()
        bad = sum(1 for w, i in zip(want, idx) if result(b, i) != want_of(w))
        b.close()
        # the same payload again on the warm buffer pool (steady state: each batch's result
        # capacities sized by the one before on the image): submit -> results, with the H2D copy,
        # the first pass, the on-device follow-ups, any host re-run and the D2H copy; best of 3.
        # The device step of the last one is timed (HIP events, 5 repeats).
        full_ms = None
        for k in range(3):
            b2 = ctx.batch()
            add(b2, payload)
            t0 = time.perf_counter()
            b2.submit()
            b2.wait()
            t = (time.perf_counter() - t0) * 1e3
            full_ms = t if full_ms is None else min(full_ms, t)
            n_big, fus = b2.reruns(), b2.followups()
            if k == 2:
                ms = b2.time(5) / 5  # complete step: first pass + gather + on-device follow-ups
            b2.close()
        out[name] = {"what": what, "requests": n_req_b, "kernel_ms": ms, "kernel_decisions_per_s": n_req_b / (ms * 1e-3),
                     "submit_to_results_ms": full_ms, "decisions_per_s": n_req_b / (full_ms * 1e-3),
                     "rerun_requests": n_big, "device_followup_requests": fus,
                     "host_encode_per_s": n_req_b / enc_s,
                     "parity_sample": {"requests": len(items), "mismatches": bad, "oracle": "oracle/cedar_ref.cpp"}}

    pop = synth.Population(seed=21)
    sars = synth.random_sars(n_req, seed=2000, pop=pop)
    items, idx = oracle_items(sars[:sample])

    def authz_want(w):
        ok, _, diag, _ = w
        d = 1 if ok else (0 if diag.startswith('{"reasons"') else 2)
        return (d, diag if d != 2 else "")

    run("c2_rbac_1k", [cedargpu.MemoryStore("rbac.cedar", synth.rbac_policies(1000, seed=21, pop=pop))],
        synth.sars_json(sars), lambda b, p: b.add_sar_json(p), lambda b, i: b.authz(i), authz_want, items, idx,
        "1k RBAC-converted policies x synthetic SubjectAccessReviews (authorizer.Decision + reason)")

    reviews = synth.admission_reviews(n_req, seed=4000)
    items, idx = [], []
    for i, r in enumerate(reviews[:sample]):
        em, req = km.admission_to_cedar(km.admission_request_from_review(r))
        items.append((co.entities_to_json(em), co.request_to_json(req)))
        idx.append(i)

    def admit_want(w):
        ok, _, _, reasons = w
        return (ok, 200, reasons if not ok and reasons not in ("", "[]", "null") else "")

    # C5: 100k policies over 1,000 tenants (one CRD document each): compile, incremental rebuild
    # after one tenant changes, device load + activate, evaluation
    tpop = synth.Population(seed=7, n_namespaces=1000)
    docs = synth.multitenant_policies(100_000, seed=51, pop=tpop)
    comp = cedargpu.Compiler()
    t0 = time.perf_counter()
    comp.build([cedargpu.CRDStore(docs)], epoch=200)
    t_full = time.perf_counter() - t0
    docs[500] = (docs[500][0], docs[500][1], docs[500][2].replace("permit", "forbid", 1))
    t0 = time.perf_counter()
    img5 = comp.build([cedargpu.CRDStore(docs)], epoch=201)
    t_inc = time.perf_counter() - t0
    comp.close()
    t0 = time.perf_counter()
    ctx.load(img5, 201)
    t_load = time.perf_counter() - t0
    tsars = synth.random_sars(n_req, seed=5000, pop=tpop)
    items5, idx5 = oracle_items(tsars[:sample // 2])
    run("c5_multitenant_100k", [cedargpu.CRDStore(docs)], synth.sars_json(tsars), lambda b, p: b.add_sar_json(p),
        lambda b, i: b.authz(i), authz_want, items5, idx5,
        "100k namespace-scoped policies over 1,000 tenant CRD documents x synthetic SubjectAccessReviews")
    out["c5_multitenant_100k"].update({"compile_s": t_full, "incremental_rebuild_s": t_inc, "image_bytes": len(img5),
                                       "load_activate_s": t_load})

    run("c4_admission_1k", [cedargpu.MemoryStore("adm.cedar", synth.admission_policies(1000, seed=3)),
                            cedargpu.ALLOW_ALL_ADMISSION],
        json.dumps(reviews, separators=(",", ":")), lambda b, p: b.add_admission_json(p), lambda b, i: b.admit(i),
        admit_want, items, idx,
        "1k admission forbids + allow-all tier x synthetic AdmissionReviews on ConfigMaps / Secrets "
        "(allowed + message)")
    return out


def hot_reload(ctx, policies, rank, world, device, dist_on, timeout_s=180.0, entities=None, c5=True):
    """Policy hot reload after the timed region: rank 0 compiles epoch 2 (the policies plus one
    forbid), one RCCL broadcast ships it to every GPU, each rank activates it and checks a request
    the new forbid decides; then C5's incremental rebuild + broadcast (`c5`). Runs in a daemon thread
    with a deadline so that a stuck collective cannot hang the benchmark; reports the
    broadcast+load+activate times."""
    import threading

    import cedargpu
    from cedargpu import dist as cdist

    out = {}

    def run():
        try:
            uid = cdist.exchange_unique_id(rank) if dist_on else cdist.unique_id()
            comm = cdist.Comm(device, world, rank, uid)
            extra = 'forbid (principal, action == k8s::Action::"reload-check", resource);'
            image = (cedargpu.build_image([cedargpu.MemoryStore("c3.cedar", policies + "\n" + extra)], epoch=2,
                                          entities=entities) if rank == 0 else None)
            t0 = time.perf_counter()
            n = comm.broadcast_image(ctx, image, 2)
            dt = time.perf_counter() - t0
            b = ctx.batch()
            b.add([], {"principal": {"type": "k8s::User", "id": "u"}, "action": {"type": "k8s::Action", "id": "reload-check"},
                       "resource": {"type": "k8s::Resource", "id": "/api/v1/pods"}, "context": {}})
            b.submit()
            b.wait()
            ok = b.decision(0)[0] is False and len(b.reasons(0)[0]) == 1
            b.close()
            out.update({"via": "rccl broadcast", "image_bytes": n, "ms": dt * 1e3, "ranks": world, "epoch": 2,
                        "new_policy_applied": ok})
            if c5:
                # C5's reload path end to end: one tenant CRD edited (crd.go:62 update event), the
                # incremental rebuild on rank 0 (only that document parsed and lowered), the RCCL
                # broadcast of the 100k-policy image into every rank's image storage, activation
                from cedargpu import synth
                comp, docs, img0 = None, None, None
                if rank == 0:
                    tpop = synth.Population(seed=7, n_namespaces=1000)
                    docs = synth.multitenant_policies(100_000, seed=51, pop=tpop)
                    comp = cedargpu.Compiler()
                    img0 = comp.build([cedargpu.CRDStore(docs)], epoch=300)  # the epoch before the event (not timed)
                    docs[500] = (docs[500][0], docs[500][1], docs[500][2].replace("permit", "forbid", 1))
                comm.broadcast_image(ctx, img0, 300, activate=False)  # every rank holds the base (not timed)
                t0 = time.perf_counter()
                img5 = comp.build([cedargpu.CRDStore(docs)], epoch=301) if rank == 0 else None
                t1 = time.perf_counter()
                n5 = comm.broadcast_image(ctx, img5, 301)
                t2 = time.perf_counter()
                # the same event shipped as a delta image against epoch 300 (§8 f2): diff on rank 0,
                # broadcast of the delta, rebuilt on every GPU from its copy of epoch 300, activated
                d5 = cedargpu.image_delta(img0, img5) if rank == 0 else None
                t3 = time.perf_counter()
                nd = comm.broadcast_delta(ctx, 300, d5, 302)
                t4 = time.perf_counter()
                lb = comp.last_build() if rank == 0 else {}
                out["c5_100k"] = {"policies": 100_000, "image_bytes": n5, "incremental_compile_ms": (t1 - t0) * 1e3,
                                  "broadcast_load_activate_ms": (t2 - t1) * 1e3, "total_ms": (t2 - t0) * 1e3,
                                  "incremental": lb.get("incremental"), "lowered_policies": lb.get("lowered"),
                                  "what": "one tenant CRD edited -> incremental compile on rank 0 -> RCCL broadcast into "
                                          "every rank's image storage -> activate",
                                  "delta": {"bytes": nd, "frac_of_image": nd / max(n5, 1), "diff_ms": (t3 - t2) * 1e3,
                                            "broadcast_apply_activate_ms": (t4 - t3) * 1e3,
                                            "total_ms": (t1 - t0 + t4 - t2) * 1e3,
                                            "what": "the same event as a delta image against the held epoch: diff on "
                                                    "rank 0 -> RCCL broadcast of the delta -> rebuilt on each GPU from its "
                                                    "copy of the base (copy kernel), checksum, host tables -> activate"}}
                if comp:
                    comp.close()
            comm.close()
        except Exception as e:  # reported, not fatal: the decision path does not depend on it
            out["error"] = f"{type(e).__name__}: {e}"

    # RCCL prints its banner on stdout; keep stdout for the one JSON line (fd-level redirect)
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    try:
        th = threading.Thread(target=run, daemon=True)
        th.start()
        th.join(timeout_s)
    finally:
        sys.stdout.flush()
        os.dup2(saved, 1)
        os.close(saved)
    if th.is_alive():
        return {"error": f"timed out after {timeout_s:.0f} s"}
    return out


def serve(ctx, sars, threads, total, max_batch, sweep=(16, 32, 48, 64, 96, 192, 256, 384, 512),
          batched_sweep=(8, 16, 24, 32, 48, 64)):
    """End-to-end webhook path through the serving queue: `threads` native caller threads each
    issue blocking cg_queue_authorize_sar calls (SAR JSON in, Decision + reason out), which the
    queue batches onto the GPU. Host JSON parsing, SAR conversion and encoding are inside. Then the
    same at fewer and at more callers (`sweep`, up to 4x the box's 128 default): the highest rate
    whose p99 stays under 1 ms is `best_under_1ms` (the north star's latency bound), and
    `knee_threads` the first caller count whose p99 crosses 1 ms."""
    import cedargpu
    enc = [json.dumps(s, separators=(",", ":")) for s in sars]
    q = cedargpu.Queue(ctx, max_batch=max_batch, max_delay_us=0)
    q.loadgen(enc[:4096], threads, 8192)  # warm the pool's buffer classes
    q.close()

    def point(nt, n, per_call=1):
        q = cedargpu.Queue(ctx, max_batch=max_batch, max_delay_us=0)
        r = q.loadgen(enc, nt, n, per_call=per_call)
        st = q.stats()
        q.close()
        return {"decisions_per_s": n / r["seconds"], "requests": n, "threads": nt,
                "p50_us": r["p50_us"], "p99_us": r["p99_us"], "max_us": r["max_us"],
                "batches": st["batches"], "mean_batch": st["requests"] / max(1, st["batches"]),
                "max_batch": st["max_batch"], "device_busy_frac": st["device_ns"] / 1e9 / r["seconds"]}

    out = point(threads, total)
    curve = [point(nt, max(16384, total // 4)) for nt in sweep if nt != threads]
    allp = sorted(curve + [out], key=lambda p: p["threads"])
    ok = [p for p in allp if p["p99_us"] < 1000.0]
    out["curve"] = [{k: p[k] for k in ("threads", "decisions_per_s", "p50_us", "p99_us", "max_us", "mean_batch")} for p in allp]
    out["knee_threads"] = next((p["threads"] for p in allp if p["p99_us"] >= 1000.0), None)
    out["max_threads_tested"] = allp[-1]["threads"]
    out["best_under_1ms"] = max(ok, key=lambda p: p["decisions_per_s"])["decisions_per_s"] if ok else None
    out["best_under_1ms_threads"] = max(ok, key=lambda p: p["decisions_per_s"])["threads"] if ok else None
    out["what"] = ("cg_queue_authorize_sar per request from native threads (JSON parse, SAR conversion, columnar encode, "
                   "batched H2D + kernel + D2H, reason rendering)")
    # a host-side batcher's path (north_star's batching layer: one goroutine gathers the webhook
    # goroutines' requests and crosses into cgo once per group): cg_queue_authorize_sar_n calls of
    # `per_call` SARs from fewer caller threads; each request's latency is its call's
    per_call = 8
    bcurve = [point(nt, max(16384, total // 4), per_call) for nt in batched_sweep]
    bok = [p for p in bcurve if p["p99_us"] < 1000.0]
    best = max(bok, key=lambda p: p["decisions_per_s"]) if bok else None
    out["batched"] = {"per_call": per_call,
                      "curve": [{k: p[k] for k in ("threads", "decisions_per_s", "p50_us", "p99_us", "max_us", "mean_batch",
                                                    "device_busy_frac")} for p in bcurve],
                      "best_under_1ms": best["decisions_per_s"] if best else None,
                      "best_under_1ms_threads": best["threads"] if best else None,
                      "what": f"cg_queue_authorize_sar_n: {per_call} SAR bodies per call, per-request encode and rendering "
                              "on the calling thread, one wait per call"}
    return out


def cpu_barrier(dist, torch):
    """A barrier over gloo on a CPU tensor. With dist.barrier() between init_process_group and the
    contexts, cg_ctx_create found no usable GPU in both ranks of a 2-rank rehearsal (torch's
    accelerator query alone did not break it, profiles/r03/multi); torch's bundled HIP runtime must
    stay out of this process, libcedargpu.so links ROCm's own."""
    dist.all_reduce(torch.zeros(1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--policies", type=int, default=10_000)
    ap.add_argument("--batch", type=int, default=1_048_576, help="requests per GPU per step (one launch)")
    ap.add_argument("--order", default="random", choices=["random", "user"],
                    help="request order within the batch (locality study; random is the benchmark)")
    ap.add_argument("--variant", default="full", help="policy-shape study: full | scope-only | no-group | atomic-only")
    ap.add_argument("--hierarchy", default="dag", choices=["dag", "flat"],
                    help="k8s::Group hierarchy: a static depth-12 DAG over the 5k groups (C3 as BASELINE.json "
                         "states it) or none (groups without parents, round 1's workload)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--parity-sample", type=int, default=2048)
    ap.add_argument("--no-reload", dest="reload", action="store_false",
                    help="skip the RCCL hot-reload check after the timed region")
    ap.add_argument("--cpu-workers", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--latency-batches", type=int, default=10_000)
    ap.add_argument("--latency-batch", type=int, default=2048)
    ap.add_argument("--serve-threads", type=int, default=128,
                    help="caller threads of the serving-queue check (0: skip)")
    ap.add_argument("--serve-requests", type=int, default=262_144)
    ap.add_argument("--serve-max-batch", type=int, default=8192)
    ap.add_argument("--no-submit-to-results", dest="submit_to_results", action="store_false",
                    help="skip the 1M-request submit -> results measurement after the timed region")
    ap.add_argument("--configs-requests", type=int, default=262_144,
                    help="requests per secondary config (C2, C4) after the timed region (0: skip)")
    args = ap.parse_args()

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    from cedargpu import synth

    pop = synth.Population(seed=7, dag_depth=12 if args.hierarchy == "dag" else 0)
    entities = pop.static_entities() or None  # the image's static group hierarchy
    policies = synth.abac_policies(args.policies, seed=31, pop=pop, variant=args.variant)
    sars = synth.random_sars(args.batch, seed=1000 + rank, pop=pop)
    if args.order == "user":  # locality study: the batch grouped by caller
        sars.sort(key=lambda s: s["spec"]["user"])

    baseline = None
    usable, cpu_info = host_cpus()
    threads = args.cpu_workers or usable
    items, idx = oracle_items(sars[:args.parity_sample]) if rank == 0 else ([], [])
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        baseline = cpu_baseline(policies, items, args.cpu_seconds, threads, cpu_info, entities)

    # torch is plumbing only: the cross-rank barrier / max-reduce of timings runs over gloo on CPU
    # tensors. torch's bundled HIP runtime is never initialised in this process (it would clash
    # with the ROCm runtime libcedargpu.so links); device sync goes through the library.
    import torch
    import torch.distributed as dist

    import cedargpu
    from cedargpu.store import device_synchronize

    dist_on = world > 1
    if dist_on:
        # gloo prints its connection lines on stdout; rank 0's stdout carries only the JSON line
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group(backend="gloo")
            cpu_barrier(dist, torch)
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    # one GPU per rank; CEDARGPU_BENCH_DEVICE pins every rank to one device (a multi-rank rehearsal
    # on a one-GPU box: the RCCL reload then reports its error, RCCL wants distinct devices)
    device = int(os.environ.get("CEDARGPU_BENCH_DEVICE", local))

    image = cedargpu.build_image([cedargpu.MemoryStore("c3.cedar", policies)], epoch=1, entities=entities)
    ctx = cedargpu.Context(device)
    ctx.load(image, 1)
    # steady state: the batch before the measured one on this image sizes its result capacities
    # (the context's CapHint: first-pass reasons, on-device follow-up worklists)
    sizing = ctx.batch()
    sizing.add_sar_json(synth.sars_json(sars[:65536]))
    sizing.submit()
    sizing.wait()
    sizing.close()
    payload = synth.sars_json(sars).encode()  # the SAR bodies as the webhook receives them: bytes (not timed)
    t_build = time.perf_counter()
    b = ctx.batch()
    b.add_sar_json(payload)  # cg_batch_add_sar_json: SAR conversion + columnar encode, host threads
    t_enc = time.perf_counter()
    del payload
    b.submit()
    b.wait()  # correctness pass: results downloaded, follow-ups folded, host re-runs (if any) done
    t_first = time.perf_counter()
    followups, host_reruns = b.followups(), b.reruns()
    try:
        io = b.io()
    except AttributeError:  # an A/B build (CEDARGPU_AB_LIB) that predates cg_batch_io
        io = {"h2d_bytes": 0, "d2h_bytes": 0, "list_words": 0, "list_words_shared": 0}
    # the deciding lists as the device wrote them (a duplicate class reported whole is one word;
    # its members are listed on the host, not by the step)
    n_reasons = [b.route_words(i)[1] for i in range(len(b))]
    alg_bytes = algorithmic_bytes(sars, n_reasons, has_like=True)

    if args.warmup:
        b.time(args.warmup)
    device_synchronize(device)
    if dist_on:
        cpu_barrier(dist, torch)
    t0 = time.perf_counter()
    kernel_ms = b.time(args.steps)  # HIP events on the evaluation stream, K launches
    device_synchronize(device)
    wall_s = time.perf_counter() - t0
    if dist_on:
        cpu_barrier(dist, torch)
        t = torch.tensor([wall_s, kernel_ms], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        wall_s, kernel_ms = float(t[0]), float(t[1])

    # per-phase split of the same step (HIP events at each phase boundary; outside the timed region)
    split_steps = max(1, min(args.steps, 5))
    try:
        phases, split_total = b.time_split(split_steps)
        phases = {k: v / split_steps for k, v in phases.items()}
    except AttributeError:  # an A/B build (CEDARGPU_AB_LIB) that predates cg_batch_time_split
        phases, split_total = {"total": kernel_ms / args.steps * split_steps}, kernel_ms / args.steps * split_steps

    # the same 1M-request batch from the webhook's side: encoded again (SAR bodies -> request
    # blocks on the host threads), then submit -> results visible on the host, timed on the warm
    # buffer pool: string finalize, pinned staging, the one H2D copy, the complete step, the D2H
    # copy and the result binding. Outside the timed region (PCIe-inclusive; not `value`).
    s2r = None
    if rank == 0 and args.submit_to_results:
        # Twice: the first pass takes this batch size's pool blocks (the timed batch `b` still holds
        # its own), so the second, timed one runs on a warm pool with no allocation inside.
        payload2 = synth.sars_json(sars).encode()
        for rep in range(2):
            b2 = ctx.batch()
            t0e = time.perf_counter()
            b2.add_sar_json(payload2)
            t1e = time.perf_counter()
            try:
                b2.set_profile(True)
            except AttributeError:  # an A/B build without cg_batch_set_profile
                pass
            b2.submit()
            b2.wait()
            t2e = time.perf_counter()
            if rep == 0:
                b2.close()
        del payload2
        try:
            io2 = b2.io()
        except AttributeError:
            io2 = {"h2d_bytes": 0, "d2h_bytes": 0}
        try:
            split = b2.profile()
        except Exception:
            split = None
        s2r = {"requests": len(b2), "encode_s": t1e - t0e, "encode_per_s": len(b2) / (t1e - t0e),
               "submit_to_results_ms": (t2e - t1e) * 1e3, "decisions_per_s": len(b2) / (t2e - t1e),
               "h2d_bytes": io2["h2d_bytes"], "d2h_bytes": io2["d2h_bytes"], "split_ms": split,
               "what": "cg_batch_add_sar_json over the 1M SAR bodies (host threads), then cg_batch_submit -> "
                       "cg_batch_wait on a warm buffer pool (the second of two such batches): H2D of the request "
                       "heap / rows / strings, the complete device step, D2H of the results; split_ms from "
                       "cg_batch_profile (host phases, and HIP events around the copies and the step)"}
        b2.close()

    # submit -> results-visible latency on small batches (includes H2D, launch, D2H)
    lat = []
    if rank == 0 and args.latency_batches:
        # 8 different slices of the batch in rotation; each batch is encoded before its timed
        # submit -> wait (the encode is the caller's work, outside the interval)
        L = args.latency_batch
        chunks = [synth.sars_json(sars[k * L:(k + 1) * L]) for k in range(min(8, max(1, len(sars) // L)))]
        nxt = ctx.batch()
        nxt.add_sar_json(chunks[0])
        for k in range(args.latency_batches):
            lb = nxt
            t1 = time.perf_counter()
            lb.submit()
            lb.wait()
            lat.append((time.perf_counter() - t1) * 1e3)
            lb.close()
            if k + 1 < args.latency_batches:
                nxt = ctx.batch()
                nxt.add_sar_json(chunks[(k + 1) % len(chunks)])
        lat.sort()

    # small batches (the serving path's sizes): the complete step's device time (HIP events, one
    # launch below CEDARGPU_SMALL_N = 2,048 requests) and submit -> results wall time per size
    small = None
    if rank == 0 and args.latency_batches:
        small = {}
        for n in (64, 256, 2048):
            chunks = [synth.sars_json(sars[k * n:(k + 1) * n]).encode() for k in range(8)]
            sl, dev = [], None
            for it in range(80):
                sb = ctx.batch()
                sb.add_sar_json(chunks[it % 8])
                t1 = time.perf_counter()
                sb.submit()
                sb.wait()
                sl.append((time.perf_counter() - t1) * 1e3)
                if it == 79:
                    dev = sb.time(50) / 50
                sb.close()
            sl = sorted(sl[16:])
            small[str(n)] = {"device_step_ms": dev, "device_us_per_batch": dev * 1e3, "s2r_p50_ms": sl[len(sl) // 2],
                             "s2r_p90_ms": sl[int(len(sl) * 0.9)]}

    serving = None
    if rank == 0 and args.serve_threads and args.serve_requests:
        serving = serve(ctx, sars, args.serve_threads, args.serve_requests, args.serve_max_batch)

    parity = parity_sample(policies, items, idx, b, threads, entities) if rank == 0 and items else None
    configs = (secondary_configs(ctx, args.configs_requests, threads)
               if rank == 0 and world == 1 and args.configs_requests else None)
    reload = hot_reload(ctx, policies, rank, world, device, dist_on, entities=entities) if args.reload else None

    if rank == 0:
        ms_per_step = wall_s * 1e3 / args.steps
        decisions = args.batch * world * args.steps
        avg_kernel_ms = kernel_ms / args.steps
        step_achieved = alg_bytes / (avg_kernel_ms * 1e-3) / 1e9
        # the dominant kernel: the step phase with the most device time (HIP events on the step's
        # stream at every phase boundary); SURVEY §8(d) prices the whole decision's bytes, so
        # `achieved` is those bytes over that kernel's time (the whole step's figure beside it)
        dom = max((k for k in phases if k != "total"), key=phases.get) if len(phases) > 1 else "total"
        dom_ms = phases.get(dom, avg_kernel_ms)
        achieved = alg_bytes / (dom_ms * 1e-3) / 1e9
        dom_kernel = {"scan": "cedar_scan_kernel<8, 6, true>", "candidates": "cedar_probe_kernel<8, 32, 4, SPLIT, HOTC 16> (pooled, compact)",
                      "fu_big": "cedar_probe_kernel<64, 1024, 4, SPLIT, SLIM>", "group": "rocPRIM onesweep"}.get(dom, dom)
        traffic, pmc_kernels = None, None
        pmc = os.path.join(ROOT, "profiles", "pmc_latest.json")
        if os.path.exists(pmc):
            try:
                pj = json.load(open(pmc))
                if (pj.get("policies") == args.policies and pj.get("batch") == args.batch
                        and pj.get("hierarchy", "flat") == args.hierarchy):
                    traffic = pj.get("hbm_bytes_per_launch")
                    pmc_kernels = pj.get("kernels")
            except Exception:
                traffic = None
        # VALU busy fraction of the dominant kernel (SURVEY §8(d) honesty note): a wave64 VALU
        # instruction occupies its SIMD for 2 cycles (MI355X_MICROARCH.md), 1,024 SIMDs at 2.4 GHz
        valu = None
        prefix = {"scan": "cedar_scan_kernel<8u, 6u, true", "candidates": "cedar_probe_kernel<8u, 32u"}.get(dom)
        if pmc_kernels and prefix:
            for name, c in pmc_kernels.items():
                if name.startswith(prefix) and "SQ_INSTS_VALU" in c:
                    valu = {"kernel": name, "valu_insts": c["SQ_INSTS_VALU"],
                            "valu_busy_frac": c["SQ_INSTS_VALU"] * 2 / (1024 * 2.4e9 * dom_ms * 1e-3),
                            "valu_share_of_issued": c["SQ_INSTS_VALU"] / max(1.0, c["SQ_INSTS_VALU"] + c.get("SQ_INSTS_SALU", 0)
                                                                            + c.get("SQ_INSTS_VMEM_RD", 0) + c.get("SQ_INSTS_LDS", 0))}
                    break
        out = {
            "metric": "authz decisions/sec (node) at 10k policies",
            "value": decisions / wall_s,
            "unit": "decisions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32",
            "data": "synthetic (seeded SubjectAccessReviews + generated ABAC policies; no dataset)",
            "config": {"workload": "C3 single-GPU shard: 10k ABAC policies (k8s::Group scope, namespace/apiGroup/"
                                   "resource/labelSelector/like conditions) x synthetic SARs"
                                   + (", deep k8s::Group `in` hierarchy (static DAG over 5k groups, depth <= 12, "
                                      "compiled in-closure rows)" if entities else ""),
                       "policies": args.policies, "requests_per_gpu": args.batch, "tiers": 1,
                       "variant": args.variant, "hierarchy": args.hierarchy,
                       "static_entities": len(entities or []),
                       "step": "first pass + gather + on-device follow-up launches (every request decided, "
                               "all reasons and errors listed, on the device)",
                       "device_followup_requests": followups,
                       "rerun_requests": host_reruns,
                       "request_order": (f"{args.order} as uploaded; batches of >= 65,536 requests are grouped on the "
                                         "device inside every timed step (rocPRIM radix sort of the encoder's per-request "
                                         "key over (action, resource type), principal key ancestors, hot values; the "
                                         "first-pass kernels read the rows through that order)" if os.environ.get("CEDARGPU_GROUP_DEV", "1") != "0"
                                         else f"{args.order}; host radix sort at submit, outside the timed step (A/B)"),
                       "parallelism": f"request-sharded x{world}, image replicated"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "dominant_kernel": dom_kernel, "dominant_phase": dom, "dominant_kernel_ms": dom_ms,
                         "step_achieved": step_achieved, "step_frac": step_achieved / HBM_PEAK_GBS,
                         "kernel_ms": avg_kernel_ms, "alg_bytes_per_launch": alg_bytes,
                         "alg_bytes_per_decision": alg_bytes / args.batch,
                         "phases_ms": phases, "phases_total_ms": split_total / split_steps,
                         "valu": valu,
                         "launch": "one complete step on one stream: the device grouping (rocPRIM onesweep sort of the encoder's "
                                   "keys), cedar_scan_kernel, the SPLIT candidate pass, cedar_fu_gather and the follow-up "
                                   "launches (rocprofv3 kernel stats in profiles/r06/)",
                         "achieved_is": "SURVEY §8(d) algorithmic bytes of every decision in the step / the dominant kernel's "
                                        "time (HIP events at its phase boundaries); step_achieved: over the whole step",
                         "traffic_source": "PMC FETCH_SIZE x2 + WRITE_SIZE summed over one step's dispatches "
                                           "(tools/pmc_kernels.sh, profiles/pmc_latest.json)" if traffic else None},
            "transfer": {"h2d_bytes_per_request": io["h2d_bytes"] / args.batch, "d2h_bytes_per_request": io["d2h_bytes"] / args.batch,
                         "ancestor_list_words": io["list_words"], "ancestor_list_words_shared": io["list_words_shared"],
                         "what": "the one H2D upload (request heap with interned ancestor lists, rows, strings, grouping "
                                 "keys) and the one D2H result copy of the 1M-request batch"},
            "submit_to_results_1m": s2r,
            "cpu_baseline": baseline,
            "parity_sample": parity,
            "reload": reload,
            "serving": serving,
            "configs": configs,
            "small_batches": small,
            "latency": {"batch": args.latency_batch, "p50_ms": lat[len(lat) // 2] if lat else None,
                        "p99_ms": lat[min(len(lat) - 1, int(len(lat) * 0.99))] if lat else None,
                        "p999_ms": lat[min(len(lat) - 1, int(len(lat) * 0.999))] if lat else None,
                        "max_ms": lat[-1] if lat else None, "batches": len(lat),
                        "what": "cg_batch_submit -> cg_batch_wait (string finalize, H2D, kernel writing its "
                                "results into pinned host memory, the counters' D2H, overflow folds and re-runs) "
                                "per batch of pre-encoded SubjectAccessReviews"},
            "host": {"encode_s": t_enc - t_build, "first_pass_s": t_first - t_enc},
        }
        if baseline:
            out["speedup_vs_cpu_baseline"] = out["value"] / baseline["value"]
        print(json.dumps(out), flush=True)
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
