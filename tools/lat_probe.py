"""Latency breakdown of one small batch (submit vs wait, kernel alone, re-run share) on the bench's
C3 workload. Diagnostic only: python tools/lat_probe.py [--batch 2048] [--batches 200]."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cedar-access-control-for-k8s_amd"))

import cedargpu  # noqa: E402
from cedargpu import synth  # noqa: E402


def pct(xs, p):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(p * len(xs)))]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=2048)
    ap.add_argument("--batches", type=int, default=200)
    ap.add_argument("--policies", type=int, default=10000)
    args = ap.parse_args()
    pop = synth.Population(seed=7)
    policies = synth.abac_policies(args.policies, seed=31, pop=pop)
    sars = synth.random_sars(args.batch * 8, seed=1000, pop=pop)
    image = cedargpu.build_image([cedargpu.MemoryStore("c3.cedar", policies)], epoch=1)
    ctx = cedargpu.Context(0)
    ctx.load(image, 1)
    chunks = [synth.sars_json(sars[k * args.batch:(k + 1) * args.batch]) for k in range(8)]
    out = {"batch": args.batch, "batches": args.batches}
    big = []
    for c in chunks:
        b = ctx.batch()
        b.add_sar_json(c)
        b.submit()
        b.wait()
        nr = [b.reasons(i) for i in range(len(b))]
        big.append((sum(1 for r, e in nr if len(r) > 8 or e > 4), sum(1 for r, _ in nr if len(r) > 64)))
        out.setdefault("kernel_ms_per_launch", []).append(b.time(20) / 20)
        b.close()
    out["rerun_requests_over_cap8_and_over_64_per_batch"] = big
    sub, wai, tot = [], [], []
    pending = []
    for k in range(args.batches):
        lb = ctx.batch()
        lb.add_sar_json(chunks[k % 8])
        pending.append(lb)
    for lb in pending:
        t0 = time.perf_counter()
        lb.submit()
        t1 = time.perf_counter()
        lb.wait()
        t2 = time.perf_counter()
        sub.append((t1 - t0) * 1e3)
        wai.append((t2 - t1) * 1e3)
        tot.append((t2 - t0) * 1e3)
        lb.close()
    for name, xs in (("submit_ms", sub), ("wait_ms", wai), ("total_ms", tot)):
        out[name] = {"p50": pct(xs, 0.5), "p99": pct(xs, 0.99), "max": max(xs)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
