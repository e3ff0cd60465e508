"""C4 (admission) work profile: kernel time per launch, reasons per request, overflow share.
Run with CEDARGPU_PROBE_STATS=1 for the probe kernel's per-request work counters (stderr).
Diagnostic only: python tools/c4_probe.py [--requests 32768] [--policies 1000]."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cedar-access-control-for-k8s_amd"))

import cedargpu  # noqa: E402
from cedargpu import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=32768)
    ap.add_argument("--policies", type=int, default=1000)
    args = ap.parse_args()
    stores = [cedargpu.MemoryStore("adm.cedar", synth.admission_policies(args.policies, seed=3)),
              cedargpu.ALLOW_ALL_ADMISSION]
    image = cedargpu.build_image(stores, epoch=1)
    ctx = cedargpu.Context(0)
    ctx.load(image, 1)
    reviews = synth.admission_reviews(args.requests, seed=4000)
    b = ctx.batch()
    b.add_admission_json(json.dumps(reviews, separators=(",", ":")))
    t0 = time.perf_counter()
    b.submit()
    b.wait()
    first_ms = (time.perf_counter() - t0) * 1e3
    out = {"requests": len(b), "cold_submit_to_results_ms": first_ms, "reruns": b.reruns()}
    if not os.environ.get("CEDARGPU_PROBE_STATS"):
        out["kernel_ms"] = b.time(5) / 5
    hist = {}
    for i in range(len(b)):
        try:
            n = len(b.reasons(i)[0])
        except Exception:
            n = -1
        k = "0" if n == 0 else "1-8" if n <= 8 else "9-64" if n <= 64 else ">64" if n > 0 else "skip"
        hist[k] = hist.get(k, 0) + 1
    out["reasons_per_request"] = hist
    b.close()
    warm = []
    for _ in range(3):  # the first batch's blocks are back in the pool
        b2 = ctx.batch()
        b2.add_admission_json(json.dumps(reviews, separators=(",", ":")))
        t0 = time.perf_counter()
        b2.submit()
        b2.wait()
        warm.append((time.perf_counter() - t0) * 1e3)
        b2.close()
    out["warm_submit_to_results_ms"] = warm
    print(json.dumps(out))


if __name__ == "__main__":
    main()
