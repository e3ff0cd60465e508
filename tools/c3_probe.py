"""C3 work profile: the probe kernel's per-request counters on the benchmark's workload.
Diagnostic only: CEDARGPU_PROBE_STATS=1 python tools/c3_probe.py [--hierarchy dag|flat] [--requests N]
(without the variable: the complete step's time and the follow-up / re-run counts)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cedar-access-control-for-k8s_amd"))

import cedargpu  # noqa: E402
from cedargpu import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--requests", type=int, default=1 << 20)
    ap.add_argument("--policies", type=int, default=10_000)
    ap.add_argument("--hierarchy", default="dag", choices=["dag", "flat"])
    args = ap.parse_args()
    pop = synth.Population(seed=7, dag_depth=12 if args.hierarchy == "dag" else 0)
    entities = pop.static_entities() or None
    policies = synth.abac_policies(args.policies, seed=31, pop=pop)
    sars = synth.random_sars(args.requests, seed=1000, pop=pop)
    image = cedargpu.build_image([cedargpu.MemoryStore("c3.cedar", policies)], epoch=1, entities=entities)
    ctx = cedargpu.Context(0)
    ctx.load(image, 1)
    for rep in range(2):  # the first batch sizes the capacities of the second
        b = ctx.batch()
        b.add_sar_json(synth.sars_json(sars))
        t0 = time.perf_counter()
        b.submit()
        b.wait()
        print(f"batch {rep}: submit->results {1e3 * (time.perf_counter() - t0):.2f} ms, followups {b.followups()}, "
              f"reruns {b.reruns()}", flush=True)
        if rep == 1 and not os.environ.get("CEDARGPU_PROBE_STATS"):
            print(f"complete step {b.time(10) / 10:.3f} ms", flush=True)
        b.close()
    ctx.close()


if __name__ == "__main__":
    main()
