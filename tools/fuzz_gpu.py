"""Wider differential fuzz on the GPU than the test suite's fixed seeds: random atomic corpora
(probe kernels) and random general corpora (stream kernel), half of them over a random static
hierarchy, each vs the C++ oracle on the merged EntityMaps. Prints mismatches per kind.
Usage: python tools/fuzz_gpu.py FIRST_SEED N_SEEDS"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "cedar-access-control-for-k8s_amd")]
import cedargpu  # noqa: E402
from cedar_ref import RefPolicySet, items_json  # noqa: E402
from randgen import Gen  # noqa: E402
from test_gpu_parity import _atomic_only  # noqa: E402


def run(ctx, stores, items, ents):
    tiers = cedargpu.TieredPolicyStores(stores, ctx=ctx, entities=ents)
    got = tiers.is_authorized_batch(items)
    ref = RefPolicySet.from_stores(stores, ents)
    ref.load_items(items_json(items))
    want = ref.evaluate(8)
    ref.close()
    return sum(1 for (ok, d), (wok, _, wd, _) in zip(got, want) if (ok, d) != (wok, wd))


def main():
    first, n = int(sys.argv[1]), int(sys.argv[2])
    ctx = cedargpu.Context(0)
    tot = {"atomic": [0, 0], "general": [0, 0]}
    t0 = time.time()
    for seed in range(first, first + n):
        static = seed % 2 == 1
        g = Gen(seed, static=static)
        ents = g.static_entities() if static else None
        texts = [(f"p{t}.cedar", g.atomic_policies(g.r.randint(1, 60))) for t in range(g.r.randint(1, 3))]
        items = [g.item() for _ in range(300)]
        bad = run(ctx, _atomic_only(texts), items, ents)
        tot["atomic"][0] += bad
        tot["atomic"][1] += len(items)
        g2 = Gen(seed + 500000, static=static)
        ents2 = g2.static_entities() if static else None
        stores2 = [cedargpu.MemoryStore(f"t{t}.cedar", g2.policies(g2.r.randint(0, 14))) for t in range(g2.r.randint(1, 3))]
        items2 = [g2.item() for _ in range(200)]
        bad2 = run(ctx, stores2, items2, ents2)
        tot["general"][0] += bad2
        tot["general"][1] += len(items2)
        if bad or bad2:
            print(f"seed {seed}: atomic mismatches {bad}, general {bad2}", flush=True)
        if (seed - first) % 20 == 19:
            print(f"{seed - first + 1} seeds, {time.time() - t0:.0f} s, {tot}", flush=True)
    print("total", tot, f"{time.time() - t0:.0f} s")
    ctx.close()


if __name__ == "__main__":
    main()
