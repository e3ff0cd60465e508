"""Differential fuzz of the device-grouped path (>= 65,536 requests per batch): random all-atomic
corpora (scope bitsets, bucket filters, duplicate classes) over random static hierarchies, each
batch checked request by request against the C++ oracle. Usage: python tools/fuzz_grouped.py
FIRST_SEED N_SEEDS [REQUESTS]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "cedar-access-control-for-k8s_amd")]
import cedargpu  # noqa: E402
from cedar_ref import RefPolicySet, items_json  # noqa: E402
from randgen import Gen  # noqa: E402
from test_gpu_parity import _atomic_only  # noqa: E402


def main():
    first, n = int(sys.argv[1]), int(sys.argv[2])
    n_req = int(sys.argv[3]) if len(sys.argv) > 3 else 70000
    ctx = cedargpu.Context(0)
    bad_all = total = 0
    t0 = time.time()
    for seed in range(first, first + n):
        g = Gen(seed, static=seed % 2 == 1)
        ents = g.static_entities() if seed % 2 == 1 else None
        stores = _atomic_only([(f"p{t}.cedar", g.atomic_policies(g.r.randint(5, 80))) for t in range(g.r.randint(1, 3))])
        pool = [g.item() for _ in range(4000)]
        items = [pool[g.r.randrange(len(pool))] for _ in range(n_req)]  # (repeats: grouped neighbours)
        got = cedargpu.TieredPolicyStores(stores, ctx=ctx, entities=ents).is_authorized_batch(items)
        ref = RefPolicySet.from_stores(stores, ents)
        ref.load_items(items_json(items))
        want = ref.evaluate(16)
        ref.close()
        bad = sum(1 for (ok, d), (wok, _, wd, _) in zip(got, want) if (ok, d) != (wok, wd))
        bad_all += bad
        total += len(items)
        print(f"seed {seed}: {bad} mismatches of {len(items)} ({time.time() - t0:.0f} s)", flush=True)
    print("total", bad_all, "of", total)
    ctx.close()
    sys.exit(1 if bad_all else 0)


if __name__ == "__main__":
    main()
