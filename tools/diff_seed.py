"""Debug helper: print GPU vs oracle diagnostics for the first mismatching item of a randgen seed."""
import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "tests"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "cedar-access-control-for-k8s_amd")]
import cedar_oracle as co
import cedargpu
from randgen import Gen

seed = int(sys.argv[1])
g = Gen(seed)
nt = g.r.randint(1, 2)
texts = [g.atomic_policies(g.r.randint(1, 40)) for _ in range(nt)]
items = [g.item() for _ in range(400)]
stores = [cedargpu.MemoryStore(f"a{t}.cedar", x) for t, x in enumerate(texts)]
ctx = cedargpu.Context(0)
tiers = cedargpu.TieredPolicyStores(stores, ctx=ctx)
got = tiers.is_authorized_batch(items)
ot = [co.PolicySet.from_bytes(f"a{t}.cedar", x) for t, x in enumerate(texts)]
bad = 0
for (ents, req), (ok, diag) in zip(items, got):
    want_ok, want, _ = co.tiered_is_authorized(ot, co.entities_from_json(ents), co.request_from_json(req))
    if diag != want.to_go_json():
        bad += 1
        if bad <= 3:
            print("REQ", req)
            print("ENTS", ents)
            print("GPU ", diag)
            print("WANT", want.to_go_json())
print("mismatches", bad, "of", len(items))
