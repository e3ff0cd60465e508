"""Debug: test_index_kernel_hit_overflow_reruns[150] scenario, split path; prints mismatching
diagnostics and the batch's follow-up / re-run counts (CEDARGPU_LONG_SLOTS as set)."""
import json
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cedar-access-control-for-k8s_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
os.environ["CEDARGPU_SMALL_N"] = "0"
import cedargpu
import cedar_oracle as co
from randgen import Gen
n = 150
pols = "\n".join(f'permit (principal in k8s::Group::"g{i % 3}", action, resource) when {{ principal.age > {i % 7} }};' for i in range(n))
pols += '\nforbid (principal, action == k8s::Action::"create", resource) when { principal has nick };'
stores = [cedargpu.MemoryStore("many.cedar", pols)]
g = Gen(91)
items = [g.item() for _ in range(300)]
ctx = cedargpu.Context(0)
ctx.load(cedargpu.build_image(stores), 1)
b = ctx.batch()
b.add(*items[0]) if False else None
b.add_json(json.dumps([{"entities": e, "request": r} for e, r in items]))
b.submit(); b.wait()
print("followups", b.followups(), "reruns", b.reruns())
ps = co.PolicySet()
for d in stores[0].documents():
    _, fname, body, pre, suf = d
    for i, p in enumerate(co.parse_policies(body, fname)):
        ps.add(f"{pre}{i}{suf}", p)
bad = 0
for i, (e, r) in enumerate(items):
    ok, diag, _ = co.tiered_is_authorized([ps], co.entities_from_json(e), co.request_from_json(r))
    got = b.diagnostic(i)
    if got != diag.to_go_json():
        bad += 1
        if bad <= 2:
            gj, wj = json.loads(got), json.loads(diag.to_go_json())
            print("item", i, "res", b.decision(i), "n reasons got/want", len(gj.get("reasons", [])), len(wj.get("reasons", [])),
                  "errors got/want", len(gj.get("errors", [])), len(wj.get("errors", [])))
            ge = [x["policy"] + ":" + x["message"][-30:] for x in gj.get("errors", [])]
            we = [x["policy"] for x in wj.get("errors", [])]
            print("  got errors", ge[:12])
            print("  want errors", we[:12])
print("mismatches", bad)
