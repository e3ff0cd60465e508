import sys, os, json, collections
sys.path[:0] = ["/root/repo", "/root/repo/cedar-access-control-for-k8s_amd", "/root/repo/oracle"]
import bench
from cedargpu import synth
import cedar_ref as cr
pop = synth.Population(seed=7, dag_depth=12)
ents = pop.static_entities()
pols = synth.abac_policies(10000, seed=31, pop=pop)
sars = synth.random_sars(1600, seed=1000, pop=pop)
items, idx = bench.oracle_items(sars)
s = cr.RefPolicySet(); s.set_entities(json.dumps(ents)); s.add_tier(); s.add_document("c3.cedar", pols)
s.load_items(cr.items_json(items))
res = s.evaluate(threads=8)
ns = [len(json.loads(r)) if r and r != "null" else 0 for a, t, d, r in res]
ns.sort()
n = len(ns)
print("n", n, "mean", sum(ns)/n, "p50", ns[n//2], "p90", ns[n*9//10], "p96", ns[n*96//100], "p99", ns[n*99//100], "max", ns[-1])
for lim in (8, 16, 32, 64, 128, 256, 512):
    print(lim, sum(1 for x in ns if x > lim) / n)
