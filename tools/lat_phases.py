"""Median host-side phases of small-batch submit -> results (CEDARGPU_TRACE_LAT=1 lines) on the
C3 DAG workload: python tools/lat_phases.py N BATCHES (run with CEDARGPU_TRACE_LAT=1; stderr is
parsed from a child run)."""
import collections
import json
import os
import re
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if len(sys.argv) > 3 and sys.argv[3] == "child":
    sys.path.insert(0, os.path.join(ROOT, "cedar-access-control-for-k8s_amd"))
    import cedargpu
    from cedargpu import synth
    n, nb = int(sys.argv[1]), int(sys.argv[2])
    pop = synth.Population(seed=7, dag_depth=12)
    img = cedargpu.build_image([cedargpu.MemoryStore("c3.cedar", synth.abac_policies(10000, seed=31, pop=pop))], epoch=1,
                               entities=pop.static_entities())
    ctx = cedargpu.Context(0)
    ctx.load(img, 1)
    sars = synth.random_sars(n * 8, seed=1000, pop=pop)
    chunks = [synth.sars_json(sars[k * n:(k + 1) * n]).encode() for k in range(8)]
    lat = []
    for it in range(nb):
        b = ctx.batch()
        b.add_sar_json(chunks[it % 8])
        t0 = time.perf_counter()
        b.submit()
        b.wait()
        lat.append((time.perf_counter() - t0) * 1e6)
        b.close()
    lat.sort()
    print(json.dumps({"n": n, "s2r_p50_us": lat[len(lat) // 2]}), flush=True)
    sys.exit(0)
n, nb = sys.argv[1], sys.argv[2]
env = dict(os.environ, CEDARGPU_TRACE_LAT="1")
p = subprocess.run([sys.executable, os.path.abspath(__file__), n, nb, "child"], env=env, capture_output=True, text=True, timeout=300)
print(p.stdout.strip())
ph = collections.defaultdict(list)
for line in p.stderr.splitlines():
    m = re.match(r"LAT (submit|wait)(.*)", line)
    if not m:
        continue
    for k, v in re.findall(r"(\w+)=([\d.]+)", m.group(2)):
        ph[m.group(1) + "." + k].append(float(v))
for k, v in ph.items():
    v = sorted(v[len(v) // 5:])  # warm
    print(f"{k:28s} p50 {v[len(v) // 2]:9.1f} us")
