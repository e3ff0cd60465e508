"""Small-batch step on C3 (10k policies, group DAG): device time of the complete step (HIP events,
cg_batch_time) and submit -> results wall time, per batch size, for the one-launch small path
(CEDARGPU_SMALL_N large) and the split path (CEDARGPU_SMALL_N=0)."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cedar-access-control-for-k8s_amd"))
import cedargpu  # noqa: E402
from cedargpu import synth  # noqa: E402

pop = synth.Population(seed=7, dag_depth=12)
ents = pop.static_entities()
pol = synth.abac_policies(10000, seed=31, pop=pop)
img = cedargpu.build_image([cedargpu.MemoryStore("c3.cedar", pol)], epoch=1, entities=ents)
ctx = cedargpu.Context(0)
ctx.load(img, 1)
sars = synth.random_sars(65536, seed=1000, pop=pop)
sizes = [int(x) for x in os.environ.get("SIZES", "16,64,128,256,512,1024,2048,4096").split(",")]
out = []
for small in ("0", "100000"):
    os.environ["CEDARGPU_SMALL_N"] = small
    for n in sizes:
        payloads = [synth.sars_json(sars[k * n:(k + 1) * n]) for k in range(8)]
        lat = []
        dev = None
        for it in range(60):
            b = ctx.batch()
            b.add_sar_json(payloads[it % 8])
            t0 = time.perf_counter()
            b.submit()
            b.wait()
            lat.append((time.perf_counter() - t0) * 1e3)
            if it == 59:
                dev = b.time(50) / 50
                rr = b.reruns()
            b.close()
        lat = sorted(lat[10:])
        row = {"path": "split" if small == "0" else "one-launch", "n": n, "device_step_ms": round(dev, 4),
               "s2r_p50_ms": round(lat[len(lat) // 2], 4), "s2r_p90_ms": round(lat[int(len(lat) * 0.9)], 4), "reruns": rr}
        print(json.dumps(row), flush=True)
        out.append(row)
