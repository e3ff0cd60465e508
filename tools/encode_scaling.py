"""Host encode scaling: cg_batch_add_sar_json over C3 SAR bodies with 2..16 worker threads
(CEDARGPU_HOST_THREADS), each run in a fresh process (the variable is read per call, the image's
encoder cache per process). Prints wall seconds and per-request microseconds per thread count."""
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = int(os.environ.get("N", "262144"))

if len(sys.argv) > 1 and sys.argv[1] == "child":
    sys.path.insert(0, os.path.join(ROOT, "cedar-access-control-for-k8s_amd"))
    import cedargpu
    from cedargpu import synth
    pop = synth.Population(seed=7, dag_depth=12)
    img = cedargpu.build_image([cedargpu.MemoryStore("c3.cedar", synth.abac_policies(10000, seed=31, pop=pop))], epoch=1,
                               entities=pop.static_entities())
    ctx = cedargpu.Context(0)
    ctx.load(img, 1)
    payload = synth.sars_json(synth.random_sars(N, seed=1000, pop=pop)).encode()
    out = []
    for rep in range(3):
        b = ctx.batch()
        t0 = time.perf_counter()
        b.add_sar_json(payload)
        out.append(time.perf_counter() - t0)
        b.close()
    print(json.dumps({"threads": os.environ.get("CEDARGPU_HOST_THREADS"), "n": N, "runs_s": out,
                      "us_per_req_wall": min(out) / N * 1e6}), flush=True)
    sys.exit(0)

for t in (2, 4, 8, 16):
    env = dict(os.environ, CEDARGPU_HOST_THREADS=str(t))
    subprocess.run([sys.executable, os.path.abspath(__file__), "child"], env=env, check=True, timeout=300)
