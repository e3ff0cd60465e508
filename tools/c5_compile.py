"""C5's one-CRD incremental compile on the host (CEDARGPU_COMPILE_TIMES=1 prints its phases): 100k
policies over 1,000 tenant documents, one document edited, rebuilt incrementally; prints the
rebuild time and the image's SHA-1 (the parallel index build writes the same bytes)."""
import hashlib
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cedar-access-control-for-k8s_amd"))
import cedargpu  # noqa: E402
from cedargpu import synth  # noqa: E402

tpop = synth.Population(seed=7, n_namespaces=1000)
docs = synth.multitenant_policies(100_000, seed=51, pop=tpop)
comp = cedargpu.Compiler()
img0 = comp.build([cedargpu.CRDStore(docs)], epoch=300)
print("=== incremental", file=sys.stderr, flush=True)
docs[500] = (docs[500][0], docs[500][1], docs[500][2].replace("permit", "forbid", 1))
times = []
for rep in range(3):
    t0 = time.perf_counter()
    img = comp.build([cedargpu.CRDStore(docs)], epoch=301 + rep)
    times.append((time.perf_counter() - t0) * 1e3)
    print("split ms", {k: round(v * 1e3, 1) for k, v in comp.last_times.items()}, flush=True)
print("incremental rebuild ms", [round(t, 1) for t in times], hashlib.sha1(img).hexdigest(), len(img), flush=True)
