"""Debug: the retire-under-stall sequence of test_authorizer_deadline_under_stall, printing every
outcome and exception instead of failing safe."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "cedar-access-control-for-k8s_amd"), os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
import cedargpu
from cedargpu import synth
CORPUS = json.load(open(os.path.join(ROOT, "tests", "golden", "reference_corpus.json")))
DEMO = "\n".join(v for k, v in sorted(CORPUS["demo"].items()) if k.startswith("authorization"))
ctx = cedargpu.Context(0)
tiers = cedargpu.TieredPolicyStores([cedargpu.MemoryStore("demo.cedar", DEMO)], ctx=ctx)
sars = synth.random_sars(200, seed=71, pop=synth.Population(seed=71, n_users=300, n_groups=30))
payload = json.dumps(sars)
def run(timeout, tag):
    b = ctx.batch()
    b.add_sar_json(payload)
    t0 = time.perf_counter()
    try:
        b.submit()
        b.wait(timeout)
        print(tag, "ok", round(time.perf_counter() - t0, 3), [b.authz(i)[0] for i in range(5)], flush=True)
    except Exception as e:
        print(tag, "exc", type(e).__name__, e, round(time.perf_counter() - t0, 3), flush=True)
    t1 = time.perf_counter()
    b.close()
    print(tag, "close", round(time.perf_counter() - t1, 4), flush=True)
run(5.0, "warm")
ctx.inject_fault(cedargpu.FAULT_STALL, 400_000)
run(0.05, "stall1")
run(0.05, "stall2")
ctx.inject_fault(cedargpu.FAULT_NONE)
time.sleep(1.0)
run(5.0, "after")
run(5.0, "after2")
ctx.close()
