"""Serving-queue latency probe: the bench's serving check alone (C3 image, 256 caller threads).
Diagnostic only: CEDARGPU_TRACE_LAT=1 python tools/serve_probe.py [--threads 256]."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "cedar-access-control-for-k8s_amd"))
sys.path.insert(0, ROOT)

import cedargpu  # noqa: E402
from cedargpu import synth  # noqa: E402
from bench import serve  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--threads", type=int, default=256)
    ap.add_argument("--requests", type=int, default=131072)
    ap.add_argument("--max-batch", type=int, default=8192)
    args = ap.parse_args()
    pop = synth.Population(seed=7)
    image = cedargpu.build_image([cedargpu.MemoryStore("c3.cedar", synth.abac_policies(10000, seed=31, pop=pop))], epoch=1)
    ctx = cedargpu.Context(0)
    ctx.load(image, 1)
    sars = synth.random_sars(32768, seed=1000, pop=pop)
    print(json.dumps(serve(ctx, sars, args.threads, args.requests, args.max_batch)))


if __name__ == "__main__":
    main()
