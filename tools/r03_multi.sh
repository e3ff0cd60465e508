#!/bin/bash
# Multi-rank rehearsal of bench.py on a one-GPU box: 2 ranks (torchrun, gloo barrier / max-reduce),
# both pinned to GPU 0; checks the distributed path end to end (the RCCL reload needs distinct GPUs).
set -o pipefail
TAG=${1:-r03multi}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 120 python -c "import sys; sys.path.insert(0, 'cedar-access-control-for-k8s_amd'); import cedargpu; print('devices', cedargpu.device_count()); c = cedargpu.Context(0); c.close(); print('context ok')" || exit 1
# does torch's accelerator query (what dist.barrier() makes) before the first context break it?
timeout -k 10 120 python -c "import sys; sys.path.insert(0, 'cedar-access-control-for-k8s_amd'); import torch; print('accelerator', torch._C._get_accelerator()); import cedargpu; c = cedargpu.Context(0); c.close(); print('context after accelerator query ok')" || echo "context after accelerator query FAILED"
CEDARGPU_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 1 --latency-batches 0 --serve-threads 0 --configs-requests 0 > gpurun_out/$TAG/bench2.json 2> gpurun_out/$TAG/bench2.err || { echo "2-rank bench failed"; tail -30 gpurun_out/$TAG/bench2.err; exit 1; }
python3 -c "import json; l=open('gpurun_out/$TAG/bench2.json').read().strip().splitlines(); assert len(l) == 1, l[:3]; d=json.loads(l[0]); print('n_gpus', d['n_gpus'], 'value', d['value'], 'ms', d['ms_per_step'], 'reload', str(d['reload'])[:200])"
