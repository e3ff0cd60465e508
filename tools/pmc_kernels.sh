#!/bin/bash
# PMC passes over a short C3 bench run, reduced per kernel of the complete step (scan, candidate
# pass, large stage): vL1D accesses, L2 requests, instruction mix, wave cycles, LDS bank conflicts
# (SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE: conflict cycles over LDS-active cycles), HBM fetch.
# Usage: tools/pmc_kernels.sh TAG   (extra env, e.g. CEDARGPU_NO_CLOSURE=1, applies to every pass)
set -o pipefail
TAG=${1:-pmck}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --latency-batches 0 --parity-sample 0 --no-reload --serve-threads 0 --configs-requests 0 ${BENCH_ARGS}"
run() {
  local name=$1; shift
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS) > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -20 $OUT/$name.log; return 1; }
}
run tcp TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum && \
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAIT_ANY && \
run lds SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE && \
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
for K in cedar_scan_kernel "cedar_probe_kernel<8u, 32u" "cedar_probe_kernel<64u, 1024u"; do
  echo "== $K"; PMC_KERNEL="$K" python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT
done > $OUT/summary.txt && cat $OUT/summary.txt && \
python3 $GRAFT_REPO_ROOT/tools/pmc_step.py $OUT 10000 1048576 dag > $OUT/step.json && python3 -c "import json; d=json.load(open('$OUT/step.json')); print('step HBM bytes', d.get('hbm_bytes_per_launch'), 'steps', d.get('steps_fetch'))"
