#!/bin/bash
# rocprofv3 PMC passes over a short bench run (one counter group per pass, each under its own
# time limit), then tools/pmc_summary.py reduces them to per-launch figures of the probe kernel.
set -o pipefail
TAG=${1:-pmc}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 1 --no-cpu-baseline --latency-batches 0 --parity-sample 0 --no-reload --serve-threads 0 --configs-requests 0 ${BENCH_ARGS}"
run() {
  local name=$1; shift
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS) > $OUT/$name.log 2>&1 || { echo "pass $name failed"; tail -20 $OUT/$name.log; return 1; }
}
run fetch FETCH_SIZE && \
run write WRITE_SIZE && \
run sq SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD && \
run tcc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE && \
run tcp TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum && \
python3 $GRAFT_REPO_ROOT/tools/pmc_summary.py $OUT > $OUT/summary.json && cat $OUT/summary.json
