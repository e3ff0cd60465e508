#!/bin/bash
# One GPU session, steps chosen by name (each GPU step under its own limit, chained: the first
# failure ends the session). Usage: tools/gpu_session.sh TAG step [step ...]
#   tests    the GPU parity suite            smoke   __graft_entry__.smoke()
#   stats    C3 work counters (scan + candidate pass, CEDARGPU_SCAN_STATS / CAND_STATS)
#   quick    short bench (no CPU baseline, latency, serving or reload)
#   bench    the full default bench line     prof    rocprofv3 kernel stats of a short bench
#   pmc      per-kernel PMC passes (tools/pmc_kernels.sh)
# Environment: BENCH_ARGS (extra bench.py flags), AB_ENV (env assignments for an A/B leg, e.g.
# "CEDARGPU_X=0"; the quick bench then runs once per leg separated by ';').
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
for step in "$@"; do
  case $step in
    tests)
      timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
      tail -2 $O/pytest.log ;;
    smoke)
      timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $O/smoke.log; exit 1; }
      tail -1 $O/smoke.log ;;
    stats)
      CEDARGPU_SCAN_STATS=1 CEDARGPU_CAND_STATS=1 timeout -k 10 240 python -u tools/c3_probe.py > $O/stats.log 2>&1 || { echo "stats failed"; tail -20 $O/stats.log; exit 1; }
      tail -4 $O/stats.log ;;
    quick)
      IFS=';' read -ra LEGS <<< "${AB_ENV:-}"
      [ ${#LEGS[@]} -eq 0 ] && LEGS=("")
      k=0
      for leg in "${LEGS[@]}" "${LEGS[@]}"; do
        env $leg timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-batches 0 --serve-threads 0 --no-reload --configs-requests 0 ${QUICK_S2R:---no-submit-to-results} ${BENCH_ARGS} > $O/quick_$k.json 2> $O/quick_$k.err || { echo "bench failed ($leg)"; tail -20 $O/quick_$k.err; exit 1; }
        python3 -c "
import json; d=json.load(open('$O/quick_$k.json')); p=d['roofline'].get('phases_ms',{})
s=d.get('submit_to_results_1m') or {}; print('[$leg]', round(d['value']/1e6,1), 'M/s ms', round(d['ms_per_step'],4), 'phases', {a: round(b,4) for a,b in p.items()}, 'parity', d['parity_sample']['mismatches'], 's2r', s and (round(s['submit_to_results_ms'],1), 'ms', round(s['h2d_bytes']/s['requests']), 'B/req h2d', 'enc', round(s['encode_s'],3), 's', s.get('split_ms')))"
        k=$((k+1))
      done ;;
    bench)
      timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
      cat $O/bench.json ;;
    prof)
      (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/rocprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --latency-batches 0 --serve-threads 0 --configs-requests 0 --no-reload --parity-sample 0 --no-submit-to-results) > $O/rocprof_bench.json 2> $O/rocprof.err || { echo "rocprof failed"; tail -20 $O/rocprof.err; exit 1; }
      find $O/rocprof -name "*kernel_stats.csv" -exec head -12 {} \; ;;
    pmc)
      bash tools/pmc_kernels.sh $TAG/pmc || exit 1 ;;
    pmcb)
      # memory-pipeline busy / stall counters per kernel (each pass its own run, within the per-block
      # limits: TA 2, TD 2, TCP 4, TCC 4, GRBM 2)
      P=$GRAFT_REPO_ROOT/$O/pmcb
      mkdir -p $P
      ARGS="--steps 3 --warmup 1 --no-cpu-baseline --latency-batches 0 --parity-sample 0 --no-reload --serve-threads 0 --configs-requests 0 --no-submit-to-results ${BENCH_ARGS}"
      for pass in "ta:TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum GRBM_GUI_ACTIVE" \
                  "tcp:TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
                  "tcc:TCC_HIT_sum TCC_MISS_sum TCC_TAG_STALL_sum TCC_BUSY_sum" ; do
        name=${pass%%:*}; ctrs=${pass#*:}
        (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d $P/$name -o run -- python3 $GRAFT_REPO_ROOT/bench.py $ARGS) > $P/$name.log 2>&1 || { echo "pass $name failed"; tail -20 $P/$name.log; exit 1; }
      done
      for K in cedar_scan_kernel "cedar_probe_kernel<8u, 32u" "cedar_probe_kernel<8u, 64u" "cedar_probe_kernel<64u, 1024u"; do
        echo "== $K"; PMC_KERNEL="$K" python3 tools/pmc_summary.py $P
      done > $P/summary.txt; cat $P/summary.txt ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
