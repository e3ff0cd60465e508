set -o pipefail
mkdir -p gpurun_out/ab_seg8
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python -u bench.py --no-cpu-baseline --latency-batches 0 --serve-threads 0 --configs-requests 0 --no-reload --parity-sample 1024 --steps 5 > gpurun_out/ab_seg8/$tag.json 2> gpurun_out/ab_seg8/$tag.err || { echo "$tag failed"; tail -5 gpurun_out/ab_seg8/$tag.err; return 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/ab_seg8/$tag.json')); print('$tag', round(d['value']/1e6,1), 'M/s ms', round(d['roofline']['kernel_ms'],3), 'mism', d['parity_sample']['mismatches'])"; }
run s16 CEDARGPU_PROBE_SEG=16 && run s8_o3_w1 CEDARGPU_PROBE_SEG=8 CEDARGPU_PROBE_OCC=3 CEDARGPU_PROBE_WPB=1 && run s8_o3_w4 CEDARGPU_PROBE_SEG=8 CEDARGPU_PROBE_OCC=3 CEDARGPU_PROBE_WPB=4 && run s8_o4_w1 CEDARGPU_PROBE_SEG=8 CEDARGPU_PROBE_OCC=4
