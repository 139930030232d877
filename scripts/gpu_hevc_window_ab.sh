#!/bin/bash
# H.265 intra TU schedule, end to end on one box: per-level launches (VEP_HEVC_TU_WINDOW=0) vs
# queue windows of 8 levels, alternated, 32 x 1080p and 8 x 4K through the RTSP farm.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-hwab}; mkdir -p "$O"
run() {  # name, window, bench args...
  local n=$1 w=$2; shift 2
  VEP_HEVC_TU_WINDOW=$w timeout -k 10 300 python -u bench.py --codec h265 --latency-samples 0 --clients 0 "$@" \
    > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; tail -20 "$O/$n.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d.get('rank0_gpu_kernel_ms_per_step'))"
}
for i in 1 2; do
  for w in 0 8; do run h265_1080p_w${w}_$i $w --steps 80 --warmup 8; done
  for w in 0 8; do run h265_4k_w${w}_$i $w --width 3840 --height 2160 --cams-per-gpu 8 --steps 50 --warmup 6; done
done
