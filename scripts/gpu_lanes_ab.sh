#!/bin/bash
# Headline (RTSP, 32 x 1080p H.264, 100 steps) at 2 / 3 / 4 GPU lanes and 3 / 4 stages per
# lane, alternated on one box (the defaults are 3 lanes x 3 stages).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-lanesab}; mkdir -p "$O"
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --latency-samples 0 --clients 0 "$@" > "$O/$n.json" 2> "$O/$n.err" \
    || { echo "$n failed"; tail -20 "$O/$n.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d.get('frames_dropped'), d.get('rank0_gpu_kernel_ms_per_step'), d.get('gpu_lanes'), d.get('gpu_stages'))"
}
for i in 1 2; do
  run l3s3_$i --lanes 3 --stages 3
  run l2s3_$i --lanes 2 --stages 3
  run l4s3_$i --lanes 4 --stages 3
  run l3s4_$i --lanes 3 --stages 4
done
