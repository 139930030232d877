#!/bin/bash
# End-of-round record on one box: a long headline run (stability: drops, errors over ~3000
# steps), BASELINE config 5 as one workload (8 x 4K H.265 + RTMP pass-through + annotation
# upload) and config 3 (keyframe-only), each with the out-of-process latency clients.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-finalrec}; mkdir -p "$O"
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; tail -20 "$O/$n.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d.get('frames_dropped'), d.get('decode_errors'), d.get('p50_latency_ms'), d.get('p99_latency_ms'), d.get('rank0_gpu_kernel_ms_per_step'))"
}
run headline_3000 --steps 3000 --warmup 30
run cfg5_4k_h265_rtmp_annotate --codec h265 --width 3840 --height 2160 --cams-per-gpu 8 --rtmp --annotate --steps 60 --warmup 8
run cfg3_keyframe_only --keyframe-only --steps 60 --warmup 8
