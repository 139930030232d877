#!/bin/bash
# Round 4: BASELINE config 5 (8 x 4K H.265 per GPU, RTMP passthrough, annotate, 8 clients) for
# 300 steps with 8 slices per picture (parallel slice parse) vs 1 slice, at the default parse
# share or (PART=t7) at 7 parse threads; and (PART=h264) the H.264 headline with 4 slices per
# picture (parallel H.264 slice parse) vs 1.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4f}
mkdir -p "$O"
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 ${LIMIT:-500} python -u bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; tail -30 "$O/$n.err"; exit 1; }
  python - "$O/$n.json" "$n" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], "dropped", d.get("frames_dropped"), "gpu_ms", d.get("rank0_gpu_kernel_ms_per_step"),
      "p50", d.get("p50_latency_ms"), "p99", d.get("p99_latency_ms"), "published", d.get("frames_published"),
      "decoded", d.get("frames_decoded"), "threads", d.get("parse_threads"), flush=True)
PY
}
C5="--codec h265 --width 3840 --height 2160 --cams-per-gpu 8 --rtmp --annotate --steps 300 --warmup 20 --clients 8"
case "${PART:-c5}" in
  c5)
    run cfg5_slices8 $C5 --slices 8
    run cfg5_slices1 $C5 --slices 1 ;;
  t7)
    run cfg5_slices8_t7 $C5 --slices 8 --threads 7
    run cfg5_slices1_t7 $C5 --slices 1 --threads 7 ;;
  h264)
    run h264_slices4 --gpus 1 --steps 200 --warmup 20 --slices 4
    run h264_slices1 --gpus 1 --steps 200 --warmup 20 --slices 1 ;;
esac
echo "[f] done"
