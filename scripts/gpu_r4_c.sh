#!/bin/bash
# Round 4, third check: H.265 intra TU schedules that pass the SQ counter pass (one ticketed
# launch per round, persistent queue at several sizes) against per-level launches; then BASELINE
# config 5 (8 x 4K H.265 + RTMP + annotate) with 1 vs 8 slices per picture (independent slices
# parsed in parallel), at the default and at a 7-thread parse share. Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4c}
mkdir -p "$O"
run() {  # name, env assignments (or -), bench args...
  local n=$1 e=$2; shift 2
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 ${LIMIT:-400} python -u bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; tail -30 "$O/$n.err"; exit 1; }
  python - "$O/$n.json" "$n" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], "dropped", d.get("frames_dropped"), "gpu_ms", d.get("rank0_gpu_kernel_ms_per_step"),
      "p50", d.get("p50_latency_ms"), "p99", d.get("p99_latency_ms"), "skipped", d.get("access_units_skipped"))
PY
}
H="--codec h265 --source replay --latency-samples 0 --clients 0"
if [ "${TU:-1}" = "1" ]; then
  for rep in 1 2; do
    run t1080_w0_$rep VEP_HEVC_TU_WINDOW=0 $H --steps 60 --warmup 8
    run t1080_round_$rep VEP_HEVC_TU_WINDOW=65536 $H --steps 60 --warmup 8
    for q in 64 128 512; do
      run t1080_q${q}_$rep "VEP_HEVC_TU_QUEUE=1 VEP_HEVC_TU_QUEUE_WGS=$q" $H --steps 60 --warmup 8
    done
  done
  run t4k_w0 VEP_HEVC_TU_WINDOW=0 $H --width 3840 --height 2160 --cams-per-gpu 8 --steps 40 --warmup 6
  run t4k_round VEP_HEVC_TU_WINDOW=65536 $H --width 3840 --height 2160 --cams-per-gpu 8 --steps 40 --warmup 6
  run t4k_q128 "VEP_HEVC_TU_QUEUE=1 VEP_HEVC_TU_QUEUE_WGS=128" $H --width 3840 --height 2160 --cams-per-gpu 8 --steps 40 --warmup 6
fi
if [ "${CFG5:-1}" = "1" ]; then
  C5="--codec h265 --width 3840 --height 2160 --cams-per-gpu 8 --rtmp --annotate --steps 300 --warmup 20 --clients 8"
  LIMIT=600 run cfg5_slices8 - $C5 --slices 8
  LIMIT=600 run cfg5_slices1 - $C5 --slices 1
  LIMIT=600 run cfg5_slices8_t7 - $C5 --slices 8 --threads 7
  LIMIT=600 run cfg5_slices1_t7 - $C5 --slices 1 --threads 7
fi
echo "[c] done"
