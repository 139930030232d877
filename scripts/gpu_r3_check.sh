#!/bin/bash
# Round-3 GPU check in one gpurun call: GPU tests, smoke, the driver's bench config, then an
# A/B of the H.265 intra transform-block schedules (per level / queue windows of k levels).
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
O=gpurun_out/${TAG:-r3s2}
mkdir -p "$O"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  echo "[check] pytest -m gpu"
  timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
    || { echo "pytest failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
  tail -2 "$O/pytest_gpu.log"
  echo "[check] smoke"
  timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
    || { echo "smoke failed"; tail -20 "$O/smoke.log"; exit 1; }
  tail -1 "$O/smoke.log"
fi
run() {  # name, env assignment ("-" for none), bench args...
  local n=$1 e=$2; shift 2
  if [ "$e" = "-" ]; then
    timeout -k 10 400 python -u bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; tail -30 "$O/$n.err"; exit 1; }
  else
    env "$e" timeout -k 10 400 python -u bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; tail -30 "$O/$n.err"; exit 1; }
  fi
  python -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d.get('frames_dropped'), d.get('rank0_gpu_kernel_ms_per_step'), d.get('p50_latency_ms'))"
}
if [ "${SKIP_DRIVER:-0}" != "1" ]; then
  echo "[check] driver bench config"
  run bench_driver - --gpus 1 --steps 20 --warmup 5
fi
if [ "${KF:-1}" = "1" ]; then
  echo "[check] keyframe-only (BASELINE config 3)"
  run kf_only - --keyframe-only --steps 60 --warmup 8
  run kf_only_phases VEP_AVC_PROF=1 --keyframe-only --steps 30 --warmup 5 --latency-samples 0 --clients 0
fi
if [ "${HEVC_AB:-1}" = "1" ]; then
  echo "[check] H.265 intra TU schedules (replay, decode path only)"
  for w in ${W1080:-0 8 4 16}; do
    run h265_1080p_w$w VEP_HEVC_TU_WINDOW=$w --codec h265 --source replay --steps 60 --warmup 8 --latency-samples 0 --clients 0
  done
  for w in ${W4K:-0 8}; do
    run h265_4k_w$w VEP_HEVC_TU_WINDOW=$w --codec h265 --source replay --width 3840 --height 2160 --cams-per-gpu 8 --steps 40 --warmup 6 --latency-samples 0 --clients 0
  done
fi
echo "[check] done"
