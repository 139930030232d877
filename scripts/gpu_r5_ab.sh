#!/bin/bash
# Round 5 A/Bs on one box, alternated so box drift hits both sides:
#  PART=dbk  — H.264 deblocking: per-edge LDS lines (VEP_DBK_REGS=0, round 4) vs lines in VGPRs
#              (default), on the driver's headline command; GPU kernel ms per step and, in
#              VEP_AVC_PROF=1 runs, the wavefront phase cycles per MB.
#  PART=hevc — H.265 4K intra TU queue: fixed 256-cycle polls (VEP_HEVC_TU_NAP=1, round 4) vs
#              exponential backoff (default 16) vs per-level launches (VEP_HEVC_TU_WINDOW=0).
# Outputs gpurun_out/$TAG/*.json (+ .err), one summary line per run on stdout.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-r5ab}; mkdir -p "$O"
run() {  # name, env assignments..., --, bench args...
  local n=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done
  shift
  env "${envs[@]}" timeout -k 10 400 python -u bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" \
    || { echo "$n failed"; tail -20 "$O/$n.err"; exit 1; }
  python - "$O/$n.json" "$n" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keys = ("value", "ms_per_step", "rank0_gpu_kernel_ms_per_step", "frames_dropped", "dbk_cycles_per_mb",
        "intra_cycles_per_mb", "rank0_pictures_per_launch", "rank0_launches_merged", "p50_latency_ms",
        "p99_latency_ms")
print(sys.argv[2], {k: d.get(k) for k in keys if k in d})
PY
}
if [ "${PART:-dbk}" = dbk ]; then
  for i in 1 2; do
    for g in 0 1; do
      run dbk_regs${g}_$i VEP_DBK_REGS=$g -- --gpus 1 --steps 20 --warmup 5
      run dbk_regs${g}_prof_$i VEP_DBK_REGS=$g VEP_AVC_PROF=1 -- --gpus 1 --steps 10 --warmup 3 --clients 0 \
        --latency-samples 0
    done
  done
fi
if [ "${PART:-dbk}" = lanes ]; then  # lane launchers merging queued batches vs not vs round 4's launcher
  for i in 1 2; do
    for v in single:VEP_LANE_THREADS=0 merge:VEP_LANE_THREADS=1 nomerge:VEP_LANE_MERGE=0:VEP_LANE_THREADS=1; do
      IFS=: read -r nm e1 e2 <<< "$v"
      run lanes_${nm}_$i $e1 ${e2:-VEP_NOP=1} -- --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-}
    done
  done
fi
if [ "${PART:-dbk}" = hevc ]; then
  for i in 1 2; do
    for v in nap1:VEP_HEVC_TU_NAP=1 nap16:VEP_HEVC_TU_NAP=16 levels:VEP_HEVC_TU_WINDOW=0; do
      run h265_4k_${v%%:*}_$i "${v#*:}" -- --codec h265 --width 3840 --height 2160 --cams-per-gpu 8 \
        --steps ${STEPS:-40} --warmup 4 --latency-samples 0 --clients 0
    done
  done
fi
echo "[ab] done"
