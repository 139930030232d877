#!/bin/bash
# Round 4: H.265 intra transform-block schedules on one box.
#  1. GPU tests of the H.265 paths (every schedule bit-exact),
#  2. replay A/B: per-level launches (0), ticketed windows of 8 levels (8), one workgroup per
#     picture (-1), at 1080p (32 cameras) and 4K (8 cameras),
#  3. rocprofv3 SQ counter pass (the round-3 stall) over each queue schedule: frames dropped,
#  4. kernel stats of the picture schedule.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4hevc}
mkdir -p "$O"
echo "[hevc] pytest"
timeout -k 10 300 python -u -m pytest tests/test_gpu_hevc.py tests/test_gpu_hevc_tools.py -x -v --timeout 120 \
  --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.log"; exit 1; }
tail -1 "$O/pytest.log"
run() {  # name, window, bench args...
  local n=$1 w=$2; shift 2
  VEP_HEVC_TU_WINDOW=$w timeout -k 10 300 python -u bench.py --codec h265 --source replay --latency-samples 0 \
    --clients 0 "$@" > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; tail -30 "$O/$n.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d.get('frames_dropped'), d.get('rank0_gpu_kernel_ms_per_step'))"
}
for rep in 1 2; do
  for w in ${WS:--1 8 0}; do
    run h265_1080p_w${w}_$rep $w --steps 60 --warmup 8
  done
done
for w in ${WS:--1 8 0}; do
  run h265_4k_w$w $w --width 3840 --height 2160 --cams-per-gpu 8 --steps 40 --warmup 6
done
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
for w in -1 8; do
  s=$(date +%s)
  VEP_HEVC_TU_WINDOW=$w timeout -s KILL 200 rocprofv3 --pmc $P1 -d "$O/pmc_w$w" -o pmc -- python3 "$R/bench.py" \
    --codec h265 --source replay --steps 12 --warmup 3 --latency-samples 0 --clients 0 > "$O/pmc_w$w.log" 2>&1
  rc=$?
  echo "pmc window $w rc=$rc secs=$(( $(date +%s) - s )) $(grep -o '"frames_dropped": [0-9]*' "$O/pmc_w$w.log")"
  [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit 1
done
VEP_HEVC_TU_WINDOW=-1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$O/kt" -o kt -- python3 "$R/bench.py" \
  --codec h265 --source replay --steps 30 --warmup 5 --latency-samples 0 --clients 0 > "$O/kt.log" 2>&1 \
  || { echo "kernel trace failed"; tail -20 "$O/kt.log"; exit 1; }
find "$O/kt" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats_h265_1080p_picture.csv" \;
rm -rf "$O/kt" "$O"/pmc_w*/
echo "[hevc] done"
