#!/bin/bash
# Round 4, second check: GPU tests of the new paths, the H.265 intra schedules under the SQ
# counter pass (which of them drop pictures when rocprofv3 instruments dispatches), kernel stats,
# then the serving benchmark. Every GPU step has its own time limit; stop at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4b}
mkdir -p "$O"
echo "[b] pytest (new GPU paths)"
timeout -k 10 400 python -u -m pytest tests/test_consumer_snapshot.py tests/test_gpu_rccl.py tests/test_gpu_hevc.py \
  -m gpu -x -v --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest.log"; exit 1; }
grep -E "PASS|FAIL|SKIP" "$O/pytest.log" | sed 's/ *\[.*//' | tail -20
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
pmc() {  # name, env assignment, program...
  local n=$1 e=$2; shift 2
  local s=$(date +%s)
  env $e timeout -s KILL 200 rocprofv3 --pmc $P1 -d "$O/pmc_$n" -o pmc -- "$@" > "$O/pmc_$n.log" 2>&1
  local rc=$?
  echo "pmc $n rc=$rc secs=$(( $(date +%s) - s )) $(grep -o '"frames_dropped": [0-9]*' "$O/pmc_$n.log") $(grep -oE '[0-9]+ (passed|failed)' "$O/pmc_$n.log" | tr '\n' ' ')"
  rm -rf "$O/pmc_$n"
  [ $rc -eq 0 ] || [ $rc -eq 3 ] || [ $rc -eq 1 ] || exit 1
}
B="$R/bench.py --codec h265 --source replay --steps 12 --warmup 3 --latency-samples 0 --clients 0"
# bit-exactness under the counter pass: does instrumented dispatch keep a stream's kernels ordered?
pmc levels_exact VEP_HEVC_TU_WINDOW=0 python3 -m pytest "$R/tests/test_gpu_hevc.py" -m gpu -k "1080p" -x -q -p no:cacheprovider
pmc w8_exact VEP_HEVC_TU_WINDOW=8 python3 -m pytest "$R/tests/test_gpu_hevc.py" -m gpu -k "1080p" -x -q -p no:cacheprovider
pmc round VEP_HEVC_TU_WINDOW=65536 python3 $B
pmc queue VEP_HEVC_TU_QUEUE=1 python3 $B
pmc w8 VEP_HEVC_TU_WINDOW=8 python3 $B
cd "$R"
kt() {  # name, window, bench args
  local n=$1 w=$2; shift 2
  cd /tmp
  VEP_HEVC_TU_WINDOW=$w timeout -k 10 200 rocprofv3 --kernel-trace -d "$O/kt_$n" -o kt -- python3 "$R/bench.py" \
    --codec h265 --source replay --latency-samples 0 --clients 0 "$@" > "$O/kt_$n.log" 2>&1 \
    || { echo "kernel trace $n failed"; tail -20 "$O/kt_$n.log"; exit 1; }
  cd "$R"
  python3 tools/rocpd_kernel_stats.py "$O/kt_$n" > "$O/kernel_stats_$n.csv"
  rm -rf "$O/kt_$n"
  echo "== $n"; head -8 "$O/kernel_stats_$n.csv"
}
kt 1080p_w0 0 --steps 30 --warmup 5
kt 1080p_round 65536 --steps 30 --warmup 5
kt 1080p_pic -1 --steps 30 --warmup 5
run() {  # name, window, bench args...
  local n=$1 w=$2; shift 2
  VEP_HEVC_TU_WINDOW=$w timeout -k 10 300 python -u bench.py --codec h265 --source replay --latency-samples 0 \
    --clients 0 "$@" > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; tail -30 "$O/$n.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d.get('frames_dropped'), d.get('rank0_gpu_kernel_ms_per_step'))"
}
run h265_1080p_round 65536 --steps 60 --warmup 8
run h265_4k_round 65536 --width 3840 --height 2160 --cams-per-gpu 8 --steps 40 --warmup 6
echo "[b] serving"
TAG=${TAG:-r4b}/serve bash scripts/gpu_r4_serving.sh
echo "[b] done"
