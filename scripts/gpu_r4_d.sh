#!/bin/bash
# Round 4, fourth check: the full GPU suite + smoke with the new defaults (persistent ticket
# queue for H.265 intra blocks), the SQ counter pass and kernel stats of the default schedule,
# BASELINE config 5 with 1 vs 8 slices (and at a 7-thread parse share), and the driver's
# headline command. Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4d}
mkdir -p "$O"
if [ "${TESTS:-1}" = "1" ]; then
  echo "[d] pytest -m gpu"
  timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
    || { echo "pytest failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
  tail -2 "$O/pytest_gpu.log"
  echo "[d] smoke"
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
    || { echo "smoke failed"; tail -20 "$O/smoke.log"; exit 1; }
  tail -3 "$O/smoke.log"
fi
run() {  # name, env assignments (or -), bench args...
  local n=$1 e=$2; shift 2
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 ${LIMIT:-400} python -u bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; tail -30 "$O/$n.err"; exit 1; }
  python - "$O/$n.json" "$n" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], "dropped", d.get("frames_dropped"), "gpu_ms", d.get("rank0_gpu_kernel_ms_per_step"),
      "p50", d.get("p50_latency_ms"), "p99", d.get("p99_latency_ms"), "skipped", d.get("access_units_skipped"),
      "published", d.get("frames_published"), "decoded", d.get("frames_decoded"))
PY
}
if [ "${PROF:-1}" = "1" ]; then
  cd /tmp && export TMPDIR=/tmp
  P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
  timeout -s KILL 200 rocprofv3 --pmc $P1 -d "$O/pmc_default" -o pmc -- python3 "$R/bench.py" --codec h265 --source replay \
    --steps 12 --warmup 3 --latency-samples 0 --clients 0 > "$O/pmc_default.log" 2>&1
  rc=$?; echo "pmc default (1080p) rc=$rc $(grep -o '"frames_dropped": [0-9]*' "$O/pmc_default.log")"
  [ $rc -eq 0 ] || [ $rc -eq 3 ] || exit 1
  python3 "$R/tools/rocpd_pmc_summary.py" $(find "$O/pmc_default" -name "*.db") > "$O/pmc_default_summary.txt" 2>&1 || true
  rm -rf "$O/pmc_default"
  for shape in "1080p:" "4k:--width 3840 --height 2160 --cams-per-gpu 8"; do
    n=${shape%%:*}; args=${shape#*:}
    timeout -k 10 200 rocprofv3 --kernel-trace -d "$O/kt_$n" -o kt -- python3 "$R/bench.py" --codec h265 --source replay \
      --steps 30 --warmup 5 --latency-samples 0 --clients 0 $args > "$O/kt_$n.log" 2>&1 || { echo "kt $n failed"; tail -20 "$O/kt_$n.log"; exit 1; }
    python3 "$R/tools/rocpd_kernel_stats.py" "$O/kt_$n" > "$O/kernel_stats_h265_${n}_default.csv"
    rm -rf "$O/kt_$n"
    echo "== $n"; head -5 "$O/kernel_stats_h265_${n}_default.csv" | cut -c1-160
  done
  cd "$R"
fi
if [ "${CFG5:-1}" = "1" ]; then
  C5="--codec h265 --width 3840 --height 2160 --cams-per-gpu 8 --rtmp --annotate --steps 300 --warmup 20 --clients 8"
  LIMIT=600 run cfg5_slices8 - $C5 --slices 8
  LIMIT=600 run cfg5_slices1 - $C5 --slices 1
  LIMIT=600 run cfg5_slices8_t7 - $C5 --slices 8 --threads 7
  LIMIT=600 run cfg5_slices1_t7 - $C5 --slices 1 --threads 7
fi
if [ "${HEADLINE:-1}" = "1" ]; then
  run headline_driver - --gpus 1 --steps 20 --warmup 5
fi
echo "[d] done"
