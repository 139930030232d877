#!/bin/bash
# Round 5 check: GPU tests + smoke, the driver's 1-GPU command three times (run-to-run spread of
# the GOP-sized steps), then rocprofv3 kernel statistics of the headline. RUNS / PROF / TESTS
# select the parts (default: all).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r5check}
mkdir -p "$O"
if [ "${TESTS:-1}" = 1 ]; then
  echo "[c] GPU tests"
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    > "$O/pytest_gpu.log" 2>&1 || { echo "GPU tests failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
  tail -3 "$O/pytest_gpu.log"
  echo "[c] smoke"
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
    || { echo "smoke failed"; tail -30 "$O/smoke.log"; exit 1; }
  tail -2 "$O/smoke.log"
fi
for i in $(seq 1 "${RUNS:-3}"); do
  echo "[c] driver command, run $i"
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 ${BENCH_ARGS:-} > "$O/driver_$i.json" 2> "$O/driver_$i.err" \
    || { echo "bench run $i failed"; tail -30 "$O/driver_$i.err"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print({k: d.get(k) for k in ('value','ms_per_step','frames_dropped','frames_shed','p50_latency_ms','p99_latency_ms','rank0_gpu_kernel_ms_per_step')})" "$O/driver_$i.json"
done
if [ "${PROF:-1}" = 1 ]; then
  echo "[c] rocprof headline"
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o headline --output-format csv -- python3 "$R/bench.py" \
    --steps 4 --warmup 1 --clients 0 --latency-samples 0 > "$O/prof.log" 2>&1 || { echo "rocprof failed"; tail -30 "$O/prof.log"; exit 1; }
  cd "$R"
  find "$O/prof" -name "*kernel_stats.csv" | head -3
fi
echo "[c] done"
