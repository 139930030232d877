#!/bin/bash
# Round 6 first box: GPU tests + smoke, the driver's command once, and the parse cost per CABAC bin
# at 1080p vs a smaller picture at 1 and 15 parse threads (does the per-thread cost at full load
# come from the working set (MB state + records per picture) or from sharing the cores?).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r6a}
mkdir -p "$O"
echo "[a] GPU tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1 || { echo "GPU tests failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -3 "$O/pytest_gpu.log"
echo "[a] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
  || { echo "smoke failed"; tail -30 "$O/smoke.log"; exit 1; }
echo "[a] driver command"
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/driver_1.json" 2> "$O/driver_1.err" \
  || { echo "bench failed"; tail -30 "$O/driver_1.err"; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print({k: d.get(k) for k in ('value','ms_per_step','frames_dropped','p50_latency_ms','p99_latency_ms','rank0_gpu_kernel_ms_per_step')})" "$O/driver_1.json"
echo "[a] parse cost vs resolution"
for args in "--threads 1 --cams 4" "--threads 15 --cams 32" "--threads 1 --cams 4 --width 960 --height 544" "--threads 15 --cams 32 --width 960 --height 544"; do
  timeout -k 10 300 python -u tools/parse_ab.py --reps 3 $args 2>&1 | tail -1 | tee -a "$O/parse_res.log"
done
echo "[a] done"
