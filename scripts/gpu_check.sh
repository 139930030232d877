#!/bin/bash
# One gpurun call: GPU tests, smoke, 1-GPU bench, rocprofv3 kernel stats + roctx marker trace.
# Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
STEPS=${STEPS:-300}
echo "[gpu_check] pytest -m gpu"
timeout -k 10 420 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
echo "[gpu_check] smoke"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
echo "[gpu_check] bench"
timeout -k 10 300 python bench.py --steps $STEPS --warmup 30 > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench.log; exit 1; }
tail -1 gpurun_out/bench.log
echo "[gpu_check] rocprofv3 kernel stats"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof" -o run -- python3 "$R/bench.py" --steps 30 --warmup 5 --latency-samples 0 > "$R/gpurun_out/prof.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof.log"; exit 1; }
echo "[gpu_check] rocprofv3 roctx marker trace (host stages next to kernels)"
export VEP_ROCTX=1
cd /tmp && timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d "$R/gpurun_out/prof_markers" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --latency-samples 0 > "$R/gpurun_out/prof_markers.log" 2>&1 || { echo "marker trace failed"; tail -20 "$R/gpurun_out/prof_markers.log"; exit 1; }
unset VEP_ROCTX
find "$R/gpurun_out/prof" "$R/gpurun_out/prof_markers" -name "*.csv" | head
echo "[gpu_check] wavefront kernel phase cycles (VEP_AVC_PROF=1)"
cd "$R" && VEP_AVC_PROF=1 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --latency-samples 5 > gpurun_out/bench_phases.json 2>&1 || { echo "phase profile failed"; tail -20 gpurun_out/bench_phases.json; exit 1; }
if [ "${PMC:-0}" = "1" ]; then
  # hardware counters: one pass of <= 8 SQ counters per run, each run killed after 150 s
  echo "[gpu_check] rocprofv3 --pmc (2 passes)"
  cd /tmp
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
    -d "$R/gpurun_out/pmc1" -o pmc -- python3 "$R/bench.py" --cams-per-gpu 8 --steps 10 --warmup 2 --latency-samples 0 > "$R/gpurun_out/pmc1.log" 2>&1 || { echo "pmc pass 1 failed"; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM \
    -d "$R/gpurun_out/pmc2" -o pmc -- python3 "$R/bench.py" --cams-per-gpu 8 --steps 10 --warmup 2 --latency-samples 0 > "$R/gpurun_out/pmc2.log" 2>&1 || { echo "pmc pass 2 failed"; exit 1; }
fi
echo "[gpu_check] done"
