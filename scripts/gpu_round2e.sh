#!/bin/bash
# Full GPU test suite (incl. the general HEVC path), then the 1-GPU headline bench and a
# rocprofv3 kernel-stats pass over a short bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_all.log 2>&1 || { echo "gpu tests failed"; tail -60 gpurun_out/pytest_gpu_all.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_all.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_high.json 2> gpurun_out/bench_high.err || { echo "bench high failed"; tail -30 gpurun_out/bench_high.err; exit 1; }
cat gpurun_out/bench_high.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_e" -o run -- python3 "$R/bench.py" --steps 40 --warmup 5 > "$R/gpurun_out/prof_e.log" 2>&1 || { echo "rocprof failed"; tail -30 "$R/gpurun_out/prof_e.log"; exit 1; }
find "$R/gpurun_out/prof_e" -name "*kernel_stats.csv" | head -3
