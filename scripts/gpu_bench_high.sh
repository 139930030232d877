#!/bin/bash
# 1-GPU headline bench (High profile CABAC IBBP) + Baseline comparison + kernel stats.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/bench_high.json 2> gpurun_out/bench_high.err || { echo "bench high failed"; tail -30 gpurun_out/bench_high.err; exit 1; }
cat gpurun_out/bench_high.json
timeout -k 10 300 python -u bench.py --profile baseline --steps 150 --latency-samples 0 > gpurun_out/bench_baseline.json 2> gpurun_out/bench_baseline.err || { echo "bench baseline failed"; tail -30 gpurun_out/bench_baseline.err; exit 1; }
cat gpurun_out/bench_baseline.json
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_high -o run -- python3 bench.py --steps 100 --warmup 20 --latency-samples 0 > gpurun_out/prof_high.log 2>&1 || { echo "rocprof failed"; tail -30 gpurun_out/prof_high.log; exit 1; }
find gpurun_out/prof_high -name "*stats*" | head
