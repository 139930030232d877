#!/bin/bash
# Host parse cost on the GPU box's CPU (High CABAC 1080p): single-thread parse bench and the
# replay bench's parse pool at 1/7/14/16 threads; then the default bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
nproc; grep -m1 "model name" /proc/cpuinfo; cat /sys/fs/cgroup/cpu.max 2>/dev/null
timeout -k 10 200 ./tools/bin/parse_bench high 30 3 8 > gpurun_out/parse_bench_high.log 2>&1 || { echo "parse_bench failed"; cat gpurun_out/parse_bench_high.log; exit 1; }
cat gpurun_out/parse_bench_high.log
PROFILE=high timeout -k 10 300 python -u scripts/parse_scaling.py 32 1 7 14 16 > gpurun_out/parse_scaling_high.log 2>&1 || { echo "parse scaling failed"; tail -30 gpurun_out/parse_scaling_high.log; exit 1; }
cat gpurun_out/parse_scaling_high.log
timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed"; tail -30 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
