#!/bin/bash
# Diagnose: torch HIP init after native HEVC GPU tests in one process; then the benches.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_integration.py tests/test_gpu_hevc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_order1.log 2>&1; echo "order integration,hevc rc=$?"; tail -2 gpurun_out/pytest_gpu_order1.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_hevc.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_order2.log 2>&1; echo "order hevc,kernels rc=$?"; tail -2 gpurun_out/pytest_gpu_order2.log
timeout -k 10 400 python -u bench.py --codec h265 --steps 60 --warmup 5 --latency-samples 0 > gpurun_out/bench_h265_1080p_gpu2.json 2> gpurun_out/bench_h265_1080p_gpu2.err || { echo "bench h265 1080p failed"; tail -30 gpurun_out/bench_h265_1080p_gpu2.err; exit 1; }
cat gpurun_out/bench_h265_1080p_gpu2.json
timeout -k 10 400 python -u bench.py --codec h265 --width 3840 --height 2160 --cams-per-gpu 8 --steps 40 --warmup 5 --gop 30 > gpurun_out/bench_h265_4k_gpu2.json 2> gpurun_out/bench_h265_4k_gpu2.err || { echo "bench h265 4k failed"; tail -30 gpurun_out/bench_h265_4k_gpu2.err; exit 1; }
cat gpurun_out/bench_h265_4k_gpu2.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_h265b" -o run -- python3 "$R/bench.py" --codec h265 --steps 30 --warmup 3 --latency-samples 0 > "$R/gpurun_out/prof_h265b.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_h265b.log"; exit 1; }
echo done
