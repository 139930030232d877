#!/bin/bash
# HEVC GPU reconstruction: bit-exact tests first, then the rest of the GPU suite, then the coded
# H.265 benches (1080p x 32, 4K x 8) and a kernel-stats profile of the 1080p one.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hevc.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_hevc.log 2>&1 || { echo "hevc gpu tests failed"; tail -60 gpurun_out/pytest_gpu_hevc.log; exit 1; }
tail -5 gpurun_out/pytest_gpu_hevc.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_all2.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/pytest_gpu_all2.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_all2.log
timeout -k 10 400 python -u bench.py --codec h265 --steps 60 --warmup 5 --latency-samples 0 > gpurun_out/bench_h265_1080p_gpu.json 2> gpurun_out/bench_h265_1080p_gpu.err || { echo "bench h265 1080p failed"; tail -30 gpurun_out/bench_h265_1080p_gpu.err; exit 1; }
cat gpurun_out/bench_h265_1080p_gpu.json
timeout -k 10 400 python -u bench.py --codec h265 --width 3840 --height 2160 --cams-per-gpu 8 --steps 40 --warmup 5 --gop 30 --latency-samples 0 > gpurun_out/bench_h265_4k_gpu.json 2> gpurun_out/bench_h265_4k_gpu.err || { echo "bench h265 4k failed"; tail -30 gpurun_out/bench_h265_4k_gpu.err; exit 1; }
cat gpurun_out/bench_h265_4k_gpu.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_h265" -o run -- python3 "$R/bench.py" --codec h265 --steps 30 --warmup 3 --latency-samples 0 > "$R/gpurun_out/prof_h265.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_h265.log"; exit 1; }
echo done
