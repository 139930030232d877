#!/bin/bash
# HEVC GPU tests + 1080p/4K benches + kernel stats after the parallel intra-reference change.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hevc.py tests/test_gpu_integration.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_hevc2.log 2>&1 || { echo "hevc gpu tests failed"; tail -60 gpurun_out/pytest_gpu_hevc2.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_hevc2.log
timeout -k 10 400 python -u bench.py --codec h265 --steps 60 --warmup 5 --latency-samples 0 > gpurun_out/bench_h265_1080p_gpu2.json 2> gpurun_out/bench_h265_1080p_gpu2.err || { echo "bench h265 1080p failed"; tail -30 gpurun_out/bench_h265_1080p_gpu2.err; exit 1; }
cat gpurun_out/bench_h265_1080p_gpu2.json
timeout -k 10 400 python -u bench.py --codec h265 --width 3840 --height 2160 --cams-per-gpu 8 --steps 40 --warmup 5 --gop 30 > gpurun_out/bench_h265_4k_gpu2.json 2> gpurun_out/bench_h265_4k_gpu2.err || { echo "bench h265 4k failed"; tail -30 gpurun_out/bench_h265_4k_gpu2.err; exit 1; }
cat gpurun_out/bench_h265_4k_gpu2.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/prof_h265b" -o run -- python3 "$R/bench.py" --codec h265 --steps 30 --warmup 3 --latency-samples 0 > "$R/gpurun_out/prof_h265b.log" 2>&1 || { echo "rocprof failed"; tail -20 "$R/gpurun_out/prof_h265b.log"; exit 1; }
echo done
