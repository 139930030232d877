#!/bin/bash
# AVC GPU tests (High + Baseline streams) then the 1-GPU headline bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_avc_high.py tests/test_gpu_avc.py tests/test_gpu_integration.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_avc_all.log 2>&1 || { echo "avc gpu tests failed"; tail -60 gpurun_out/pytest_gpu_avc_all.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_avc_all.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_high.json 2> gpurun_out/bench_high.err || { echo "bench high failed"; tail -30 gpurun_out/bench_high.err; exit 1; }
cat gpurun_out/bench_high.json
timeout -k 10 400 python -u bench.py --source rtsp --steps 150 --warmup 10 > gpurun_out/bench_rtsp.json 2> gpurun_out/bench_rtsp.err || { echo "bench rtsp failed"; tail -30 gpurun_out/bench_rtsp.err; exit 1; }
cat gpurun_out/bench_rtsp.json
