#!/bin/bash
# Live H.265 RTSP on gfx950 + the integration file.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_integration.py tests/test_gpu_hevc.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_live_hevc.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/pytest_gpu_live_hevc.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_gpu_live_hevc.log | tail -12
