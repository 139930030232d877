#!/bin/bash
# GPU check of the Main/High encoder streams (B pictures, CABAC, 8x8, weighted) on the kernels.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_avc_high.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_avc_high.log 2>&1 || { echo "avc high gpu tests failed"; tail -60 gpurun_out/pytest_gpu_avc_high.log; exit 1; }
tail -8 gpurun_out/pytest_gpu_avc_high.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_avc.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_avc.log 2>&1 || { echo "avc gpu tests failed"; tail -60 gpurun_out/pytest_gpu_avc.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_avc.log
