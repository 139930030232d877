#!/bin/bash
# GPU check of the High-profile kernels: AVC GPU tests first (bit-exact vs CPU), then the rest.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_avc.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_avc.log 2>&1 || { echo "avc gpu tests failed"; tail -60 gpurun_out/pytest_gpu_avc.log; exit 1; }
tail -5 gpurun_out/pytest_gpu_avc.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
