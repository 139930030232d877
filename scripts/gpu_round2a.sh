#!/bin/bash
# Round-2 checkpoint: GPU tests (incl. the 1-rank RCCL test) + the honest 1-GPU bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/bench.log 2>&1; rc=$?
tail -2 gpurun_out/bench.log; echo "bench rc=$rc"
