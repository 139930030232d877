#!/bin/bash
# VCN backend on gfx950 (librocdecode test double, HBM surfaces) + the whole GPU suite + smoke + bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_vcn_backend.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_vcn.log 2>&1 || { echo "vcn tests failed"; tail -60 gpurun_out/pytest_gpu_vcn.log; exit 1; }
grep -E "PASSED|FAILED|passed|failed" gpurun_out/pytest_gpu_vcn.log | tail -5
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_all4.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/pytest_gpu_all4.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_all4.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed"; tail -30 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
