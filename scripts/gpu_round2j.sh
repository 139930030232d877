#!/bin/bash
# Round-end rehearsal: the whole GPU suite, smoke(), and the default bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_all3.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/pytest_gpu_all3.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_all3.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 500 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed"; tail -30 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
