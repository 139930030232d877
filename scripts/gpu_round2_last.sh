#!/bin/bash
# Last check of the tree as the driver will run it: GPU suite, smoke, default bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_last.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/pytest_gpu_last.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_last.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_last.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke_last.log; exit 1; }
echo smoke ok
timeout -k 10 300 python -u bench.py > gpurun_out/bench_last.json 2> gpurun_out/bench_last.err || { echo "bench failed"; tail -30 gpurun_out/bench_last.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_last.json')); print('default', d['value'], d['ms_per_step'], d['frames_dropped'])"
