#!/bin/bash
# In-situ host profiles of the replay parse pool on the box CPU: 1 thread and 14 threads.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
PROFILE=high timeout -k 10 300 python -u tools/hostprof_parse.py gpurun_out/hostprof_t14.txt 14 32 300 || exit 1
PROFILE=high timeout -k 10 300 python -u tools/hostprof_parse.py gpurun_out/hostprof_t1.txt 1 32 20 || exit 1
PROFILE=high timeout -k 10 300 python -u scripts/parse_scaling.py 32 14 || exit 1
timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed"; tail -30 gpurun_out/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print(d['value'], d['ms_per_step'], d['rank0_host_parse_ms_per_step'], d['frames_dropped'])"
