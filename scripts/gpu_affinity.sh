#!/bin/bash
# Replay parse pool with cache-affine camera selection: parse-only scaling and the default bench x2.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
PROFILE=high timeout -k 10 300 python -u scripts/parse_scaling.py 32 14 16 || exit 1
for i in 1 2; do
timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 > gpurun_out/bench_default_$i.json 2> gpurun_out/bench_default_$i.err || { echo "bench failed"; tail -30 gpurun_out/bench_default_$i.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_default_$i.json')); print(d['value'], d['ms_per_step'], d['rank0_host_parse_ms_per_step'], d['rank0_parse_wait_ms_per_step'], d['frames_dropped'])"
done
