#!/bin/bash
# Parse-thread / pack-thread sweep of the default bench after the locality changes.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for cfg in "14 4" "15 4" "16 4" "14 2" "12 4"; do
  set -- $cfg
  timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 --threads $1 --pack-threads $2 --latency-samples 0 > gpurun_out/sw_$1_$2.json 2> gpurun_out/sw_$1_$2.err || { echo "sweep $cfg failed"; tail -20 gpurun_out/sw_$1_$2.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/sw_$1_$2.json')); print('threads=$1 pack=$2', d['value'], d['ms_per_step'], d['rank0_parse_wait_ms_per_step'])"
done
