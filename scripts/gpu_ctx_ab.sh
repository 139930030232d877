#!/bin/bash
# A/B of the packed u16 CABAC context (b) against the u8 pair (a): H.264 High and H.265 parse,
# single thread on the box CPU; then the default bench with the packed context.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for i in 1 2 3; do
  for b in pb_a pb_b; do echo -n "$b "; timeout -k 5 120 taskset -c 3 tools/bin/$b high 30 3 | grep "best of" || exit 1; done
  for b in hb_a hb_b; do echo -n "$b "; timeout -k 5 120 taskset -c 3 tools/bin/$b 1920 1080 16 2 25 records || exit 1; done
done
timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed"; tail -30 gpurun_out/bench_default.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_default.json')); print('bench', d['value'], d['ms_per_step'], d['parse_threads_per_rank'], d['frames_dropped'])"
