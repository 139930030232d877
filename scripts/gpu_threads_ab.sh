#!/bin/bash
# Headline (RTSP, 32 x 1080p H.264, 100 steps) at 13 / 15 / 16 host parse threads, alternated on
# one box (the default on a 16-CPU share is 15).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-threadsab}; mkdir -p "$O"
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 100 --warmup 10 --latency-samples 0 --clients 0 "$@" > "$O/$n.json" 2> "$O/$n.err" \
    || { echo "$n failed"; tail -20 "$O/$n.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d.get('frames_dropped'), d.get('parse_threads_per_rank'))"
}
for i in 1 2; do
  for t in 15 13 16; do run t${t}_$i --threads $t; done
done
