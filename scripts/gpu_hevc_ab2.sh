#!/bin/bash
# HEVC parse A/B (pointer hoisting) on the box CPU, then the H.265 benches.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for i in 1 2 3; do
  for b in hb_a hb_b; do echo -n "$b "; timeout -k 5 120 taskset -c 3 tools/bin/$b 1920 1080 16 2 25 records || exit 1; done
done
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/$n.json 2> gpurun_out/$n.err || { echo "$n failed"; tail -30 gpurun_out/$n.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$n.json')); print('$n', d['value'], d['ms_per_step'], d.get('frames_dropped'))"
}
run bench_h265_4k --codec h265 --width 3840 --height 2160 --cams-per-gpu 8 --steps 60 --warmup 6
run bench_h265_1080p --codec h265 --steps 100 --warmup 10
