#!/bin/bash
# After the parse-locality changes: GPU suite, smoke, default bench, live RTSP farm bench,
# H.265 1080p x32 and 4K x8.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_all6.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/pytest_gpu_all6.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_all6.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/$n.json 2> gpurun_out/$n.err || { echo "$n failed"; tail -30 gpurun_out/$n.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$n.json')); print('$n', d['value'], d['ms_per_step'], d.get('rank0_host_parse_ms_per_step'), d.get('frames_dropped'), d.get('p50_latency_ms'))"
}
run bench_default --steps 300 --warmup 30
run bench_rtsp --source rtsp --steps 150 --warmup 10
run bench_h265_1080p --codec h265 --steps 100 --warmup 10
run bench_h265_4k --codec h265 --width 3840 --height 2160 --cams-per-gpu 8 --steps 60 --warmup 6
