#!/bin/bash
# Session-end validation: GPU suite, smoke, default bench x3 (spread), rocprofv3 kernel stats of
# the default bench, RTSP farm bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/pytest_gpu_final.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_final.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke_final.log; exit 1; }
echo smoke ok
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py > gpurun_out/bench_final_$i.json 2> gpurun_out/bench_final_$i.err || { echo "bench failed"; tail -30 gpurun_out/bench_final_$i.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_final_$i.json')); print('default', d['value'], d['steps'], d['ms_per_step'], d['p50_latency_ms'], d['frames_dropped'])"
done
timeout -k 10 400 python -u bench.py --source rtsp --steps 150 --warmup 10 > gpurun_out/bench_final_rtsp.json 2> gpurun_out/bench_final_rtsp.err || { echo "rtsp failed"; tail -30 gpurun_out/bench_final_rtsp.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_final_rtsp.json')); print('rtsp', d['value'], d['frames_dropped'])"
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o run -- python3 bench.py --steps 300 --warmup 30 > gpurun_out/bench_final_prof.json 2> gpurun_out/bench_final_prof.err || { echo "prof failed"; tail -30 gpurun_out/bench_final_prof.err; exit 1; }
echo prof ok
