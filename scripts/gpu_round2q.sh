#!/bin/bash
# GPU suite + smoke after the parse changes; keyframe-only RTSP bench with the sized ingest pool;
# rocprofv3 kernel stats of the H.265 1080p bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for i in 1 2 3; do
  for b in pb_base pb_v3 pb_zn4; do echo -n "$b "; timeout -k 5 120 taskset -c 3 tools/bin/$b high 30 3 | grep "best of" || exit 1; done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_all7.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/pytest_gpu_all7.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_all7.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log | cut -c1-80
timeout -k 10 300 python -u bench.py --source rtsp --keyframe-only --steps 20 --warmup 2 > gpurun_out/bench_keyframe_only.json 2> gpurun_out/bench_keyframe_only.err || { echo "keyframe bench failed"; tail -30 gpurun_out/bench_keyframe_only.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_keyframe_only.json')); print('kf', d['value'], d['access_units_per_s'], d['frames_decoded'], d['rank0_gpu_kernel_ms_per_step'])"
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_h265 -o run -- python3 bench.py --codec h265 --steps 100 --warmup 10 > gpurun_out/bench_h265_prof.json 2> gpurun_out/bench_h265_prof.err || { echo "h265 prof failed"; tail -30 gpurun_out/bench_h265_prof.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/bench_h265_prof.json')); print('h265 prof', d['value'])"
