#!/bin/bash
# Round 2 (session 2): parse A/B on the box CPU, full GPU suite, smoke, default bench under
# rocprofv3 kernel stats, keyframe-only RTSP bench (BASELINE config 3), H.265 1080p bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for i in 1 2; do
  for b in pb_old pb_new; do echo -n "$b "; timeout -k 5 120 taskset -c 3 tools/bin/$b high 30 3 | grep "best of" || exit 1; done
  for b in hb_old hb_new; do echo -n "$b "; timeout -k 5 120 taskset -c 3 tools/bin/$b 1920 1080 16 2 27 records || exit 1; done
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_all5.log 2>&1 || { echo "gpu suite failed"; tail -60 gpurun_out/pytest_gpu_all5.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_all5.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2n -o run -- python3 bench.py --steps 300 --warmup 30 > gpurun_out/bench_default_prof.json 2> gpurun_out/bench_default_prof.err || { echo "prof bench failed"; tail -30 gpurun_out/bench_default_prof.err; exit 1; }
cat gpurun_out/bench_default_prof.json
timeout -k 10 300 python -u bench.py --steps 300 --warmup 30 > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed"; tail -30 gpurun_out/bench_default.err; exit 1; }
cat gpurun_out/bench_default.json
timeout -k 10 300 python -u bench.py --source rtsp --keyframe-only --steps 20 --warmup 2 > gpurun_out/bench_keyframe_only.json 2> gpurun_out/bench_keyframe_only.err || { echo "keyframe bench failed"; tail -30 gpurun_out/bench_keyframe_only.err; exit 1; }
cat gpurun_out/bench_keyframe_only.json
timeout -k 10 300 python -u bench.py --codec h265 --steps 100 --warmup 10 > gpurun_out/bench_h265_1080p.json 2> gpurun_out/bench_h265_1080p.err || { echo "h265 bench failed"; tail -30 gpurun_out/bench_h265_1080p.err; exit 1; }
cat gpurun_out/bench_h265_1080p.json
