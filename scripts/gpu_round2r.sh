#!/bin/bash
# Fused level-ordered H.265 TU launch: GPU bit-exact tests first, then benches fused vs per-level
# and kernel stats of the fused path.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_hevc.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_hevc_fused.log 2>&1 || { echo "hevc gpu tests failed"; tail -40 gpurun_out/pytest_gpu_hevc_fused.log; exit 1; }
grep -cE "PASSED" gpurun_out/pytest_gpu_hevc_fused.log; tail -1 gpurun_out/pytest_gpu_hevc_fused.log
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python -u bench.py "$@" > gpurun_out/$n.json 2> gpurun_out/$n.err || { echo "$n failed"; tail -30 gpurun_out/$n.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/$n.json')); print('$n', d['value'], d['ms_per_step'], d.get('rank0_host_parse_ms_per_step'), d.get('rank0_gpu_kernel_ms_per_step'), d.get('frames_dropped'), d.get('rank0_launch_breakdown_ms_per_step'))"
}
run h265_1080p_fused --codec h265 --steps 100 --warmup 10
VEP_HEVC_TU_FUSED=0 run h265_1080p_levels --codec h265 --steps 100 --warmup 10
run h265_4k_fused --codec h265 --width 3840 --height 2160 --cams-per-gpu 8 --steps 60 --warmup 6
cd /tmp && export TMPDIR=/tmp && cd "$R"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_h265f -o run -- python3 bench.py --codec h265 --steps 100 --warmup 10 > gpurun_out/bench_h265f_prof.json 2> gpurun_out/bench_h265f_prof.err || { echo "h265 prof failed"; tail -30 gpurun_out/bench_h265f_prof.err; exit 1; }
echo prof ok
