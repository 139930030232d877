#!/bin/bash
# Live RTSP farm bench: strand affinity on vs off.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for aff in 1 0; do
  VEP_STRAND_AFFINITY=$aff timeout -k 10 400 python -u bench.py --source rtsp --steps 150 --warmup 10 > gpurun_out/bench_rtsp_aff$aff.json 2> gpurun_out/bench_rtsp_aff$aff.err || { echo "rtsp failed"; tail -20 gpurun_out/bench_rtsp_aff$aff.err; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/bench_rtsp_aff$aff.json')); print('aff=$aff', d['value'], d['frames_decoded'], d['frames_published'], d['rank0_gpu_kernel_ms_per_step'])"
done
