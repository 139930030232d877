#!/bin/bash
# Round 6, H.265 intra TU schedule: the persistent ticket queue (default),
# per-level launches (VEP_HEVC_TU_WINDOW=0) and one workgroup per picture (-1), alternated three
# times, on the GPU-side ceiling (--source records: no host parse in the loop, so the GPU time of
# the schedule is what moves the rate) at BASELINE config 5's shape (8 x 4K H.265, 8 slices).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-r6hevc}; mkdir -p "$O"
for i in 1 2 3; do
  for v in queue:X=1 levels:VEP_HEVC_TU_WINDOW=0 picture:VEP_HEVC_TU_WINDOW=-1; do
    n=${v%%:*}_$i
    env "${v#*:}" timeout -k 10 300 python -u bench.py --codec h265 --width 3840 --height 2160 --cams-per-gpu 8 \
      --source records --steps ${STEPS:-20} --warmup 3 --latency-samples 0 --clients 0 --ref-cpu off \
      > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; tail -20 "$O/$n.err"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], {k: d.get(k) for k in ('value','rank0_gpu_kernel_ms_per_step','frames_dropped')})" "$O/$n.json" "$n"
  done
done
echo "[hevc] done"
