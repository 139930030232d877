#!/bin/bash
# Round 6: GPU-side ceiling (--source records: no host parse in the loop) vs cameras per GPU — a
# tick of the replay holds one picture per camera, so more cameras means more pictures per launch
# (the live lanes merge more pictures per launch as work queues up). Output: gpurun_out/$TAG/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=$R/gpurun_out/${TAG:-r6ceiling}; mkdir -p "$O"
for C in 32 64 96; do
  timeout -k 10 500 python -u bench.py --source records --cams-per-gpu $C --steps 10 --warmup 2 --latency-samples 0 \
    --ref-cpu off > "$O/records_c$C.json" 2> "$O/records_c$C.err" || { echo "records C=$C failed"; tail -20 "$O/records_c$C.err"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('cams', sys.argv[2], d['value'], 'pictures/s', d['ms_per_step'], 'ms/step, gpu kernel ms/step', d.get('rank0_gpu_kernel_ms_per_step'), 'dropped', d.get('frames_dropped'))" "$O/records_c$C.json" $C | tee -a "$O/summary.log"
done
