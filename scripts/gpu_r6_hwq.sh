#!/bin/bash
# Round 6: do the lanes' kernels overlap? GPU-side ceiling (--source records) at HIP's default 4
# hardware queues vs 8 and 16 (GPU_MAX_HW_QUEUES), 32 and 64 cameras. Output: gpurun_out/$TAG/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=$R/gpurun_out/${TAG:-r6hwq}; mkdir -p "$O"
for Q in 4 8 16; do
  for C in 32 64; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 400 python -u bench.py --source records --cams-per-gpu $C --steps 10 --warmup 2 --latency-samples 0 \
      --ref-cpu off > "$O/records_q${Q}_c$C.json" 2> "$O/records_q${Q}_c$C.err" || { echo "records Q=$Q C=$C failed"; tail -20 "$O/records_q${Q}_c$C.err"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print('hwq', sys.argv[2], 'cams', sys.argv[3], d['value'], 'pictures/s', d['ms_per_step'], 'ms/step, gpu kernel ms/step', d.get('rank0_gpu_kernel_ms_per_step'))" "$O/records_q${Q}_c$C.json" $Q $C | tee -a "$O/summary.log"
  done
done
