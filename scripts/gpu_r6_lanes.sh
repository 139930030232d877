#!/bin/bash
# Round 6: GPU-side ceiling (--source records, no host parse) vs the number of lanes (streams),
# then the driver's command at the default and at the best lane count. Output: gpurun_out/$TAG/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=$R/gpurun_out/${TAG:-r6lanes}; mkdir -p "$O"
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], d['value'], 'fps', d['ms_per_step'], 'ms/step gpu', d.get('rank0_gpu_kernel_ms_per_step'), 'pics/launch', d.get('rank0_pictures_per_launch'))" "$1" "$2" | tee -a "$O/summary.log"; }
for L in 3 6 4 8; do
  VEP_LANES=$L timeout -k 10 400 python -u bench.py --source records --steps 20 --warmup 3 --latency-samples 0 --ref-cpu off > "$O/records_l$L.json" 2> "$O/records_l$L.err" \
    || { echo "records L=$L failed"; tail -20 "$O/records_l$L.err"; exit 1; }
  summ "$O/records_l$L.json" "records lanes=$L"
done
for L in 3 6 3 6; do
  VEP_LANES=$L timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --ref-cpu off > "$O/drv_l$L.json" 2> "$O/drv_l$L.err" \
    || { echo "driver L=$L failed"; tail -20 "$O/drv_l$L.err"; exit 1; }
  summ "$O/drv_l$L.json" "driver lanes=$L"
done
