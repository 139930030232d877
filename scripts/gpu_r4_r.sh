#!/bin/bash
# Round 4: where the headline's host CPU goes (cores per thread role in the timed region), at the
# driver's command and over 200 steps.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4r}
mkdir -p "$O"
for n in driver_1 steps200; do
  echo "[r] $n"
  if [ $n = steps200 ]; then args="--gpus 1 --steps 200 --warmup 20"; else args="--gpus 1 --steps 20 --warmup 5"; fi
  timeout -k 10 400 python -u bench.py $args > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; tail -30 "$O/$n.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print(d['value'], d['rank0_gpu_kernel_ms_per_step'], json.dumps(d['rank0_host_cpu_cores_by_thread']))"
done
echo "[r] done"
