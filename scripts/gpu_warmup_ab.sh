#!/bin/bash
# Driver-shaped headline (--steps 20) after 5 vs 60 warmup steps, alternated on one box, plus a
# 100-step run: does the short timed window start before the pipeline reaches steady state?
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-warmab}; mkdir -p "$O"
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --gpus 1 --latency-samples 0 --clients 0 "$@" > "$O/$n.json" 2> "$O/$n.err" \
    || { echo "$n failed"; tail -20 "$O/$n.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d.get('frames_dropped'), d.get('rank0_gpu_kernel_ms_per_step'))"
}
for i in 1 2; do
  run w5_s20_$i --steps 20 --warmup 5
  run w60_s20_$i --steps 20 --warmup 60
done
run w5_s100 --steps 100 --warmup 5
