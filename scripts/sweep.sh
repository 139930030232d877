#!/bin/bash
# One gpurun call: bench.py under several knob settings (SWEEP="label|args;label|args;...").
# Prints one summary line per setting; full JSON lines land in gpurun_out/sweep.jsonl.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out
: > gpurun_out/sweep.jsonl
STEPS=${STEPS:-150}
IFS=';' read -ra CFGS <<< "${SWEEP}"
for c in "${CFGS[@]}"; do
  label=${c%%|*}; args=${c#*|}
  timeout -k 10 240 python bench.py --steps $STEPS --warmup 20 --latency-samples 20 $args > gpurun_out/sweep_one.log 2>&1 || { echo "$label failed"; tail -20 gpurun_out/sweep_one.log; exit 1; }
  line=$(tail -1 gpurun_out/sweep_one.log)
  echo "{\"label\": \"$label\", \"result\": $line}" >> gpurun_out/sweep.jsonl
  python -c "import json,sys; d=json.loads(sys.argv[2]); b=d['rank0_launch_breakdown_ms_per_step']; print(sys.argv[1], d['value'], 'ms', d['ms_per_step'], 'pwait', d['rank0_parse_wait_ms_per_step'], 'parse', d['rank0_host_parse_ms_per_step'], 'gpu', d['rank0_gpu_kernel_ms_per_step'], 'wait', b['wait_ms'], 'copy', b['copy_ms'])" "$label" "$line"
done
