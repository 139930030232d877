#!/bin/bash
# Wavefront LDS polls with vs without s_sleep: keyframe-only shape (intra + deblocking
# wavefronts dominate), per-MB phase cycles and GPU ms per step, builds alternated on one box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-sleepab}; mkdir -p "$O"
SO=video_edge_ai_proxy_amd/_vep.cpython-310-x86_64-linux-gnu.so
cp "$SO" /tmp/vep_A.so
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --keyframe-only --steps 40 --warmup 8 --latency-samples 0 --clients 0 \
    > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; tail -20 "$O/$n.err"; cp /tmp/vep_A.so "$SO"; exit 1; }
  python - "$O/$n.json" "$n" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d['value'], d.get('rank0_gpu_kernel_ms_per_step'), d.get('frames_dropped'),
      d.get('dbk_cycles_per_mb'), d.get('intra_cycles_per_mb', {}).get('wait') if d.get('intra_cycles_per_mb') else None)
PY
}
for i in 1 2; do
  cp /tmp/vep_A.so "$SO"; run A_$i VEP_NOP=1; run A_prof_$i VEP_AVC_PROF=1
  cp tools/ab_dbk/vep_B.so "$SO"; run B_$i VEP_NOP=1; run B_prof_$i VEP_AVC_PROF=1
done
cp /tmp/vep_A.so "$SO"
