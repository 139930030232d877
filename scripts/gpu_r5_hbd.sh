#!/bin/bash
# Round 5: the driver's headline configuration with H.264 High 10 / High 4:2:2 / 10-bit 4:2:2
# streams (avc_inter_kernel<P, CF> + avc_hbd_kernel<P, CF> + narrow). JSON lines under
# gpurun_out/$TAG/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-r5hbd}; mkdir -p "$O"
for v in high10:--bit-depth=10 h422:--chroma-format=2 h422_10:--bit-depth=10:--chroma-format=2; do
  IFS=: read -r nm f1 f2 <<< "$v"
  timeout -k 10 500 python -u bench.py --gpus 1 --steps ${STEPS:-10} --warmup 3 $f1 ${f2:-} > "$O/$nm.json" 2> "$O/$nm.err" \
    || { echo "$nm failed"; tail -20 "$O/$nm.err"; exit 1; }
  python - "$O/$nm.json" "$nm" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
keys = ("value", "ms_per_step", "rank0_gpu_kernel_ms_per_step", "frames_dropped", "frames_shed",
        "rank0_pictures_per_launch", "p50_latency_ms", "p99_latency_ms")
print(sys.argv[2], {k: d.get(k) for k in keys if k in d})
PY
done
echo "[hbd] done"
