#!/bin/bash
# Round 4 closing evidence on a fresh box: BASELINE config 5 (8 x 4K H.265, RTMP, annotate, 8
# clients, 8 slices) at 300 steps, the 4K and 1080p serving tails with publish-latency
# percentiles, and the headline twice.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4p}
mkdir -p "$O"
run() {
  local n=$1; shift
  echo "[p] $n"
  timeout -k 10 500 python -u bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; tail -30 "$O/$n.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print(json.dumps({k: d.get(k) for k in ('value', 'frames_decoded', 'frames_published', 'p50_latency_ms', 'p99_latency_ms', 'rank0_gpu_kernel_ms_per_step')}))"
}
C5="--codec h265 --width 3840 --height 2160 --cams-per-gpu 8 --clients 8 --rtmp --annotate --steps 300 --warmup 30"
run cfg5_slices8 $C5 --slices 8
echo "[p] serving 4K"
timeout -k 10 400 python -u tools/bench_serving.py --codec h265 --width 3840 --height 2160 --cams 8 --slices 8 \
  --clients 8,32 --frontends 0,2 --duration 6 --out "$O/s4k.jsonl" > "$O/s4k.log" 2>&1 \
  || { echo "serving 4k failed"; tail -30 "$O/s4k.log"; exit 1; }
cut -c180-560 "$O/s4k.jsonl"
run headline_1 --gpus 1 --steps 20 --warmup 5
run headline_2 --gpus 1 --steps 20 --warmup 5
echo "[p] done"
