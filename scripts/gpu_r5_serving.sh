#!/bin/bash
# Round 5 serving measurement (VideoLatestImage at node scale) on one box: 32 x 1080p cameras,
# 32 / 128 / 256 clients, the native HTTP/2 endpoint in-process (the one-GPU `vep serve` default)
# and in 2 serving processes vs grpcio in 2 serving processes; then 8 x 4K H.265 with 8 / 32
# clients. JSON lines (p50 / p99 client latency, frames/s served, serving CPU per GB) under
# gpurun_out/$TAG/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-r5serve}; mkdir -p "$O"
timeout -k 10 600 python -u tools/bench_serving.py --cams 32 --clients 32,128,256 \
  --modes native:0,native:2,grpcio:2 --duration ${DURATION:-5} --out "$O/s1080.jsonl" > "$O/s1080.log" 2>&1 \
  || { echo "1080p serving failed"; tail -30 "$O/s1080.log"; exit 1; }
tail -12 "$O/s1080.log"
if [ "${K4:-1}" = 1 ]; then
  timeout -k 10 500 python -u tools/bench_serving.py --codec h265 --width 3840 --height 2160 --cams 8 --slices 8 \
    --clients 8,32 --modes native:0,native:2 --duration ${DURATION:-5} --out "$O/s4k.jsonl" > "$O/s4k.log" 2>&1 \
    || { echo "4K serving failed"; tail -30 "$O/s4k.log"; exit 1; }
  tail -6 "$O/s4k.log"
fi
echo "[serve] done"
