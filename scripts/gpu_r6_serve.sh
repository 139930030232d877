#!/bin/bash
# Round 6 serving A/B: the native endpoint with bus slot leases (zero copy, default) vs one copy
# per frame per serving process (VEP_RPC_ZERO_COPY=0), 32 x 1080p cameras, 128 / 256 clients,
# in-process (one-GPU default) and 2 serving processes; grpcio in 2 serving processes for the
# serving-CPU-per-GB comparison.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-r6serve}; mkdir -p "$O"
for zc in 1 0 1; do
  VEP_RPC_ZERO_COPY=$zc timeout -k 10 400 python -u tools/bench_serving.py --cams 32 --clients 128,256 \
    --modes native:0,native:2 --duration ${DURATION:-5} --out "$O/s1080_zc$zc.jsonl" > "$O/s1080_zc$zc.log" 2>&1 \
    || { echo "serving zc=$zc failed"; tail -30 "$O/s1080_zc$zc.log"; exit 1; }
  echo "== zero_copy=$zc"; tail -5 "$O/s1080_zc$zc.log"
done
timeout -k 10 400 python -u tools/bench_serving.py --cams 32 --clients 128,256 --modes grpcio:2 \
  --duration ${DURATION:-5} --out "$O/s1080_grpcio.jsonl" > "$O/s1080_grpcio.log" 2>&1 \
  || { echo "grpcio serving failed"; tail -30 "$O/s1080_grpcio.log"; exit 1; }
echo "== grpcio"; tail -3 "$O/s1080_grpcio.log"
echo "[serve] done"
