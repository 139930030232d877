#!/bin/bash
# Round 6 serving with the native load generator (csrc/vep/h2load.h) as the clients: 32 x 1080p
# live cameras, 128 / 256 back-to-back VideoLatestImage clients, native endpoint in-process and in
# 2 serving processes; then the Python grpcio clients at 128 on the same box for comparison.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-r6serve2}; mkdir -p "$O"
timeout -k 10 500 python -u tools/bench_serving.py --cams 32 --clients 128,256 --client-threads 16 \
  --modes native:2,native:0 --client native --duration ${DURATION:-5} --out "$O/native_clients.jsonl" \
  > "$O/native_clients.log" 2>&1 || { echo "native-client serving failed"; tail -30 "$O/native_clients.log"; exit 1; }
python - "$O/native_clients.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print(r["serving"], r["frontends"], r["clients"], "p50", r["p50_ms"], "p99", r["p99_ms"], "fps", r["frames_served_per_s"],
          "GB/s", r["served_gbytes_per_s"], "client_cpu", r["client_cpu"], "serving_cpu", r["serving_cpu"], "busy", r["machine_cpu_busy"])
PY
timeout -k 10 400 python -u tools/bench_serving.py --cams 32 --clients 128 --modes native:2 --client grpcio \
  --duration ${DURATION:-5} --out "$O/grpcio_clients.jsonl" > "$O/grpcio_clients.log" 2>&1 \
  || { echo "grpcio-client serving failed"; tail -30 "$O/grpcio_clients.log"; exit 1; }
python - "$O/grpcio_clients.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    r = json.loads(l)
    print("grpcio clients:", r["serving"], r["frontends"], r["clients"], "p50", r["p50_ms"], "p99", r["p99_ms"], "fps",
          r["frames_served_per_s"], "GB/s", r["served_gbytes_per_s"], "client_cpu", r["client_cpu"], "busy", r["machine_cpu_busy"])
PY
echo "[serve2] done"
