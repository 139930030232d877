#!/bin/bash
# Round 4: node-scale serving on one box (tools/bench_serving.py): live 1080p H.264 and 4K H.265
# cameras; in-process server (frontends=0) vs K serving processes on the frame bus, at growing
# client counts. Each run has its own time limit; the script stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4serve}
mkdir -p "$O"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 ${LIMIT:-420} python -u tools/bench_serving.py --out "$O/$n.jsonl" "$@" > "$O/$n.log" 2>&1 \
    || { echo "$n failed"; tail -30 "$O/$n.log"; exit 1; }
  python - "$O/$n.jsonl" <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["resolution"], "K=%d" % d["frontends"], "clients=%d" % d["clients"], "p50", d["p50_ms"], "p99", d["p99_ms"],
          "served/s", d["frames_served_per_s"], "GB/s", d["served_gbytes_per_s"], "cpu", d["machine_cpu_busy"],
          "srv", d["serving_cpu"], "cli", d["client_cpu"], "dma/s", d["bus_dma_gbytes_per_s"])
PY
}
run s1080 --cams 32 --clients ${C1080:-32,128,256} --frontends ${F1080:-0,1,2,4} --duration ${DUR:-4}
run s4k --codec h265 --width 3840 --height 2160 --cams 8 --clients ${C4K:-8,32} --frontends ${F4K:-0,2} --duration ${DUR:-4}
echo "[serving] done"
