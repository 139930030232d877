#!/bin/bash
# Round 4 final: bench.py with no flags (the driver's default contract) and a kernel-stats profile
# of the headline at the end of the round.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4t}
mkdir -p "$O"
echo "[t] bench.py (defaults)"
timeout -k 10 500 python -u bench.py > "$O/default.json" 2> "$O/default.err" || { echo "default failed"; tail -30 "$O/default.err"; exit 1; }
cut -c1-400 "$O/default.json"
echo "[t] rocprof headline"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o headline --output-format csv -- python3 "$R/bench.py" \
  --steps 60 --warmup 10 --clients 0 --latency-samples 0 > "$O/prof.log" 2>&1 || { echo "rocprof failed"; tail -30 "$O/prof.log"; exit 1; }
cd "$R"
find "$O/prof" -name "*kernel_stats.csv" | head -3
echo "[t] done"
