#!/bin/bash
# Round 4, fifth check: Main10 on the GPU (u16 surfaces, narrowing) + the 8-bit HEVC / H.264
# GPU suites unchanged, then the 8-bit H.265 replay kernel stats (the templated kernels must
# not slow the 8-bit path) and a Main10 replay bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4e}
mkdir -p "$O"
echo "[e] main10 + hevc gpu tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_hevc_main10.py tests/test_gpu_hevc.py tests/test_gpu_hevc_tools.py \
  -x -v --timeout 120 --timeout-method thread > "$O/pytest_hevc.log" 2>&1 || { echo "pytest failed"; tail -40 "$O/pytest_hevc.log"; exit 1; }
tail -3 "$O/pytest_hevc.log"
run() {
  local n=$1; shift
  timeout -k 10 300 python -u bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; tail -30 "$O/$n.err"; exit 1; }
  python - "$O/$n.json" "$n" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], "dropped", d.get("frames_dropped"), "gpu_ms", d.get("rank0_gpu_kernel_ms_per_step"))
PY
}
run h265_1080p --codec h265 --source replay --steps 60 --warmup 10 --latency-samples 0 --clients 0
run h265_1080p_main10 --codec h265 --source replay --steps 60 --warmup 10 --latency-samples 0 --clients 0 --bit-depth 10
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d "$O/kt" -o kt -- python3 "$R/bench.py" --codec h265 --source replay \
  --steps 30 --warmup 5 --latency-samples 0 --clients 0 > "$O/kt.log" 2>&1 || { echo "kt failed"; tail -20 "$O/kt.log"; exit 1; }
python3 "$R/tools/rocpd_kernel_stats.py" "$O/kt" > "$O/kernel_stats_h265_1080p.csv"
rm -rf "$O/kt"
head -6 "$O/kernel_stats_h265_1080p.csv" | cut -c1-150
timeout -k 10 200 rocprofv3 --kernel-trace -d "$O/kt10" -o kt -- python3 "$R/bench.py" --codec h265 --source replay \
  --steps 30 --warmup 5 --latency-samples 0 --clients 0 --bit-depth 10 > "$O/kt10.log" 2>&1 || { echo "kt10 failed"; tail -20 "$O/kt10.log"; exit 1; }
python3 "$R/tools/rocpd_kernel_stats.py" "$O/kt10" > "$O/kernel_stats_h265_1080p_main10.csv"
rm -rf "$O/kt10"
head -8 "$O/kernel_stats_h265_1080p_main10.csv" | cut -c1-150
echo "[e] done"
