#!/bin/bash
# Round 6 check after the parse work: GPU tests + smoke (bit-exact decodes on gfx950 with the new
# records path), the driver's command twice (with the reference-equivalent run once), and a
# rocprofv3 kernel-stats profile of the headline. Output: gpurun_out/$TAG/. Stops at the first failure.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=$R/gpurun_out/${TAG:-r6check2}; mkdir -p "$O"
echo "[check] GPU tests"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
  > "$O/pytest_gpu.log" 2>&1 || { echo "GPU tests failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
echo "[check] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 \
  || { echo "smoke failed"; tail -30 "$O/smoke.log"; exit 1; }
tail -3 "$O/smoke.log"
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); c=d['rank0_host_cpu_cores_by_thread']['vep-parse']; print({k: d.get(k) for k in ('value','ms_per_step','frames_dropped','decode_errors','p50_latency_ms','p99_latency_ms','rank0_gpu_kernel_ms_per_step','rank0_pictures_per_launch','reference_equivalent_cpu_fps','vs_baseline')}, 'parse core-ms/picture', round(c * d['ms_per_step'] * d['steps'] / d['frames_decoded'], 3))" "$1"; }
echo "[check] driver command (with the reference-equivalent run)"
timeout -k 10 500 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/driver_1.json" 2> "$O/driver_1.err" \
  || { echo "bench failed"; tail -30 "$O/driver_1.err"; exit 1; }
summ "$O/driver_1.json"
echo "[check] driver command, 100 steps, no reference run"
timeout -k 10 500 python -u bench.py --gpus 1 --steps 100 --warmup 5 --ref-cpu off > "$O/driver_100.json" 2> "$O/driver_100.err" \
  || { echo "bench 100 failed"; tail -30 "$O/driver_100.err"; exit 1; }
summ "$O/driver_100.json"
echo "[check] rocprofv3 kernel stats of the headline"
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- python3 "$R/bench.py" --steps 20 --warmup 5 --latency-samples 0 --ref-cpu off > "$O/prof.log" 2>&1 \
  || { echo "rocprof failed"; tail -20 "$O/prof.log"; exit 1; }
find "$O/prof" -name "*kernel_stats.csv" -exec head -12 {} \;
echo "[check] done"
