#!/bin/bash
# Round 6: the 10-bit / 4:2:2 / Main10 GPU tests with the full-depth surface readback, then the
# driver's command with the reference-equivalent CPU child run (vs_baseline).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r6c}
mkdir -p "$O"
echo "[c] 10-bit GPU tests"
timeout -k 10 600 python -u -m pytest tests/test_avc_high10.py tests/test_avc_422.py tests/test_gpu_hevc_main10.py \
  tests/test_hevc_camera.py tests/test_records_replay.py -m gpu -x -v --timeout 240 --timeout-method thread > "$O/pytest_gpu_10bit.log" 2>&1 \
  || { echo "GPU tests failed"; tail -40 "$O/pytest_gpu_10bit.log"; exit 1; }
tail -3 "$O/pytest_gpu_10bit.log"
echo "[c] driver command (with the reference-equivalent child)"
T0=$SECONDS
timeout -k 10 580 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/driver_1.json" 2> "$O/driver_1.err" \
  || { echo "bench failed"; tail -30 "$O/driver_1.err"; exit 1; }
echo "driver command wall: $((SECONDS - T0)) s" | tee "$O/driver_wall.txt"
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print({k: d.get(k) for k in ('value','vs_baseline','reference_equivalent_cpu_fps','reference_equivalent_p50_latency_ms','p50_latency_ms','scope')}); print(d.get('reference_equivalent_run'))" "$O/driver_1.json"
echo "[c] GPU-side ceiling: records replay (no host parse in the loop)"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --source records --steps 20 --warmup 3 --clients 0 --latency-samples 0 --ref-cpu off \
    > "$O/records_$i.json" 2> "$O/records_$i.err" || { echo "records bench failed"; tail -20 "$O/records_$i.err"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print({k: d.get(k) for k in ('value','frames_dropped','rank0_gpu_kernel_ms_per_step','ms_per_step','gpu_lanes')})" "$O/records_$i.json"
done
echo "[c] rocprof records replay"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_records" -o records --output-format csv -- python3 "$R/bench.py" \
  --source records --steps 6 --warmup 2 --clients 0 --latency-samples 0 --ref-cpu off > "$O/prof_records.log" 2>&1 \
  || { echo "rocprof failed"; tail -20 "$O/prof_records.log"; exit 1; }
cd "$R"
find "$O/prof_records" -name "*kernel_stats.csv" | head -3
echo "[c] done"
