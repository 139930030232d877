#!/bin/bash
# Round 4: the new H.264 GPU cases (B field pairs, marking / long-term coverage in frames and
# fields, the live field-pair camera), then the whole GPU suite, smoke, and a kernel-stats profile
# of the PAFF IBBP bench.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4k}
mkdir -p "$O"
echo "[k] new gpu cases"
timeout -k 10 300 python -u -m pytest tests/test_gpu_avc_high.py tests/test_avc_paff.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "paff or marking" > "$O/pytest_new.log" 2>&1 || { echo "new cases failed"; tail -40 "$O/pytest_new.log"; exit 1; }
tail -1 "$O/pytest_new.log"
echo "[k] gpu suite"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
  || { echo "pytest failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
echo "[k] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$O/smoke.log"; exit 1; }
tail -2 "$O/smoke.log"
echo "[k] rocprof PAFF IBBP"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_paff" -o paff --output-format csv -- python3 "$R/bench.py" \
  --steps 60 --warmup 10 --interlaced 2 --clients 0 --latency-samples 0 > "$O/prof_paff.log" 2>&1 \
  || { echo "rocprof failed"; tail -30 "$O/prof_paff.log"; exit 1; }
cd "$R"
ls "$O/prof_paff" | head
echo "[k] serving with publish-latency percentiles"
timeout -k 10 400 python -u tools/bench_serving.py --codec h265 --width 3840 --height 2160 --cams 8 --slices 8 \
  --clients 8 --frontends 0,2 --duration 6 --out "$O/s4k_pub.jsonl" > "$O/s4k.log" 2>&1 \
  || { echo "serving 4k failed"; tail -30 "$O/s4k.log"; exit 1; }
cut -c1-900 "$O/s4k_pub.jsonl"
timeout -k 10 400 python -u tools/bench_serving.py --cams 32 --clients 128 --frontends 2 --duration 6 \
  --out "$O/s1080_pub.jsonl" > "$O/s1080.log" 2>&1 || { echo "serving 1080p failed"; tail -30 "$O/s1080.log"; exit 1; }
cut -c1-900 "$O/s1080_pub.jsonl"
echo "[k] done"
