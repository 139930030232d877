#!/bin/bash
# Round 4: the GPU suite parts changed since run D (interlaced frame pictures on the H.264 GPU
# path, Main10, parallel tiles / rows / H.264 slices feed the same kernels), then the serving
# benchmark at 4K with 8 slices per picture (parallel slice parse) and at 1080p 128 clients.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4g}
mkdir -p "$O"
echo "[g] gpu tests"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
  || { echo "pytest failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -2 "$O/pytest_gpu.log"
echo "[g] serving 4K (8 slices)"
timeout -k 10 400 python -u tools/bench_serving.py --codec h265 --width 3840 --height 2160 --cams 8 --slices 8 \
  --clients 8,32 --frontends 0,2 --duration 6 --out "$O/s4k_slices8.jsonl" > "$O/s4k.log" 2>&1 \
  || { echo "serving 4k failed"; tail -30 "$O/s4k.log"; exit 1; }
cat "$O/s4k_slices8.jsonl" | cut -c1-260
echo "[g] serving 1080p"
timeout -k 10 400 python -u tools/bench_serving.py --cams 32 --clients 128 --frontends 2,3 --duration 6 \
  --out "$O/s1080_128.jsonl" > "$O/s1080.log" 2>&1 || { echo "serving 1080p failed"; tail -30 "$O/s1080.log"; exit 1; }
cat "$O/s1080_128.jsonl" | cut -c1-260
echo "[g] done"
