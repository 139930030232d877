#!/bin/bash
# Round 4: after the backlog / keyframe merge fix — the GOP-boundary backlog test on the GPU, the
# whole GPU suite, smoke, the live compressed cameras on the GPU, and the headline twice.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4q}
mkdir -p "$O"
echo "[q] backlog across IDR (gpu)"
timeout -k 10 200 python -u -m pytest tests/test_live_compressed.py tests/test_hevc_camera.py tests/test_avc_mono.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "backlog or mono" > "$O/pytest_backlog.log" 2>&1 || { echo "backlog failed"; tail -40 "$O/pytest_backlog.log"; exit 1; }
tail -1 "$O/pytest_backlog.log"
echo "[q] gpu suite"
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
  || { echo "pytest failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
echo "[q] smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$O/smoke.log"; exit 1; }
tail -2 "$O/smoke.log"
for n in 1 2; do
  echo "[q] headline $n"
  timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/headline_$n.json" 2> "$O/headline_$n.err" \
    || { echo "headline failed"; tail -30 "$O/headline_$n.err"; exit 1; }
  cut -c1-300 "$O/headline_$n.json"
done
echo "[q] done"
