#!/bin/bash
# Sparse coefficient records: GPU bit-exactness (pytest -m gpu, smoke), host parse A/B on the
# box CPU against the dense-record build (tools/abso/vep_dense.so), then the driver bench,
# keyframe-only and rocprof kernel statistics.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
O=gpurun_out/${TAG:-sparse}
mkdir -p "$O"
echo "[sparse] pytest -m gpu"
timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
  || { echo "pytest failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$O/smoke.log"; exit 1; }
tail -1 "$O/smoke.log"
echo "[sparse] parse A/B (single thread, box CPU)"
for i in 1 2 3; do
  timeout -k 10 200 taskset -c 2 python tools/parse_ab.py --so tools/abso/vep_dense.so --reps 3 2>&1 | tail -1 | tee -a "$O/parse_ab.log" || exit 1
  timeout -k 10 200 taskset -c 2 python tools/parse_ab.py --reps 3 2>&1 | tail -1 | tee -a "$O/parse_ab.log" || exit 1
done
SKIP_TESTS=1 HEVC_AB=0 TAG=${TAG:-sparse} bash scripts/gpu_r3_check.sh || exit 1
TAG=${TAG:-sparse} bash scripts/gpu_r3_prof.sh || exit 1
echo "[sparse] done"
