#!/bin/bash
# Round 4: B field pairs and the live field-pair camera on gfx950, then the 1080i PAFF bench
# (IBBP field pairs), a node-scale serving rehearsal on the box's CPU share (CPU-backend worker
# processes standing in for GPUs) and the headline.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4j}
mkdir -p "$O"
echo "[j] paff gpu tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_avc_high.py tests/test_avc_paff.py -m gpu -x -q --timeout 120 \
  --timeout-method thread -k "paff" > "$O/pytest_paff.log" 2>&1 || { echo "paff tests failed"; tail -40 "$O/pytest_paff.log"; exit 1; }
tail -1 "$O/pytest_paff.log"
echo "[j] bench 1080i PAFF IBBP"
timeout -k 10 400 python -u bench.py --steps 200 --warmup 20 --interlaced 2 > "$O/bench_paff_ibbp.json" 2> "$O/bench_paff.err" \
  || { echo "paff bench failed"; tail -30 "$O/bench_paff.err"; exit 1; }
cut -c1-300 "$O/bench_paff_ibbp.json"
echo "[j] serving node rehearsal (cpu workers)"
timeout -k 10 500 python -u -m vep_bench.serving_node --workers 1,2,4,8 --cams-per-worker 4 --clients-per-cam 2 \
  --duration 4 --out "$O/node_rehearsal_box16.jsonl" > "$O/node.log" 2>&1 || { echo "node rehearsal failed"; tail -30 "$O/node.log"; exit 1; }
cut -c1-400 "$O/node_rehearsal_box16.jsonl"
echo "[j] headline"
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/headline.json" 2> "$O/headline.err" \
  || { echo "headline failed"; tail -30 "$O/headline.err"; exit 1; }
cut -c1-300 "$O/headline.json"
echo "[j] done"
