#!/bin/bash
# Round 4: H.264 field pictures (PAFF) on gfx950 — the GPU bit-exact tests first (field slots,
# field MC / bS, the weave), then the whole GPU suite, a 1080i PAFF bench (32 cameras, field
# pairs), a rocprofv3 kernel summary of it, and the headline bench as the driver runs it.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4i}
mkdir -p "$O"
echo "[i] paff gpu tests"
timeout -k 10 300 python -u -m pytest tests/test_gpu_avc_high.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "paff or interlaced" > "$O/pytest_paff.log" 2>&1 || { echo "paff tests failed"; tail -40 "$O/pytest_paff.log"; exit 1; }
tail -1 "$O/pytest_paff.log"
echo "[i] gpu suite"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
  || { echo "pytest failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
echo "[i] bench 1080i PAFF"
timeout -k 10 400 python -u bench.py --steps 200 --warmup 20 --interlaced 2 > "$O/bench_paff.json" 2> "$O/bench_paff.err" \
  || { echo "paff bench failed"; tail -30 "$O/bench_paff.err"; exit 1; }
cut -c1-400 "$O/bench_paff.json"
echo "[i] bench 1080i frame pictures"
timeout -k 10 400 python -u bench.py --steps 200 --warmup 20 --interlaced 1 > "$O/bench_i1.json" 2> "$O/bench_i1.err" \
  || { echo "interlaced-frames bench failed"; tail -30 "$O/bench_i1.err"; exit 1; }
cut -c1-300 "$O/bench_i1.json"
echo "[i] rocprof PAFF"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_paff" -o paff -- python3 "$R/bench.py" --steps 60 --warmup 10 \
  --interlaced 2 --clients 0 --latency-samples 0 > "$O/prof_paff.log" 2>&1 || { echo "rocprof failed"; tail -30 "$O/prof_paff.log"; exit 1; }
cd "$R"
find "$O/prof_paff" -name "*kernel_stats.csv" | head -3
echo "[i] headline"
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/headline.json" 2> "$O/headline.err" \
  || { echo "headline failed"; tail -30 "$O/headline.err"; exit 1; }
cut -c1-300 "$O/headline.json"
echo "[i] done"
