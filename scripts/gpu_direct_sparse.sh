#!/bin/bash
# Direct sparse emission: GPU bit-exactness, then parse A/B (1 and 15 threads) and the
# end-to-end headline A/B against the dense-record build, all on one box.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-dsparse}; mkdir -p "$O"
timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
  || { echo "pytest failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$O/smoke.log"; exit 1; }
for i in 1 2; do
  timeout -k 10 200 taskset -c 2 python tools/parse_ab.py --so tools/abso/vep_dense.so --reps 3 2>&1 | tail -1 | tee -a "$O/parse_ab.log" || exit 1
  timeout -k 10 200 taskset -c 2 python tools/parse_ab.py --reps 3 2>&1 | tail -1 | tee -a "$O/parse_ab.log" || exit 1
done
for i in 1 2; do
  timeout -k 10 240 python tools/parse_ab.py --so tools/abso/vep_dense.so --reps 3 --threads 15 --cams 32 2>&1 | tail -1 | tee -a "$O/parse_ab15.log" || exit 1
  timeout -k 10 240 python tools/parse_ab.py --reps 3 --threads 15 --cams 32 2>&1 | tail -1 | tee -a "$O/parse_ab15.log" || exit 1
done
TAG=${TAG:-dsparse} bash scripts/gpu_e2e_ab.sh
# host CPU profile of the headline's timed region (every thread: farm, ingest, parse, lanes)
VEP_HOSTPROF="$R/$O/hostprof_headline.txt" timeout -k 10 300 python -u bench.py --steps 200 --warmup 10 --latency-samples 0 --clients 0 \
  > "$O/hostprof_headline.json" 2> "$O/hostprof_headline.err" || { echo "hostprof bench failed"; tail -20 "$O/hostprof_headline.err"; exit 1; }
echo "hostprof samples: $(wc -l < "$O/hostprof_headline.txt") lines"
