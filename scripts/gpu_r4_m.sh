#!/bin/bash
# Round 4: packed LDS accesses for the vertical deblocking edges — the H.264 GPU bit-exact tests
# (every config incl. field pairs), then the phase clocks (compare filter cycles per MB with
# profiles/r4/final/avc_phase_clocks_headline.json) and the headline.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4m}
mkdir -p "$O"
echo "[m] h264 gpu tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_avc.py tests/test_gpu_avc_high.py tests/test_avc_paff.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$O/pytest_avc.log" 2>&1 || { echo "avc tests failed"; tail -40 "$O/pytest_avc.log"; exit 1; }
tail -1 "$O/pytest_avc.log"
echo "[m] avc phase clocks"
VEP_AVC_PROF=1 timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --clients 0 --latency-samples 0 \
  > "$O/avc_prof.json" 2> "$O/avc_prof.err" || { echo "avc prof failed"; tail -20 "$O/avc_prof.err"; exit 1; }
python -c "import json; d=json.loads(open('$O/avc_prof.json').read().strip().splitlines()[-1]); print(json.dumps({k: v for k, v in d.items() if 'cycles' in k or k in ('value', 'rank0_gpu_kernel_ms_per_step')})[:1500])"
echo "[m] rocprof headline kernels"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o hl --output-format csv -- python3 "$R/bench.py" \
  --steps 60 --warmup 10 --clients 0 --latency-samples 0 > "$O/prof.log" 2>&1 || { echo "rocprof failed"; tail -30 "$O/prof.log"; exit 1; }
cd "$R"
head -6 "$O/prof/hl_kernel_stats.csv" | cut -c1-200
echo "[m] done"
