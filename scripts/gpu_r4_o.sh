#!/bin/bash
# Round 4: A/B of one wave sync per deblocking direction (default) vs one after every edge
# (VEP_DBK_SYNC=1): the H.264 GPU bit-exact tests, then phase clocks of each variant twice,
# alternating, then the whole GPU suite.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4o}
mkdir -p "$O"
echo "[o] h264 gpu tests"
timeout -k 10 400 python -u -m pytest tests/test_gpu_avc.py tests/test_gpu_avc_high.py tests/test_avc_paff.py -m gpu -x -q \
  --timeout 120 --timeout-method thread > "$O/pytest_avc.log" 2>&1 || { echo "avc tests failed"; tail -40 "$O/pytest_avc.log"; exit 1; }
tail -1 "$O/pytest_avc.log"
for run in 1 2; do
  for p in 1 0; do
    VEP_DBK_SYNC=$p VEP_AVC_PROF=1 timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --clients 0 --latency-samples 0 \
      > "$O/prof_p${p}_$run.json" 2> "$O/prof_p${p}_$run.err" || { echo "prof failed"; tail -20 "$O/prof_p${p}_$run.err"; exit 1; }
    python -c "import json; d=json.loads(open('$O/prof_p${p}_$run.json').read().strip().splitlines()[-1]); print('sync_each=$p run $run', json.dumps({k: d[k] for k in ('value', 'rank0_gpu_kernel_ms_per_step', 'dbk_cycles_per_mb')}))"
  done
done
echo "[o] gpu suite"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
  || { echo "pytest failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
echo "[o] done"
