#!/bin/bash
# Round 4: the process-isolated hub on the GPU under more load (16 x 1080p cameras in one worker
# process, 200 frames served through the frame bus, 50 steady-state RCCL gathers, a SIGKILLed
# worker restarted and regrouped).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4h}
mkdir -p "$O"
timeout -k 10 300 python -u -m vep_bench.isolated_check --devices=0 --cams 16 --width 1920 --height 1080 \
  --letterbox 640 --samples 200 --gathers 50 --kill > "$O/isolated_check_gpu.json" 2> "$O/isolated_check_gpu.err" \
  || { echo "isolated check failed"; tail -30 "$O/isolated_check_gpu.err"; tail -c 2000 "$O/isolated_check_gpu.json"; exit 1; }
python3 - "$O/isolated_check_gpu.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print({k: d.get(k) for k in ["ok", "shm_pinned", "serve_samples", "serve_p50_ms", "served_MBps", "first_gather_ms",
                             "steady_gathers", "steady_gather_ms_p50", "steady_gather_ms_max", "batch_max_abs_err",
                             "restarted", "batch_after_restart_max_abs_err"]})
print(d["group"][0].get("backend"))
PY
echo "[h] done"
