#!/bin/bash
# GPU tests + smoke, then the headline bench with lanes that sleep-poll their stage's completion
# event (default) vs hipEventSynchronize (VEP_SPIN_WAIT=1), alternated on one box, plus the
# keyframe-only and 4K H.265 shapes once each.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-waitab}; mkdir -p "$O"
timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
  || { echo "pytest failed"; tail -40 "$O/pytest_gpu.log"; exit 1; }
tail -1 "$O/pytest_gpu.log"
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || { echo "smoke failed"; tail -20 "$O/smoke.log"; exit 1; }
run() {  # name, env, bench args...
  local n=$1 e=$2; shift 2
  env "$e" timeout -k 10 300 python -u bench.py --latency-samples 0 --clients 0 "$@" > "$O/$n.json" 2> "$O/$n.err" \
    || { echo "$n failed"; tail -20 "$O/$n.err"; exit 1; }
  python -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d.get('rank0_gpu_kernel_ms_per_step'))"
}
for i in 1 2 3; do
  run polite_$i VEP_SPIN_WAIT=0 --steps 100 --warmup 10
  run spin_$i VEP_SPIN_WAIT=1 --steps 100 --warmup 10
done
run kf_only VEP_SPIN_WAIT=0 --keyframe-only --steps 60 --warmup 8
run h265_4k VEP_SPIN_WAIT=0 --codec h265 --width 3840 --height 2160 --cams-per-gpu 8 --steps 40 --warmup 6
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench_driver.json" 2> "$O/bench_driver.err" \
  || { echo "driver bench failed"; tail -20 "$O/bench_driver.err"; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_driver.json').read().strip().splitlines()[-1]); print('driver', d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['frames_dropped'])"
