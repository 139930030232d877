#!/bin/bash
# Round 6 parse A/B #3 on the box CPU: commit fe522e0 (ab_so/head.so) vs the tree (ring-buffer
# MB state, 16x16 MV predictor fast path, skipped MBs without the vector clear), alternated at 1 thread x 4 cameras and 16 threads x 32
# cameras; then the driver's command on the tree. Output: gpurun_out/$TAG/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-r6parse3}; mkdir -p "$O"
run() {  # label, args...
  local l=$1; shift
  timeout -k 10 300 python -u tools/parse_ab.py "$@" 2>&1 | tail -1 | sed "s/^/$l: /" | tee -a "$O/parse_ab.log"
}
for i in 1 2 3; do
  run "head 1t" --so ab_so/head.so --reps 4 || exit 1
  run "tree 1t" --reps 4 || exit 1
done
for i in 1 2; do
  run "head 16t" --so ab_so/head.so --reps 3 --threads 16 --cams 32 || exit 1
  run "tree 16t" --reps 3 --threads 16 --cams 32 || exit 1
done
echo "[driver command, tree]"
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/driver_1.json" 2> "$O/driver_1.err" \
  || { echo "bench failed"; tail -30 "$O/driver_1.err"; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); c=d['rank0_host_cpu_cores_by_thread']['vep-parse']; print({k: d.get(k) for k in ('value','ms_per_step','frames_dropped','p50_latency_ms','p99_latency_ms','rank0_gpu_kernel_ms_per_step','vs_baseline')}, 'parse core-ms/picture', round(c * d['ms_per_step'] * d['steps'] / d['frames_decoded'], 3))" "$O/driver_1.json"
