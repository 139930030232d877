#!/bin/bash
# Round 6 driver A/B on one box: an earlier build
# (ab_so/head.so, in a copy of the tree) vs the tree, as the driver's command (without the
# reference-equivalent run) alternated 3 times each, then parse_ab at 1 thread x 4 cameras and 16 threads x 32 cameras.
# Output: gpurun_out/$TAG/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=$R/gpurun_out/${TAG:-r6ab}; mkdir -p "$O"
ALT=/tmp/vep_alt_$$
rm -rf "$ALT"; mkdir -p "$ALT"
tar --exclude=./gpurun_out --exclude=./ab_so -cf - . | tar -xf - -C "$ALT"
cp ab_so/head.so "$ALT"/video_edge_ai_proxy_amd/_vep.cpython-310-x86_64-linux-gnu.so
drv() {  # label dir
  ( cd "$2" && timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 --ref-cpu off > "$O/drv_$1.json" 2> "$O/drv_$1.err" ) \
    || { echo "bench $1 failed"; tail -20 "$O/drv_$1.err"; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); c=d['rank0_host_cpu_cores_by_thread']['vep-parse']; print(sys.argv[2], d['value'], 'fps', d['ms_per_step'], 'ms/step', 'parse core-ms/picture', round(c * d['ms_per_step'] * d['steps'] / d['frames_decoded'], 3), 'gpu', d['rank0_gpu_kernel_ms_per_step'])" "$O/drv_$1.json" "$1" | tee -a "$O/drivers.log"
}
for i in 1 2 3; do
  drv head_$i "$ALT" || exit 1
  drv tree_$i "$R" || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python -u tools/parse_ab.py --so ab_so/head.so --reps 4 2>&1 | tail -1 | sed "s/^/head 1t: /" | tee -a "$O/parse_ab.log" || exit 1
  timeout -k 10 300 python -u tools/parse_ab.py --reps 4 2>&1 | tail -1 | sed "s/^/tree 1t: /" | tee -a "$O/parse_ab.log" || exit 1
done
for i in 1 2; do
  timeout -k 10 300 python -u tools/parse_ab.py --so ab_so/head.so --reps 3 --threads 16 --cams 32 2>&1 | tail -1 | sed "s/^/head 16t: /" | tee -a "$O/parse_ab.log" || exit 1
  timeout -k 10 300 python -u tools/parse_ab.py --reps 3 --threads 16 --cams 32 2>&1 | tail -1 | sed "s/^/tree 16t: /" | tee -a "$O/parse_ab.log" || exit 1
done
rm -rf "$ALT"
