#!/bin/bash
# H.265 end to end on one box: the tree (sparse transform-block coefficients) vs the dense-record
# build (tools/abso/vep_dense.so), alternated, 32 x 1080p and 8 x 4K through the RTSP farm.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-hsab}; mkdir -p "$O"
SO=video_edge_ai_proxy_amd/_vep.cpython-310-x86_64-linux-gnu.so
cp "$SO" /tmp/vep_tree.so
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --codec h265 --latency-samples 0 --clients 0 "$@" > "$O/$n.json" 2> "$O/$n.err" \
    || { echo "$n failed"; tail -20 "$O/$n.err"; cp /tmp/vep_tree.so "$SO"; exit 1; }
  python -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d.get('rank0_gpu_kernel_ms_per_step'))"
}
for i in 1 2; do
  cp /tmp/vep_tree.so "$SO"
  run h265_1080p_sparse_$i --steps 60 --warmup 8
  run h265_4k_sparse_$i --width 3840 --height 2160 --cams-per-gpu 8 --steps 40 --warmup 6
  cp tools/abso/vep_dense.so "$SO"
  run h265_1080p_dense_$i --steps 60 --warmup 8
  run h265_4k_dense_$i --width 3840 --height 2160 --cams-per-gpu 8 --steps 40 --warmup 6
done
cp /tmp/vep_tree.so "$SO"
