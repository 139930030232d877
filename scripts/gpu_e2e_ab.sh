#!/bin/bash
# End-to-end A/B on one box: the headline bench (RTSP, 32 x 1080p H.264) with the tree's
# extension (sparse coefficient records) and with the dense-record build swapped in, alternated.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-e2eab}; mkdir -p "$O"
SO=video_edge_ai_proxy_amd/_vep.cpython-310-x86_64-linux-gnu.so
cp "$SO" /tmp/vep_sparse.so
run() {  # name
  timeout -k 10 300 python -u bench.py --steps ${STEPS:-100} --warmup 10 --latency-samples 0 --clients 0 ${ARGS:-} \
    > "$O/$1.json" 2> "$O/$1.err" || { echo "$1 failed"; tail -20 "$O/$1.err"; cp /tmp/vep_sparse.so "$SO"; exit 1; }
  python -c "import json; d=json.loads(open('$O/$1.json').read().strip().splitlines()[-1]); print('$1', d['value'], d['ms_per_step'], d.get('rank0_gpu_kernel_ms_per_step'), d.get('rank0_record_bytes_gathered_per_step'))"
}
for i in 1 2; do
  cp /tmp/vep_sparse.so "$SO"; run sparse_$i
  cp tools/abso/vep_dense.so "$SO"; run dense_$i
done
cp /tmp/vep_sparse.so "$SO"
