#!/bin/bash
# Single-thread parse A/B on the box CPU: the dense-record build vs the tree, alternated.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/${TAG:-pab}
for i in 1 2 3 4; do
  timeout -k 10 200 taskset -c 2 python tools/parse_ab.py --so tools/abso/vep_dense.so --reps 3 2>&1 | tail -1 | tee -a gpurun_out/${TAG:-pab}/parse_ab.log || exit 1
  timeout -k 10 200 taskset -c 2 python tools/parse_ab.py --reps 3 2>&1 | tail -1 | tee -a gpurun_out/${TAG:-pab}/parse_ab.log || exit 1
done
