#!/bin/bash
# Multi-thread parse throughput on the box CPU (15 threads, 32 cameras): dense-record build vs
# the tree, alternated.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out/${TAG:-pab3}
for i in 1 2 3; do
  timeout -k 10 240 python tools/parse_ab.py --so tools/abso/vep_dense.so --reps 3 --threads 15 --cams 32 2>&1 | tail -1 | tee -a gpurun_out/${TAG:-pab3}/parse_ab.log || exit 1
  timeout -k 10 240 python tools/parse_ab.py --reps 3 --threads 15 --cams 32 2>&1 | tail -1 | tee -a gpurun_out/${TAG:-pab3}/parse_ab.log || exit 1
done
