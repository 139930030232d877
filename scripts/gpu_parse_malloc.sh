#!/bin/bash
# Replay parse pool (no GPU work) at 1 and 14 threads, default glibc malloc vs fixed mmap / trim
# thresholds (allocation page-fault hypothesis).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
echo "default malloc:"; PROFILE=high timeout -k 10 200 python -u scripts/parse_scaling.py 32 1 14 || exit 1
echo "mmap/trim thresholds 32M/1G:"; MALLOC_MMAP_THRESHOLD_=33554432 MALLOC_TRIM_THRESHOLD_=1073741824 PROFILE=high timeout -k 10 200 python -u scripts/parse_scaling.py 32 1 14 || exit 1
