#!/bin/bash
# A/B of host parse binaries on the GPU box's CPU (single thread, High CABAC 1080p):
# every tools/bin/pb_* binary, alternated 3 times.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
for i in 1 2 3; do
  for b in tools/bin/pb_*; do
    echo "== $b"
    timeout -k 5 120 taskset -c 2 "$b" high 30 3 | grep -E "best|  [PBI]:|parse" || exit 1
  done
done
