#!/bin/bash
# Host parse under CPU contention on the box: K concurrent single-threaded parse_bench
# processes (separate decoders, as the parse pool's threads are), per-process ms/frame.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
B=${1:-tools/bin/pb_new}
for K in 1 4 8 12 16; do
  for i in $(seq 1 $K); do timeout -k 5 200 $B high 30 3 > gpurun_out/pc_${K}_${i}.log 2>&1 & done
  wait
  echo -n "K=$K: "; cat gpurun_out/pc_${K}_*.log | grep "best of" | awk '{s+=$5; n++} END {printf "%.3f ms/frame avg over %d procs\n", s/n, n}'
  rm -f gpurun_out/pc_${K}_*.log
done
