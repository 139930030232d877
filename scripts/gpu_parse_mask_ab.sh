#!/bin/bash
# Single-thread and 15-thread parse throughput on the box CPU: the tree (non-zero masks built in
# the macroblock layer) vs the previous build (masks computed in store_mb), alternated.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-pmask}; mkdir -p "$O"
for i in 1 2 3; do
  timeout -k 10 240 python tools/parse_ab.py --so tools/ab_parse/vep_base.so --reps 4 2>&1 | tail -1 | sed 's/^/base 1t: /' | tee -a "$O/parse_ab.log" || exit 1
  timeout -k 10 240 python tools/parse_ab.py --reps 4 2>&1 | tail -1 | sed 's/^/mask 1t: /' | tee -a "$O/parse_ab.log" || exit 1
done
for i in 1 2; do
  timeout -k 10 240 python tools/parse_ab.py --so tools/ab_parse/vep_base.so --reps 3 --threads 15 --cams 32 2>&1 | tail -1 | sed 's/^/base 15t: /' | tee -a "$O/parse_ab.log" || exit 1
  timeout -k 10 240 python tools/parse_ab.py --reps 3 --threads 15 --cams 32 2>&1 | tail -1 | sed 's/^/mask 15t: /' | tee -a "$O/parse_ab.log" || exit 1
done
