#!/bin/bash
# Round 5 parse A/B on the box CPU: the tree vs the build kept in tools/ab_parse/vep_base.so,
# alternated — 1 parse thread x 4 cameras and 15 threads x 32 cameras (CABAC bins / picture and
# TSC cycles / bin per line). Output: gpurun_out/$TAG/parse_ab.log.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-r5parse}; mkdir -p "$O"
for i in 1 2 3; do
  timeout -k 10 240 python tools/parse_ab.py --so tools/ab_parse/vep_base.so --reps 4 2>&1 | tail -1 | sed 's/^/base 1t: /' | tee -a "$O/parse_ab.log" || exit 1
  timeout -k 10 240 python tools/parse_ab.py --reps 4 2>&1 | tail -1 | sed 's/^/tree 1t: /' | tee -a "$O/parse_ab.log" || exit 1
done
for i in 1 2; do
  timeout -k 10 240 python tools/parse_ab.py --so tools/ab_parse/vep_base.so --reps 3 --threads 15 --cams 32 2>&1 | tail -1 | sed 's/^/base 15t: /' | tee -a "$O/parse_ab.log" || exit 1
  timeout -k 10 240 python tools/parse_ab.py --reps 3 --threads 15 --cams 32 2>&1 | tail -1 | sed 's/^/tree 15t: /' | tee -a "$O/parse_ab.log" || exit 1
done
