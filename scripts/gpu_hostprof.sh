#!/bin/bash
# In-situ host profiles of the replay parse pool on the box CPU: 1 thread and 14 threads.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
PROFILE=high timeout -k 10 300 python -u tools/hostprof_parse.py gpurun_out/hostprof_t14.txt 14 32 300 || exit 1
PROFILE=high timeout -k 10 300 python -u tools/hostprof_parse.py gpurun_out/hostprof_t1.txt 1 32 20 || exit 1
