#!/bin/bash
# H.265 queue windows (VEP_HEVC_TU_WINDOW=8) under the profiler: frames dropped with one GRBM
# counter, with the SQ counter pass, and with kernel tracing only (replay source, 12 steps).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --codec h265 --source replay --steps 12 --warmup 3 --latency-samples 0 --clients 0"
run() {  # name, rocprofv3 args...
  local n=$1; shift
  local start=$(date +%s)
  VEP_HEVC_TU_WINDOW=8 timeout -s KILL 200 rocprofv3 "$@" -d "$R/gpurun_out/pw_$n" -o p -- python3 $B > "$R/gpurun_out/pw_$n.log" 2>&1
  echo "$n rc=$? secs=$(( $(date +%s) - start )) $(grep -o '"frames_dropped": [0-9]*' $R/gpurun_out/pw_$n.log)"
  rm -rf "$R/gpurun_out/pw_$n"
}
run grbm --pmc GRBM_COUNT
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT
run ktrace --kernel-trace --stats
