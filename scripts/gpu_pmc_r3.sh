#!/bin/bash
# Round-3 hardware counters: H.264 High (replay, 32x1080p) and H.265 (32x1080p) kernels, two
# passes of <= 8 SQ counters each, summarised per kernel into gpurun_out/pmc_r3_{avc,hevc}.csv.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
P2="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM"
run() {  # name, bench args
  local name=$1; shift
  cd /tmp && export TMPDIR=/tmp
  for k in 1 2; do
    local C=P$k
    timeout -s KILL 200 rocprofv3 --pmc ${!C} -d "$R/gpurun_out/${name}_p$k" -o pmc -- python3 "$R/bench.py" "$@" \
      > "$R/gpurun_out/${name}_p$k.log" 2>&1 || { echo "pmc $name pass $k failed"; tail -20 "$R/gpurun_out/${name}_p$k.log"; exit 1; }
    echo "$name pass $k ok"
  done
  cd "$R"
  python3 tools/rocpd_pmc_summary.py $(find "gpurun_out/${name}_p1" "gpurun_out/${name}_p2" -name "*.db") \
    > "gpurun_out/pmc_r3_${name}.csv" || { echo "summary failed"; exit 1; }
  rm -rf "gpurun_out/${name}_p1" "gpurun_out/${name}_p2"
  cat "gpurun_out/pmc_r3_${name}.csv"
}
run avc --source replay --steps 12 --warmup 3 --latency-samples 0 --clients 0
run hevc --codec h265 --source replay --steps 12 --warmup 3 --latency-samples 0 --clients 0
