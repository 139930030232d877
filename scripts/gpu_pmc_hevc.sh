#!/bin/bash
# Hardware counters of the H.265 kernels (32x1080p H.265 bench), two passes of <= 8 SQ counters.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
B="$R/bench.py --codec h265 --steps 12 --warmup 3 --latency-samples 0 --clients 0"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
  -d "$R/gpurun_out/hpmc1" -o pmc -- python3 $B > "$R/gpurun_out/hpmc1.log" 2>&1 || { echo "pmc pass 1 failed"; tail -20 "$R/gpurun_out/hpmc1.log"; exit 1; }
echo hpmc1 ok
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM \
  -d "$R/gpurun_out/hpmc2" -o pmc -- python3 $B > "$R/gpurun_out/hpmc2.log" 2>&1 || { echo "pmc pass 2 failed"; tail -20 "$R/gpurun_out/hpmc2.log"; exit 1; }
echo hpmc2 ok
cd "$R"
python3 tools/rocpd_pmc_summary.py $(find gpurun_out/hpmc1 gpurun_out/hpmc2 -name "*.db") > gpurun_out/pmc_hevc_kernels.csv || { echo "summary failed"; exit 1; }
rm -rf gpurun_out/hpmc1 gpurun_out/hpmc2
cat gpurun_out/pmc_hevc_kernels.csv
