#!/bin/bash
# Round 5 hardware counters of the headline kernels (H.264 High 1080p, the live RTSP bench) and the
# H.265 4K shape: four passes, each within one block's counter limits (8 SQ; 4 TCC, FETCH_SIZE
# taking 3 and WRITE_SIZE 2), summarised by tools/rocpd_pmc_summary.py, which fails when a
# required ratio's counters are missing. Output: gpurun_out/r5pmc/pmc_<shape>.txt
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/r5pmc
mkdir -p "$O"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS"
P2="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT"
P3="FETCH_SIZE"
P4="WRITE_SIZE TCC_HIT_sum TCC_MISS_sum"
run() {  # name, bench args
  local name=$1; shift
  cd /tmp && export TMPDIR=/tmp
  for k in 1 2 3 4; do
    local C=P$k
    timeout -s KILL 240 rocprofv3 --pmc ${!C} -d "$O/${name}_p$k" -o pmc -- python3 "$R/bench.py" "$@" \
      > "$O/${name}_p$k.log" 2>&1 || { echo "pmc $name pass $k failed"; tail -20 "$O/${name}_p$k.log"; exit 1; }
    echo "$name pass $k ok"
  done
  cd "$R"
  python3 tools/rocpd_pmc_summary.py --require valu_per_wave_cycle,wait_per_wave_cycle,lds_bank_conflicts_per_lds_inst,l2_hit_rate \
    $(find "$O/${name}_p1" "$O/${name}_p2" "$O/${name}_p3" "$O/${name}_p4" -name "*.db") > "$O/pmc_${name}.txt" \
    || { echo "summary failed"; cat "$O/pmc_${name}.txt"; exit 1; }
  rm -rf "$O/${name}_p1" "$O/${name}_p2" "$O/${name}_p3" "$O/${name}_p4"
  cat "$O/pmc_${name}.txt"
}
run h264_1080p --steps 2 --warmup 1 --clients 0 --latency-samples 0
run h265_4k --codec h265 --width 3840 --height 2160 --cams-per-gpu 8 --steps 1 --warmup 1 --clients 0 --latency-samples 0
echo "[pmc] done"
