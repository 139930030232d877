#!/bin/bash
# rocprofv3 kernel statistics of the three shapes the round-3 kernel work targets: the headline
# (32 x 1080p H.264 High over RTSP), keyframe-only (BASELINE config 3) and 32 x 1080p H.265, each
# summarised per kernel into gpurun_out/$TAG/kernel_stats_<name>.csv. PMC=1 adds two SQ counter
# passes of the keyframe-only shape (the intra / deblocking wavefronts).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
O=gpurun_out/${TAG:-r3prof}
mkdir -p "$O"
export TMPDIR=/tmp
prof() {  # name, bench args...
  local n=$1; shift
  cd /tmp
  timeout -k 10 300 rocprofv3 --kernel-trace -d "$R/$O/db_$n" -o run -- python3 "$R/bench.py" "$@" \
    > "$R/$O/prof_$n.json" 2> "$R/$O/prof_$n.err" || { echo "rocprof $n failed"; tail -20 "$R/$O/prof_$n.err"; exit 1; }
  cd "$R"
  python3 tools/rocpd_kernel_stats.py "$O/db_$n" > "$O/kernel_stats_$n.csv" || { echo "stats $n failed"; exit 1; }
  rm -rf "$O/db_$n"
  head -8 "$O/kernel_stats_$n.csv"
}
prof headline --steps 30 --warmup 5 --latency-samples 0 --clients 0
prof keyframe_only --keyframe-only --steps 40 --warmup 6 --latency-samples 0 --clients 0
prof h265_1080p --codec h265 --source replay --steps 40 --warmup 6 --latency-samples 0 --clients 0
if [ "${PMC:-0}" = "1" ]; then
  P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
  P2="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM"
  for k in 1 2; do
    C=P$k
    cd /tmp
    timeout -s KILL 200 rocprofv3 --pmc ${!C} -d "$R/$O/pmc_p$k" -o pmc -- python3 "$R/bench.py" --keyframe-only --steps 12 --warmup 3 \
      --latency-samples 0 --clients 0 > "$R/$O/pmc_p$k.log" 2>&1 || { echo "pmc pass $k failed"; tail -20 "$R/$O/pmc_p$k.log"; exit 1; }
    cd "$R"
  done
  python3 tools/rocpd_pmc_summary.py $(find "$O/pmc_p1" "$O/pmc_p2" -name "*.db") > "$O/pmc_keyframe_only.csv" \
    || { echo "pmc summary failed"; exit 1; }
  rm -rf "$O/pmc_p1" "$O/pmc_p2"
  cat "$O/pmc_keyframe_only.csv"
fi
echo "[prof] done"
