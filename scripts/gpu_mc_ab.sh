#!/bin/bash
# A/B of the H.265 motion compensation kernels on one box: the LDS-staged separable kernel
# (default) vs the per-sample one (VEP_HEVC_MC_DIRECT=1), rocprofv3 kernel statistics of the
# same replay bench (1080p x 32 and 4K x 8), twice each in alternation.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
O=gpurun_out/${TAG:-mcab}
mkdir -p "$O"
export TMPDIR=/tmp
prof() {  # name, env, bench args...
  local n=$1 e=$2; shift 2
  cd /tmp
  env "$e" timeout -k 10 240 rocprofv3 --kernel-trace -d "$R/$O/db_$n" -o run -- python3 "$R/bench.py" "$@" \
    > "$R/$O/$n.json" 2> "$R/$O/$n.err" || { echo "rocprof $n failed"; tail -20 "$R/$O/$n.err"; exit 1; }
  cd "$R"
  python3 tools/rocpd_kernel_stats.py "$O/db_$n" > "$O/kernel_stats_$n.csv" || { echo "stats $n failed"; exit 1; }
  rm -rf "$O/db_$n"
  echo "$n $(grep -h hevc_mc "$O/kernel_stats_$n.csv" | cut -d, -f2-4)"
}
for rep in 1 2; do
  for v in staged direct; do
    e=VEP_HEVC_MC_DIRECT=0; [ $v = direct ] && e=VEP_HEVC_MC_DIRECT=1
    prof h265_1080p_${v}_$rep $e --codec h265 --source replay --steps 20 --warmup 4 --latency-samples 0 --clients 0
    prof h265_4k_${v}_$rep $e --codec h265 --source replay --width 3840 --height 2160 --cams-per-gpu 8 --steps 16 --warmup 3 --latency-samples 0 --clients 0
  done
done
echo "[mcab] done"
