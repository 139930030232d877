set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
for w in 0 8; do
  VEP_HEVC_TU_WINDOW=$w timeout -s KILL 200 rocprofv3 --pmc $P1 -d "$R/gpurun_out/pmchw$w" -o pmc -- python3 "$R/bench.py" --codec h265 --source replay --steps 12 --warmup 3 --latency-samples 0 --clients 0 > "$R/gpurun_out/pmchw$w.log" 2>&1
  echo "window $w rc=$? $(grep -o 'frames dropped[^"]*' $R/gpurun_out/pmchw$w.log | head -1) $(grep -o '"frames_dropped": [0-9]*' $R/gpurun_out/pmchw$w.log)"
  rm -rf "$R/gpurun_out/pmchw$w"
done
