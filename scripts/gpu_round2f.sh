#!/bin/bash
# Hardware counters of the current H.264 kernels (High CABAC IBBP headline workload, 3 passes),
# then coded H.265 benches (4K x 8 cameras = BASELINE config 5 per-GPU slice, and 1080p x 32).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; mkdir -p gpurun_out
B="$R/bench.py --steps 12 --warmup 3 --latency-samples 0 --clients 0"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT \
  -d "$R/gpurun_out/pmc1" -o pmc -- python3 $B > "$R/gpurun_out/pmc1.log" 2>&1 || { echo "pmc pass 1 failed"; tail -20 "$R/gpurun_out/pmc1.log"; exit 1; }
echo pmc1 ok
timeout -s KILL 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SMEM \
  -d "$R/gpurun_out/pmc2" -o pmc -- python3 $B > "$R/gpurun_out/pmc2.log" 2>&1 || { echo "pmc pass 2 failed"; tail -20 "$R/gpurun_out/pmc2.log"; exit 1; }
echo pmc2 ok
timeout -s KILL 200 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE GRBM_COUNT \
  -d "$R/gpurun_out/pmc3" -o pmc -- python3 $B > "$R/gpurun_out/pmc3.log" 2>&1 || { echo "pmc pass 3 failed"; tail -20 "$R/gpurun_out/pmc3.log"; exit 1; }
echo pmc3 ok
cd "$R"
timeout -k 10 400 python -u bench.py --codec h265 --width 3840 --height 2160 --cams-per-gpu 8 --steps 40 --warmup 5 --gop 30 > gpurun_out/bench_h265_4k.json 2> gpurun_out/bench_h265_4k.err || { echo "bench h265 4k failed"; tail -30 gpurun_out/bench_h265_4k.err; exit 1; }
cat gpurun_out/bench_h265_4k.json
timeout -k 10 400 python -u bench.py --codec h265 --steps 60 --warmup 5 > gpurun_out/bench_h265_1080p.json 2> gpurun_out/bench_h265_1080p.err || { echo "bench h265 1080p failed"; tail -30 gpurun_out/bench_h265_1080p.err; exit 1; }
cat gpurun_out/bench_h265_1080p.json
