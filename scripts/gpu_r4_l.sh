#!/bin/bash
# Round 4 closing run: the H.264 wavefront phase clocks (VEP_AVC_PROF=1: cycles per macroblock
# in wait / load / filter / store for the intra and deblocking wavefronts), the PAFF IBBP farm
# with the batched weave, and the headline bench as the driver runs it (and over 200 steps).
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r4l}
mkdir -p "$O"
echo "[l] avc phase clocks"
VEP_AVC_PROF=1 timeout -k 10 300 python -u bench.py --steps 60 --warmup 10 --clients 0 --latency-samples 0 \
  > "$O/avc_prof.json" 2> "$O/avc_prof.err" || { echo "avc prof failed"; tail -20 "$O/avc_prof.err"; exit 1; }
python -c "import json,sys; d=json.loads(open('$O/avc_prof.json').read().strip().splitlines()[-1]); print(json.dumps({k: v for k, v in d.items() if 'prof' in k or 'cycles' in k})[:1500])"
echo "[l] PAFF IBBP farm"
timeout -k 10 400 python -u bench.py --steps 200 --warmup 20 --interlaced 2 > "$O/bench_paff_ibbp.json" 2> "$O/bench_paff.err" \
  || { echo "paff bench failed"; tail -30 "$O/bench_paff.err"; exit 1; }
cut -c1-300 "$O/bench_paff_ibbp.json"
echo "[l] headline (driver command)"
timeout -k 10 400 python -u bench.py --gpus 1 --steps 20 --warmup 5 > "$O/headline.json" 2> "$O/headline.err" \
  || { echo "headline failed"; tail -30 "$O/headline.err"; exit 1; }
cut -c1-300 "$O/headline.json"
echo "[l] headline 200 steps"
timeout -k 10 400 python -u bench.py --gpus 1 --steps 200 --warmup 20 > "$O/headline_200.json" 2> "$O/headline_200.err" \
  || { echo "headline 200 failed"; tail -30 "$O/headline_200.err"; exit 1; }
cut -c1-300 "$O/headline_200.json"
echo "[l] done"
