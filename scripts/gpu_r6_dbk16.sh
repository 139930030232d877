#!/bin/bash
# Round 6: deblocking wavefront with 16 MB rows per workgroup (8 waves; ab_so/dbk16.so, built
# with -DVEP_DBK_WG_ROWS=16) vs the default 8: the H.264 GPU tests on the variant (bit-exact),
# then the GPU-side ceiling (--source records) at 32 and 64 cameras, alternated.
# Output: gpurun_out/$TAG/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=$R/gpurun_out/${TAG:-r6dbk16}; mkdir -p "$O"
ALT=/tmp/vep_alt_$$
rm -rf "$ALT"; mkdir -p "$ALT"
tar --exclude=./gpurun_out --exclude=./ab_so -cf - . | tar -xf - -C "$ALT"
cp ab_so/dbk16.so "$ALT"/video_edge_ai_proxy_amd/_vep.cpython-310-x86_64-linux-gnu.so
echo "[dbk16] GPU H.264 tests on the variant"
( cd "$ALT" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread \
    -k "avc or h264 or high or records or smoke or integration" > "$O/pytest_dbk16.log" 2>&1 ) \
  || { echo "variant GPU tests failed"; tail -30 "$O/pytest_dbk16.log"; exit 1; }
tail -2 "$O/pytest_dbk16.log"
rec() {  # label dir cams
  ( cd "$2" && timeout -k 10 400 python -u bench.py --source records --cams-per-gpu $3 --steps 10 --warmup 2 \
      --latency-samples 0 --ref-cpu off > "$O/rec_$1_c$3.json" 2> "$O/rec_$1_c$3.err" ) \
    || { echo "records $1 $3 failed"; tail -20 "$O/rec_$1_c$3.err"; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], 'cams', sys.argv[3], d['value'], 'pictures/s', d['ms_per_step'], 'ms/step gpu', d.get('rank0_gpu_kernel_ms_per_step'))" "$O/rec_$1_c$3.json" "$1" "$3" | tee -a "$O/summary.log"
}
for i in 1 2; do
  for C in 32 64; do
    rec base "$R" $C || exit 1
    rec dbk16 "$ALT" $C || exit 1
  done
done
rm -rf "$ALT"
