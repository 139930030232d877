#!/bin/bash
# Round 6: BASELINE config 5 shape (8 x 4K30 H.265 Main, 8 slices per picture, RTSP) on the
# round-start build (ab_so/head.so, commit 446a660, in a copy of the tree) vs the tree — the
# H.265 parse shares the CABAC engine (cabac.h) changed in round 6. Alternated twice.
# Output: gpurun_out/$TAG/.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=$R/gpurun_out/${TAG:-r6h265}; mkdir -p "$O"
ALT=/tmp/vep_alt_$$
rm -rf "$ALT"; mkdir -p "$ALT"
tar --exclude=./gpurun_out --exclude=./ab_so -cf - . | tar -xf - -C "$ALT"
cp ab_so/head.so "$ALT"/video_edge_ai_proxy_amd/_vep.cpython-310-x86_64-linux-gnu.so
run() {  # label dir
  ( cd "$2" && timeout -k 10 400 python -u bench.py --codec h265 --width 3840 --height 2160 --cams-per-gpu 8 \
      --steps 20 --warmup 3 --ref-cpu off > "$O/h265_$1.json" 2> "$O/h265_$1.err" ) \
    || { echo "h265 $1 failed"; tail -20 "$O/h265_$1.err"; return 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); c=d['rank0_host_cpu_cores_by_thread']; print(sys.argv[2], d['value'], 'fps', d['ms_per_step'], 'ms/step', 'dropped', d.get('frames_dropped'), 'p50/p99', d.get('p50_latency_ms'), d.get('p99_latency_ms'), 'cores', c)" "$O/h265_$1.json" "$1" | tee -a "$O/summary.log"
}
for i in 1 2; do
  run start_$i "$ALT" || exit 1
  run tree_$i "$R" || exit 1
done
rm -rf "$ALT"
