#!/bin/bash
# Round 6: parse threads = the host domain's CPU share - 1 (15 of 16) vs the whole share (16):
# the one CPU left for ingest / worker / lanes measures ~0.2 cores busy in the timed region.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=gpurun_out/${TAG:-r6threads}; mkdir -p "$O"
for i in 1 2; do
  for t in 0 16; do
    n=threads${t}_$i
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --threads $t --clients 0 --latency-samples 0 --ref-cpu off \
      > "$O/$n.json" 2> "$O/$n.err" || { echo "$n failed"; tail -20 "$O/$n.err"; exit 1; }
    python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[2], {k: d.get(k) for k in ('value','rank0_gpu_kernel_ms_per_step','parse_threads_per_rank','rank0_host_cpu_cores_by_thread')})" "$O/$n.json" "$n"
  done
done
echo "[threads] done"
# clock of the busy cores: 1 vs 15 parse threads (tools/parse_ab.py), /proc/cpuinfo sampled mid-run
for t in 1 15; do
  c=$([ $t = 1 ] && echo 4 || echo 32)
  timeout -k 10 200 python -u tools/parse_ab.py --reps 6 --threads $t --cams $c > "$O/parse_t$t.log" 2>&1 &
  P=$!
  sleep 25
  python tools/cpu_mhz.py > "$O/mhz_t$t.txt" 2>&1
  wait $P || { echo "parse_ab $t failed"; tail -5 "$O/parse_t$t.log"; exit 1; }
  tail -1 "$O/parse_t$t.log"; cat "$O/mhz_t$t.txt"
done
echo "[threads] clocks done"
