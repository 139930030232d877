#!/bin/bash
# Round 6: does the parse throughput depend on how the parse threads land on physical cores?
# The box's CPU share is a cgroup quota (16 CPUs) over a NUMA node's 64 cores / 128 SMT threads;
# the host domain pins threads to the whole node and lets the scheduler place them.
set -u
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out/${TAG:-r6b}
mkdir -p "$O"
python tools/cpu_load.py | tee "$O/cpu_load_before.txt"
run() {  # name, env
  echo "[b] $1"
  env $2 timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --clients 0 --latency-samples 0 > "$O/$1.json" 2> "$O/$1.err" \
    || { echo "bench $1 failed"; tail -20 "$O/$1.err"; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print({k: d.get(k) for k in ('value','rank0_gpu_kernel_ms_per_step','parse_threads_per_rank','rank0_host_domain','rank0_host_cpu_cores_by_thread')})" "$O/$1.json"
}
run default "X=1"
run cores16 "VEP_HOST_CPUS=0-15"
run smt8x2 "VEP_HOST_CPUS=0-7,128-135"
run cores16b "VEP_HOST_CPUS=16-31"
run default2 "X=1"
python tools/cpu_load.py | tee "$O/cpu_load_after.txt"
echo "[b] done"
