#!/bin/bash
# Config-3 measurement: full 7-day chained-pathline bench with CPU baseline,
# rocprofv3 kernel stats of one bench step, FETCH/WRITE PMC passes on one pair.
set -u
out=${1:-gpurun_out/c3}
mkdir -p "$out"
export TMPDIR=/tmp
# the counter passes must see only the measured workload's kernels (bench.py's RK4 companion off)
export MOPS_BENCH_NO_RK4=1
timeout -k 10 400 python3 bench.py --config 3 --steps 1 --warmup 1 > "$out/bench.json" 2> "$out/bench.err" || { echo "bench failed"; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/stats" -o p -- \
    python3 bench.py --config 3 --steps 1 --warmup 0 --no-cpu-baseline > "$out/stats.log" 2>&1 || { echo "stats failed"; exit 1; }
timeout -k 5 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex traj_kernel --output-format csv -d "$out/fetch" -o p -- \
    python3 bench.py --config 3 --pairs 1 --steps 1 --warmup 0 --no-cpu-baseline > "$out/fetch.log" 2>&1 || { echo "fetch failed"; exit 1; }
timeout -k 5 200 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex traj_kernel --output-format csv -d "$out/write" -o p -- \
    python3 bench.py --config 3 --pairs 1 --steps 1 --warmup 0 --no-cpu-baseline > "$out/write.log" 2>&1 || { echo "write failed"; exit 1; }
echo "profile config3 ok"
