#!/bin/bash
# Collect PMC counter passes for the trajectory kernel (one counter group per
# rocprofv3 pass; never combined with tracing domains).  Usage:
#   tools/pmc.sh OUTDIR "GROUP1" "GROUP2" ...   (each group: space-separated counters)
set -u
out=$1; shift
export TMPDIR=/tmp
# the counter passes must see only the measured workload's kernels (bench.py's RK4 companion off)
export MOPS_BENCH_NO_RK4=1
i=0
mkdir -p "$out"
for grp in "$@"; do
  i=$((i+1))
  timeout -k 5 120 rocprofv3 --pmc $grp --kernel-include-regex traj_kernel --output-format csv \
      -d "$out/pass$i" -o p -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ${BENCH_ARGS:-} \
      > "$out/pass$i.log" 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo "pmc done"
