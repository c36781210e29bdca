#!/bin/bash
# Time bench.py for the base library and each build/variants/libmops_<name>.so
# (perf experiments; results are comparable within one call = one device).
for v in base "$@"; do
  if [ "$v" = base ]; then unset MOPS_TRAJ_LIB; else export MOPS_TRAJ_LIB=$PWD/build/variants/libmops_$v.so; fi
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 2 ${BENCH_ARGS:-} > gpurun_out/var_$v.log 2>&1 || { echo "$v failed"; exit 1; }
  echo "$v ok"
done
