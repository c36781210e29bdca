#!/bin/bash
# Round 6 GPU driver: STAGE selects what runs (one gpurun call per stage).
#   stall   class prices (fp64bench) + stall decomposition of the tiled RK4 and Euler pathline kernels
set -u
export TMPDIR=/tmp
O=gpurun_out/r06${TAG:-}
mkdir -p $O
case "${STAGE:-stall}" in
stall)
  bash tools/fp64bench.sh $O/fp64bench || exit 2
  python3 tools/fp64bench_summary.py $O/fp64bench > $O/fp64bench/summary.txt; cat $O/fp64bench/summary.txt
  BENCH_ARGS="--method rk4" bash tools/pmc_stall.sh $O/stall_rk4 || exit 3
  python3 tools/pmc_means.py $O/stall_rk4 "void traj_kernel<7, true, false, true>" 240 > $O/stall_rk4/summary.txt
  bash tools/pmc_stall.sh $O/stall_euler || exit 4
  python3 tools/pmc_means.py $O/stall_euler "void traj_kernel<7, true, true, true>" 1440 > $O/stall_euler/summary.txt
  tail -12 $O/stall_rk4/summary.txt $O/stall_euler/summary.txt
  ;;
esac
