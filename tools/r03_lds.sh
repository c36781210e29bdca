#!/bin/bash
# Round-3: is config 4's gain without the pathline pair test its LDS (occupancy)?  nopt vs nopt + the
# pair test's 2.5 KB of LDS as padding, and the product + 1 KB of padding.
set -u
export TMPDIR=/tmp MOPS_BENCH_NO_RK4=1
out=gpurun_out/lds; mkdir -p $out
OUT=$out/c4 ROUNDS=2 BENCH_ARGS="--config 4 --pairs 2 --steps 1 --warmup 1" bash tools/var_ab.sh base nopt noptpad pad1k || exit 1
OUT=$out/pe ROUNDS=2 BENCH_ARGS="--mode pathline --steps 3 --warmup 1" bash tools/var_ab.sh base nopt noptpad pad1k || exit 1
