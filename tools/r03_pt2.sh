#!/bin/bash
# Round-3: the pair test again at the compact LDS layout (streamline: ptoff; pathline: ptpoff).
set -u
export TMPDIR=/tmp MOPS_BENCH_NO_RK4=1
out=gpurun_out/pt2; mkdir -p $out
OUT=$out/se ROUNDS=2 BENCH_ARGS="--steps 3 --warmup 1" bash tools/var_ab.sh base ptoff || exit 1
OUT=$out/pe ROUNDS=2 BENCH_ARGS="--mode pathline --steps 3 --warmup 1" bash tools/var_ab.sh base ptpoff || exit 1
OUT=$out/c4 ROUNDS=1 BENCH_ARGS="--config 4 --pairs 2 --steps 1 --warmup 1" bash tools/var_ab.sh base ptpoff || exit 1
OUT=$out/c3 ROUNDS=1 BENCH_ARGS="--config 3 --pairs 1 --steps 1 --warmup 1" bash tools/var_ab.sh base ptpoff || exit 1
