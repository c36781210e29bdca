#!/bin/bash
# Round-3: config-2 schedule re-sweep on the current kernel, and pathline record grouping variants.
set -u
export TMPDIR=/tmp MOPS_BENCH_NO_RK4=1
out=gpurun_out/sweep; mkdir -p $out
OUT=$out/sched ROUNDS=2 bash tools/ab.sh "--chunks 6" "--chunks 4" "--chunks 8" "--parts 3 --chunks 6" || exit 1
OUT=$out/pe ROUNDS=2 BENCH_ARGS="--mode pathline --steps 3 --warmup 1" bash tools/var_ab.sh base gr1pe hexpairs0 || exit 1
OUT=$out/c3 ROUNDS=1 BENCH_ARGS="--config 3 --pairs 1 --steps 1 --warmup 1" bash tools/var_ab.sh base gr1pe hexpairs0 || exit 1
