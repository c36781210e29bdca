#!/bin/bash
# Round-3: compact per-lane LDS (MOPS_LDS_COMPACT) -- full GPU suite on the product build, then A/B
# against the 13-KB layout (ldsfull) on every trajectory mode and configs 3/4.
set -u
export TMPDIR=/tmp MOPS_BENCH_NO_RK4=1
out=gpurun_out/ldsc; mkdir -p $out
timeout -k 10 800 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo pytest failed; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
OUT=$out/se ROUNDS=2 BENCH_ARGS="--steps 3 --warmup 1" bash tools/var_ab.sh base ldsfull || exit 1
OUT=$out/pe ROUNDS=2 BENCH_ARGS="--mode pathline --steps 3 --warmup 1" bash tools/var_ab.sh base ldsfull || exit 1
OUT=$out/c4 ROUNDS=2 BENCH_ARGS="--config 4 --pairs 2 --steps 1 --warmup 1" bash tools/var_ab.sh base ldsfull || exit 1
OUT=$out/c3 ROUNDS=1 BENCH_ARGS="--config 3 --pairs 1 --steps 1 --warmup 1" bash tools/var_ab.sh base ldsfull || exit 1
OUT=$out/sr ROUNDS=1 BENCH_ARGS="--method rk4 --steps 2 --warmup 1" bash tools/var_ab.sh base ldsfull || exit 1
