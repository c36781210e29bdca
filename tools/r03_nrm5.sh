#!/bin/bash
# Round-3: MOPS_NRM_SLOTS 5 (product) vs 6 -- full GPU suite, then the RK4 modes and config 3.
set -u
export TMPDIR=/tmp MOPS_BENCH_NO_RK4=1
out=gpurun_out/nrm5; mkdir -p $out
timeout -k 10 800 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest.log 2>&1 || { echo pytest failed; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
OUT=$out/se ROUNDS=2 BENCH_ARGS="--steps 3 --warmup 1" bash tools/var_ab.sh base nrm6 || exit 1
OUT=$out/sr ROUNDS=2 BENCH_ARGS="--method rk4 --steps 2 --warmup 1" bash tools/var_ab.sh base nrm6 || exit 1
OUT=$out/pr ROUNDS=1 BENCH_ARGS="--method rk4 --mode pathline --steps 2 --warmup 1" bash tools/var_ab.sh base nrm6 || exit 1
OUT=$out/c3 ROUNDS=1 BENCH_ARGS="--config 3 --pairs 1 --steps 1 --warmup 1" bash tools/var_ab.sh base nrm6 || exit 1
