#!/bin/bash
# Round-3: fewer LDS normal slots (MOPS_NRM_SLOTS 5 / 4: the rest computed per evaluation).
set -u
export TMPDIR=/tmp MOPS_BENCH_NO_RK4=1
out=gpurun_out/nrm; mkdir -p $out
MOPS_TRAJ_LIB=$PWD/build/variants/libmops_nrm4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo pytest failed; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
OUT=$out/pe ROUNDS=2 BENCH_ARGS="--mode pathline --steps 3 --warmup 1" bash tools/var_ab.sh base nrm5 nrm4 || exit 1
OUT=$out/c4 ROUNDS=1 BENCH_ARGS="--config 4 --pairs 2 --steps 1 --warmup 1" bash tools/var_ab.sh base nrm5 nrm4 || exit 1
OUT=$out/se ROUNDS=2 BENCH_ARGS="--steps 3 --warmup 1" bash tools/var_ab.sh base nrm5 nrm4 || exit 1
