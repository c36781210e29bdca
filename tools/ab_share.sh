#!/bin/bash
# Round-3 experiment: pathline record sharing (MOPS_SHARE_P) -- parity of the variant, then A/B.
set -u
export TMPDIR=/tmp MOPS_BENCH_NO_RK4=1
out=gpurun_out/share; mkdir -p $out
MOPS_TRAJ_LIB=$PWD/build/variants/libmops_share.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_chain.py -x -q -m gpu -k "path or chain" --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo pytest failed; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
OUT=$out/pe ROUNDS=2 BENCH_ARGS="--mode pathline --steps 3 --warmup 1" bash tools/var_ab.sh base share sharept nopt || exit 1
OUT=$out/c3 ROUNDS=1 BENCH_ARGS="--config 3 --pairs 1 --steps 1 --warmup 1" bash tools/var_ab.sh base share sharept nopt || exit 1
OUT=$out/c4 ROUNDS=1 BENCH_ARGS="--config 4 --pairs 2 --steps 1 --warmup 1" bash tools/var_ab.sh base share nopt || exit 1
