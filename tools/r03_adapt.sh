#!/bin/bash
# Round-3: the per-wave pair-test switch (MOPS_PAIR_ADAPT) against always-on (noadapt) and
# pathline-off (nopt): parity of the product build, walk counters, interleaved timing.
set -u
export TMPDIR=/tmp MOPS_BENCH_NO_RK4=1
out=gpurun_out/adapt; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_chain.py -x -q -m gpu --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo pytest failed; tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
for args in "--config 4 --pairs 1" "--mode pathline"; do
  tag=$(echo $args | tr -d ' -')
  MOPS_PROF_SECTIONS=1 MOPS_TRAJ_LIB=$PWD/build/variants/libmops_profad.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 1 --warmup 0 $args > $out/${tag}_profad.json 2> $out/${tag}_profad.err || { echo "prof failed"; exit 1; }
  echo "$tag $(grep 'prof counters' $out/${tag}_profad.err)"
done
OUT=$out/c4 ROUNDS=2 BENCH_ARGS="--config 4 --pairs 2 --steps 1 --warmup 1" bash tools/var_ab.sh base noadapt nopt || exit 1
OUT=$out/c3 ROUNDS=1 BENCH_ARGS="--config 3 --pairs 1 --steps 1 --warmup 1" bash tools/var_ab.sh base noadapt || exit 1
OUT=$out/pe ROUNDS=2 BENCH_ARGS="--mode pathline --steps 3 --warmup 1" bash tools/var_ab.sh base noadapt || exit 1
OUT=$out/se ROUNDS=2 BENCH_ARGS="--steps 3 --warmup 1" bash tools/var_ab.sh base noadapt || exit 1
