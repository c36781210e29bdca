#!/bin/bash
# Round-3: the pathline pair test on the oRRS18to6-class config 4 vs the config-2 mesh (walk counters,
# SQ counters, interleaved timing).
set -u
export TMPDIR=/tmp MOPS_BENCH_NO_RK4=1
out=gpurun_out/pt; mkdir -p $out
for args in "--config 4 --pairs 1" "--mode pathline"; do
  tag=$(echo $args | tr -d ' -')
  for v in prof profnopt; do
    MOPS_PROF_SECTIONS=1 MOPS_TRAJ_LIB=$PWD/build/variants/libmops_$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --steps 1 --warmup 0 $args > $out/${tag}_$v.json 2> $out/${tag}_$v.err || { echo "$v failed"; tail -5 $out/${tag}_$v.err; exit 1; }
    echo "$tag $v $(grep 'prof counters' $out/${tag}_$v.err)"
  done
done
OUT=$out/pmc4 BENCH_ARGS="--config 4 --pairs 1" bash tools/pmc_variants.sh base nopt || exit 1
OUT=$out/ab4 ROUNDS=2 BENCH_ARGS="--config 4 --pairs 2 --steps 1 --warmup 1" bash tools/var_ab.sh base nopt || exit 1
