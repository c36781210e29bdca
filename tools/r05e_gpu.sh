# round 5: coop Euler kernel at 2 waves/SIMD (wpe2) vs 3; then the config-3 profile of the product build
set -o pipefail
out=gpurun_out/r05e
mkdir -p $out
export TMPDIR=/tmp
MOPS_BENCH_NO_RK4=1 BENCH_ARGS="--steps 2 --warmup 1" OUT=$out/wpe ROUNDS=1 bash tools/var_ab.sh base wpe2 || exit 3
BENCH_ARGS="--steps 3 --warmup 1" bash tools/profile_round.sh $out/c3 || exit 4
cat $out/wpe/ab.txt
