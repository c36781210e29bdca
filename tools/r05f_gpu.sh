# round 5: profile of the config-3 RK4 chain (bench.py --method rk4) on the product build
set -o pipefail
export TMPDIR=/tmp
BENCH_ARGS="--method rk4" bash tools/profile_round.sh gpurun_out/r05f/c3rk4 || exit 4
