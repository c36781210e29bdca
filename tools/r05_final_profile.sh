# round 5, final build: profiles of the default line (config 3, Euler) and of its RK4 companion chain
set -o pipefail
export TMPDIR=/tmp
bash tools/profile_round.sh gpurun_out/r05p/c3 || exit 3
BENCH_ARGS="--method rk4" bash tools/profile_round.sh gpurun_out/r05p/c3rk4 || exit 4
