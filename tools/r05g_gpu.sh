# round 5: profile of config 4 (2 daily pairs) on the product build
set -o pipefail
export TMPDIR=/tmp
BENCH_ARGS="--config 4 --pairs 2" bash tools/profile_round.sh gpurun_out/r05g/c4 || exit 4
