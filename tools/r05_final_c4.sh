# round 5, final build: the config-4 profile (2 daily pairs)
set -o pipefail
export TMPDIR=/tmp
BENCH_ARGS="--config 4 --pairs 2" bash tools/profile_round.sh gpurun_out/r05p/c4 || exit 4
