# round 5, final build: the config-4 profile, then the driver's default command (its line carries the
# config-3 Euler and RK4 rooflines from this build's PMC entries)
set -o pipefail
export TMPDIR=/tmp
BENCH_ARGS="--config 4 --pairs 2" bash tools/profile_round.sh gpurun_out/r05w/c4 || exit 4
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r05w/bench_driver_args.json 2> gpurun_out/r05w/bench_driver_args.err || exit 5
tail -c 400 gpurun_out/r05w/bench_driver_args.json
