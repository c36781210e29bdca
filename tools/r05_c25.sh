# round 5, final build: the config-5 year (12 calendar-month pairs) and the config-2 line
set -o pipefail
out=gpurun_out/r05v
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u bench.py --config 2 > $out/bench_c2.json 2> $out/bench_c2.err || exit 2
timeout -k 10 900 python -u bench.py --config 5 > $out/bench_c5.json 2> $out/bench_c5.err || exit 3
tail -c 300 $out/bench_c5.json
