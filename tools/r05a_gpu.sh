set -o pipefail
mkdir -p gpurun_out/r05a
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread > gpurun_out/r05a/pytest.log 2>&1
rc=$?
tail -5 gpurun_out/r05a/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
BENCH_ARGS="--method rk4 --steps 2 --warmup 1" OUT=gpurun_out/r05a/ab ROUNDS=1 bash tools/var_ab.sh base nocooppr || exit 3
timeout -k 10 600 python -u bench.py --steps 3 --warmup 1 > gpurun_out/r05a/bench.json 2> gpurun_out/r05a/bench.err || exit 4
tail -c 3000 gpurun_out/r05a/bench.json
exit $rc
