# round 5: GPU suite, then the neighbour-table stay test (MOPS_NBR_TEST) against the variant without it
set -o pipefail
out=gpurun_out/r05b
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -5 $out/pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
BENCH_ARGS="--steps 2 --warmup 1" OUT=$out/c3 ROUNDS=1 bash tools/var_ab.sh base nonbr nopt || exit 3
BENCH_ARGS="--config 4 --pairs 6 --steps 1 --warmup 1" OUT=$out/c4 ROUNDS=1 bash tools/var_ab.sh base nonbr nopt || exit 4
BENCH_ARGS="--config 2 --steps 5 --warmup 1" OUT=$out/c2 ROUNDS=1 bash tools/var_ab.sh base nonbr nopt || exit 5
cat $out/*/ab.txt
