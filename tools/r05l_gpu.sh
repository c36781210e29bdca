# round 5: the polygon's pieces by cell rank (MOPS_CPOLY_RANK, product) vs per cell (nocpr); GPU suite first
set -o pipefail
out=gpurun_out/r05l
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -3 $out/pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
BENCH_ARGS="--config 4 --pairs 6 --steps 1 --warmup 1" OUT=$out/c4 ROUNDS=2 bash tools/var_ab.sh base nocpr || exit 4
MOPS_BENCH_NO_RK4=1 BENCH_ARGS="--config 2 --mode pathline --steps 3 --warmup 1" OUT=$out/c2p ROUNDS=1 bash tools/var_ab.sh base nocpr || exit 5
cat $out/c4/ab.txt $out/c2p/ab.txt
