# round 5, final build: GPU suite + smoke, then the profiles of the default line (config 3 Euler) and its RK4 chain
set -o pipefail
out=gpurun_out/r05w
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -3 $out/pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo smoke failed; exit 2; }
tail -1 $out/smoke.log
bash tools/profile_round.sh $out/c3 || exit 3
BENCH_ARGS="--method rk4" bash tools/profile_round.sh $out/c3rk4 || exit 4
