# round 5: GPU suite on the nbr-test + no-pair-test defaults; RK4 with / without the neighbour test;
# event counters (-DMOPS_PROF) of configs 3 and 4
set -o pipefail
out=gpurun_out/r05c
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -3 $out/pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
BENCH_ARGS="--method rk4 --steps 1 --warmup 1" OUT=$out/rk4 ROUNDS=2 bash tools/var_ab.sh base nbrrk0 || exit 3
MOPS_TRAJ_LIB=$PWD/build/variants/libmops_prof.so MOPS_PROF_SECTIONS=1 MOPS_BENCH_NO_RK4=1 timeout -k 10 300 \
    python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline > $out/prof_c3.json 2> $out/prof_c3.err || exit 4
MOPS_TRAJ_LIB=$PWD/build/variants/libmops_prof.so MOPS_PROF_SECTIONS=1 timeout -k 10 400 \
    python -u bench.py --config 4 --pairs 2 --steps 1 --warmup 0 --no-cpu-baseline > $out/prof_c4.json 2> $out/prof_c4.err || exit 5
grep "prof counters" $out/prof_c*.err
cat $out/rk4/ab.txt
