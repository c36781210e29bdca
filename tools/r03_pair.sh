set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pair
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread --ignore=tests/test_full_size_orrs.py > gpurun_out/pair/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pair/pytest.log; exit 1; }
tail -2 gpurun_out/pair/pytest.log
for v in profpair profnopair; do
  MOPS_PROF_SECTIONS=1 MOPS_TRAJ_LIB=$PWD/build/variants/libmops_$v.so timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 1 --warmup 0 > gpurun_out/pair/$v.json 2> gpurun_out/pair/$v.err || { echo "$v failed"; exit 1; }
  grep "prof counters" gpurun_out/pair/$v.err
done
OUT=gpurun_out/pair ROUNDS=2 bash tools/var_ab.sh base nopair
