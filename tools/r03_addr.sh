set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/addr
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread --ignore=tests/test_full_size_orrs.py > gpurun_out/addr/pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/addr/pytest.log; exit 1; }
tail -2 gpurun_out/addr/pytest.log
OUT=gpurun_out/addr ROUNDS=2 bash tools/var_ab.sh base prev
OUT=gpurun_out/addr_c ROUNDS=2 bash tools/ab.sh "--steps 5 --warmup 1 --compact off" "--steps 5 --warmup 1 --compact on"
OUT=gpurun_out/addr/pmc bash tools/pmc_variants.sh base prev
