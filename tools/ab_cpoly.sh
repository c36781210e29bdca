set -u
export TMPDIR=/tmp MOPS_BENCH_NO_RK4=1
out=gpurun_out/cpoly; mkdir -p $out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "path or wide" --timeout 200 --timeout-method thread > $out/pytest.log 2>&1 || { echo pytest failed; tail -20 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
OUT=$out/c4 ROUNDS=2 BENCH_ARGS="--config 4 --pairs 2 --steps 1 --warmup 1" bash tools/var_ab.sh base cpoly0 || exit 1
OUT=$out/c3 ROUNDS=2 BENCH_ARGS="--config 3 --pairs 1 --steps 1 --warmup 1" bash tools/var_ab.sh base cpoly0 || exit 1
OUT=$out/pe ROUNDS=2 BENCH_ARGS="--mode pathline --steps 3 --warmup 1" bash tools/var_ab.sh base cpoly0 || exit 1
