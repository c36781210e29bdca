# round 5: RK4 stages as a loop (MOPS_RK4_LOOP, product) against the unrolled form: config-3 RK4 chain, config-2 RK4
# companion; then the GPU suite
set -o pipefail
out=gpurun_out/r05d
mkdir -p $out
export TMPDIR=/tmp
BENCH_ARGS="--method rk4 --steps 1 --warmup 1" OUT=$out/rk4 ROUNDS=2 bash tools/var_ab.sh base rk4unroll || exit 3
BENCH_ARGS="--config 2 --steps 3 --warmup 1" OUT=$out/c2 ROUNDS=2 bash tools/var_ab.sh base rk4unroll || exit 4
for v in base rk4unroll; do for r in 1 2; do python3 -c "
import json; d=json.load(open('$out/c2/${v}_$r.json')); print('$v c2 rk4', d['rk4_companion']['value'], d['rk4_companion']['ms_per_call'])"; done; done
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -3 $out/pytest.log
cat $out/rk4/ab.txt
exit $rc
