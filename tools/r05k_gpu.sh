# round 5: RK4 stage sums accumulated as they come (product) vs at the end (noacc); Morton vertex numbering
# (product) vs the caller's order (novperm0); two interleaved rounds each
set -o pipefail
out=gpurun_out/r05k
mkdir -p $out
export TMPDIR=/tmp
BENCH_ARGS="--method rk4 --steps 1 --warmup 1" OUT=$out/rk4 ROUNDS=2 bash tools/var_ab.sh base noacc || exit 3
BENCH_ARGS="--config 2 --steps 3 --warmup 1" OUT=$out/c2 ROUNDS=2 bash tools/var_ab.sh base noacc novperm0 || exit 4
BENCH_ARGS="--config 4 --pairs 6 --steps 1 --warmup 1" OUT=$out/c4 ROUNDS=2 bash tools/var_ab.sh base novperm0 || exit 5
for v in base noacc novperm0; do for r in 1 2; do python3 -c "
import json; d=json.load(open('$out/c2/${v}_$r.json')); print('$v c2 rk4 companion', d['rk4_companion']['value'], d['rk4_companion']['ms_per_call'])"; done; done
cat $out/rk4/ab.txt $out/c2/ab.txt $out/c4/ab.txt
