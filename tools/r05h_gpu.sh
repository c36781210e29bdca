# round 5: config 4's plain kernel -- polygon in registers at 2 waves/SIMD (rcw2), 2 waves alone (w2) -- and the
# pair test re-armed by the neighbour table (nbrpair), against the product build; configs 4 and 3
set -o pipefail
out=gpurun_out/r05h
mkdir -p $out
export TMPDIR=/tmp
BENCH_ARGS="--config 4 --pairs 6 --steps 1 --warmup 1" OUT=$out/c4 ROUNDS=1 bash tools/var_ab.sh base rcw2 w2 nbrpair || exit 4
MOPS_BENCH_NO_RK4=1 BENCH_ARGS="--steps 2 --warmup 1" OUT=$out/c3 ROUNDS=2 bash tools/var_ab.sh base nbrpair || exit 3
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread -k "neighbour or parity or full_size_pair" > $out/pytest.log 2>&1
tail -2 $out/pytest.log
cat $out/c4/ab.txt $out/c3/ab.txt
