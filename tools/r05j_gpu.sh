# round 5: piece-major level-pair records + Morton vertex numbering (product) against the round-4 layout
# (oldlayout) and each change alone (novperm: pieces only; nopieces: numbering only); GPU suite first
set -o pipefail
out=gpurun_out/r05j
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -3 $out/pytest.log
if [ $rc -ne 0 ]; then echo "pytest rc $rc: stopping"; exit $rc; fi
BENCH_ARGS="--config 4 --pairs 6 --steps 1 --warmup 1" OUT=$out/c4 ROUNDS=1 bash tools/var_ab.sh base oldlayout novperm nopieces || exit 4
BENCH_ARGS="--config 2 --steps 3 --warmup 1" OUT=$out/c2 ROUNDS=1 bash tools/var_ab.sh base oldlayout || exit 5
MOPS_BENCH_NO_RK4=1 BENCH_ARGS="--steps 2 --warmup 1" OUT=$out/c3 ROUNDS=1 bash tools/var_ab.sh base oldlayout || exit 3
cat $out/c4/ab.txt $out/c2/ab.txt $out/c3/ab.txt
