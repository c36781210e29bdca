#!/bin/bash
# Round-3 GPU check: the -m gpu suite without the oRRS-size module, the default bench line,
# and the self-launched 2-rank rehearsal (both ranks on the one test GPU, gloo).
set -u
out=${OUT:-gpurun_out/r03}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
    --ignore=tests/test_full_size_orrs.py > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -3 $out/pytest.log
timeout -k 10 300 python -u bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
MOPS_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --steps 2 --warmup 1 \
    --no-cpu-baseline > $out/bench_2rank.json 2> $out/bench_2rank.err || { echo "2-rank failed"; tail -20 $out/bench_2rank.err; exit 1; }
cat $out/bench_2rank.json
