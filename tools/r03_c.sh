#!/bin/bash
# Round-3 GPU check, part 3: RBF + parity suites, the oRRS18to6-size module, and kernel-trace
# stats of the RK4 companion with and without dead-particle compaction.
set -u
out=${OUT:-gpurun_out/r03}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_rbf_gpu.py tests/test_gpu_parity.py -x -v -m gpu --timeout 300 \
    --timeout-method thread > $out/pytest_rbf.log 2>&1 || { echo "rbf/parity pytest failed"; tail -40 $out/pytest_rbf.log; exit 1; }
tail -2 $out/pytest_rbf.log
for c in off on; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_rk4_$c -o p -- \
      python3 bench.py --method rk4 --no-cpu-baseline --steps 2 --warmup 1 --compact $c > $out/prof_rk4_$c.log 2>&1 \
      || { echo "rk4 prof $c failed"; tail $out/prof_rk4_$c.log; exit 1; }
done
timeout -k 10 1000 python -u -m pytest tests/test_full_size_orrs.py -x -v -m gpu --timeout 900 --timeout-method thread \
    > $out/pytest_orrs.log 2>&1 || { echo "orrs pytest failed"; tail -40 $out/pytest_orrs.log; exit 1; }
tail -6 $out/pytest_orrs.log
