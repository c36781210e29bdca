#!/bin/bash
# Round-3: derivation profiling (product + record-tile variants) and RK4 compaction timelines.
set -u
out=${OUT:-gpurun_out/r03g}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "preprocessing or locate or selftest or math" \
    --timeout 120 --timeout-method thread > $out/pytest_quick.log 2>&1 || { echo "quick pytest failed"; tail -30 $out/pytest_quick.log; exit 1; }
tail -1 $out/pytest_quick.log
for c in off on; do
  MOPS_BENCH_NO_RK4=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $out/trace_rk4_p1c6_$c -o p -- \
      python3 bench.py --method rk4 --no-cpu-baseline --steps 2 --warmup 1 --compact $c --parts 1 --chunks 6 \
      > $out/trace_rk4_p1c6_$c.log 2>&1 || { echo "rk4 trace $c failed"; tail $out/trace_rk4_p1c6_$c.log; exit 1; }
done
bash tools/r03_f.sh
