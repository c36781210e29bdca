#!/bin/bash
# Round-3 GPU check, part 2: RK4 dead-particle compaction A/B on the config-2 workload, then the
# oRRS18to6-size parity module (configs 4 and 5).
set -u
out=${OUT:-gpurun_out/r03}
mkdir -p $out
export TMPDIR=/tmp
for c in off on off on; do
  timeout -k 10 300 python -u bench.py --method rk4 --no-cpu-baseline --steps 3 --compact $c > $out/rk4_compact_$c.json 2>> $out/rk4_ab.err || { echo "rk4 $c failed"; tail $out/rk4_ab.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/rk4_compact_$c.json')); print('rk4 compact $c', round(d['ms_per_step'],2), 'ms', round(d['roofline']['avg_launch_ms'],2), 'ms launches', '%.3e' % d['value'])"
done
timeout -k 10 1000 python -u -m pytest tests/test_full_size_orrs.py -x -v -m gpu --timeout 900 --timeout-method thread > $out/pytest_orrs.log 2>&1 || { echo "orrs pytest failed"; tail -40 $out/pytest_orrs.log; exit 1; }
tail -8 $out/pytest_orrs.log
