#!/bin/bash
# Round-3: parity suite after the live-count launches, then RK4 compaction schedules.
set -u
out=${OUT:-gpurun_out/r03h}
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests -x -q -m gpu --ignore=tests/test_full_size_orrs.py --timeout 300 \
    --timeout-method thread > $out/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $out/pytest.log; exit 1; }
tail -1 $out/pytest.log
run() {
  local tag=$1; shift
  MOPS_BENCH_NO_RK4=1 timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 "$@" \
      > $out/$tag.json 2> $out/$tag.err || { echo "$tag failed"; tail -5 $out/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$tag.json')); print('$tag', round(d['ms_per_step'],2), 'ms/step', round(d['roofline']['avg_launch_ms'],2), 'ms segment', '%.4e' % d['value'])"
}
run se_default
run sr_p2c6_off --method rk4 --compact off
run sr_p2c6_on --method rk4 --compact on
run sr_p1c6_on --method rk4 --compact on --parts 1 --chunks 6
run sr_p2c3_on --method rk4 --compact on --parts 2 --chunks 3
run sr_p1c8_on --method rk4 --compact on --parts 1 --chunks 8
run sr_p2c8_on --method rk4 --compact on --parts 2 --chunks 8
run pr_p2c6_off --method rk4 --mode pathline --compact off
run pr_p2c6_on --method rk4 --mode pathline --compact on
