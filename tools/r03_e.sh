#!/bin/bash
# Round-3 GPU A/B #2: one-sided trig / div3 variants (sqrt one-sided is the default now), and the
# RK4 dead-particle compaction schedules (parts x chunks, priority streams).
set -u
out=${OUT:-gpurun_out/r03e}
mkdir -p $out
export TMPDIR=/tmp
run() {  # tag, lib ('' = product), bench args...
  local tag=$1 lib=$2; shift 2
  MOPS_BENCH_NO_RK4=1 MOPS_TRAJ_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 5 "$@" \
      > $out/$tag.json 2> $out/$tag.err || { echo "$tag failed"; tail -5 $out/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$tag.json')); print('$tag', round(d['ms_per_step'],2), 'ms/step', round(d['roofline']['avg_launch_ms'],2), 'ms segment', '%.4e' % d['value'])"
}
V=$PWD/build/variants
for rep in 1 2; do
  for v in base7 trig1 div1 both1; do run se_${v}_$rep $V/libmops_$v.so; done
  for v in base7 both1; do run sr_${v}_$rep $V/libmops_$v.so --method rk4 --compact off; done
done
L=$V/libmops_base7.so
run sr_p2c6_off $L --method rk4 --compact off
run sr_p1c6_on $L --method rk4 --compact on --parts 1 --chunks 6
run sr_p1c4_on $L --method rk4 --compact on --parts 1 --chunks 4
run sr_p1c8_on $L --method rk4 --compact on --parts 1 --chunks 8
run sr_p2c3_on $L --method rk4 --compact on --parts 2 --chunks 3
run sr_p2c6_on $L --method rk4 --compact on --parts 2 --chunks 6
run sr_p2c6_onprio $L --method rk4 --compact on --parts 2 --chunks 6 --compact-priority
run sr_p1c1_off $L --method rk4 --compact off --parts 1 --chunks 1
