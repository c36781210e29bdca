#!/bin/bash
# round 5, late: switch sweep on the final build -- config 4 with MOPS_GR_PE 1 / 3 (records in flight per
# group, plain pathline Euler), config 2 with MOPS_NRM_SE=0 (streamline Euler without LDS edge normals),
# config-3 RK4 chain with MOPS_GR_COOP_R 1 / 4 (tile records per LDS round trip in the RK4 kernel)
set -o pipefail
out=gpurun_out/r05sw
mkdir -p $out
export TMPDIR=/tmp
B=$PWD/build/variants
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  MOPS_TRAJ_LIB=$lib timeout -k 10 400 python3 -u bench.py --no-cpu-baseline "$@" \
      > $out/$name.json 2> $out/$name.err || { echo "$name failed"; tail -20 $out/$name.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$out/$name.json'))
print('%-14s ms/step %.3f value %.4e' % ('$name', d['ms_per_step'], d['value']))" | tee -a $out/ab.txt
}
part=${1:-a}
if [ "$part" = a ]; then
for r in 1 2 3; do
  run c2_base_$r $B/libmops_base.so --config 2 --steps 5 --warmup 1 || exit 3
  run c2_senrm0_$r $B/libmops_senrm0.so --config 2 --steps 5 --warmup 1 || exit 3
done
for r in 1 2; do
  for v in base prgr1 prgr4; do
    MOPS_BENCH_NO_RK4=1 run rk4_${v}_$r $B/libmops_$v.so --method rk4 --steps 1 --warmup 1 || exit 3
  done
done
else
for r in 1 2; do
  run c4_base_$r $B/libmops_base.so --config 4 --pairs 6 --steps 1 --warmup 1 || exit 3
  run c4_gr1_$r $B/libmops_pegr1.so --config 4 --pairs 6 --steps 1 --warmup 1 || exit 3
  run c4_gr3_$r $B/libmops_pegr3.so --config 4 --pairs 6 --steps 1 --warmup 1 || exit 3
done
fi
