#!/bin/bash
# Interleaved A/B of engine variants (build/variants/libmops_<v>.so; "base" = the product library):
# ${ROUNDS:-2} rounds of bench.py ${BENCH_ARGS} per variant, one summary line each in $OUT/ab.txt.
set -u
out=${OUT:-gpurun_out/var_ab}
mkdir -p $out
export TMPDIR=/tmp
: > $out/ab.txt
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in "$@"; do
    if [ "$v" = base ]; then L=""; else L=$PWD/build/variants/libmops_$v.so; fi
    MOPS_TRAJ_LIB=$L timeout -k 10 300 python3 -u bench.py --no-cpu-baseline ${BENCH_ARGS:---steps 5 --warmup 1} \
        > $out/${v}_$r.json 2> $out/${v}_$r.err || { echo "$v failed"; tail -20 $out/${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$out/${v}_$r.json')); r=d['roofline']
print('%-12s ms/step %.3f value %.4e dispatch_ms %.3f launch_ms %.3f' % ('$v', d['ms_per_step'], d['value'], r.get('avg_dispatch_ms') or 0, r.get('avg_launch_ms') or 0))" | tee -a $out/ab.txt
  done
done
