#!/bin/bash
# Round-3: derivation chain timing (product build + level-pair record tile variants) under
# rocprofv3 kernel stats, on the oRRS18to6-class mesh.
set -u
out=${OUT:-gpurun_out/r03f}
mkdir -p $out
export TMPDIR=/tmp
V=$PWD/build/variants
for v in product rec64x16 rec32x16 rec32x32 rec64x8; do
  if [ $v = product ]; then L=""; else L=$V/libmops_$v.so; fi
  MOPS_TRAJ_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof_$v -o p -- \
      python3 tools/derive_bench.py --reps 4 > $out/derive_$v.json 2> $out/derive_$v.err || { echo "derive $v failed"; tail -5 $out/derive_$v.err; exit 1; }
  echo "$v $(cat $out/derive_$v.json)" | cut -c1-220
done
