#!/bin/bash
# round 5: the plain pathline Euler kernel without LDS edge normals (MOPS_NRM_PE_PLAIN=0) against the final
# product build, interleaved: config 4 (6 pairs) x 3, config-2 mesh pathline Euler (1e6 particles) x 2
set -o pipefail
out=gpurun_out/r05nrm
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
for r in 1 2 3; do
  run c4_base_$r $B/libmops_r05final.so --config 4 --pairs 6 --steps 1 --warmup 1 || exit 3
  run c4_nrm0_$r $B/libmops_nrmplain0.so --config 4 --pairs 6 --steps 1 --warmup 1 || exit 3
done
for r in 1 2; do
  run pe_base_$r $B/libmops_r05final.so --config 2 --mode pathline --steps 5 --warmup 1 || exit 3
  run pe_nrm0_$r $B/libmops_nrmplain0.so --config 2 --mode pathline --steps 5 --warmup 1 || exit 3
done
