#!/bin/bash
# Round-3 GPU A/B: kernel variants (streamline Euler / RK4, config 2) and RK4 dead-particle
# compaction with high-priority re-sort streams.
set -u
out=${OUT:-gpurun_out/r03d}
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
  for v in base7 hexpairs sqrt1; do run se_${v}_$rep $V/libmops_$v.so; done
  for v in base7 sqrt1; do run sr_${v}_$rep $V/libmops_$v.so --method rk4 --compact off; done
  for c in off on; do run sr_compact_${c}_$rep "" --method rk4 --compact $c; done
done
