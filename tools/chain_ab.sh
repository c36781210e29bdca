#!/bin/bash
# A/B of library variants on the chained-pathline configs (3; 4 with 2 daily pairs; 5 with one
# monthly pair): tools/chain_ab.sh base VARIANT...  (build/variants/libmops_<v>.so)
set -u
out=${OUT:-gpurun_out/chab}
mkdir -p $out
for c in "3|--config 3 --steps 1 --warmup 1" "4|--config 4 --pairs 2 --steps 1 --warmup 0" "5|--config 5 --pairs 1 --steps 1 --warmup 0"; do
  n=${c%%|*}; a=${c#*|}
  for v in "$@"; do
    if [ "$v" = base ]; then L=""; else L=$PWD/build/variants/libmops_$v.so; fi
    MOPS_TRAJ_LIB=$L timeout -k 10 400 python3 bench.py --no-cpu-baseline $a > $out/c${n}_$v.json 2> $out/c${n}_$v.err || { echo "c$n $v failed"; exit 1; }
    python3 -c "import json; d=json.load(open('$out/c${n}_$v.json')); r=d['roofline']; print('c$n', '$v', round(r.get('avg_launch_ms') or r.get('avg_dispatch_ms') or 0, 3), '%.3e' % d['value'], d['ms_per_step'])"
  done
done
