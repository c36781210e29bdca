#!/bin/bash
# A/B of bench.py option sets on one box: each set runs ${ROUNDS:-2} times, interleaved, and one
# summary line per run goes to $OUT/ab.txt.  Usage: OUT=gpurun_out/x bash tools/ab.sh "<args A>" "<args B>" ...
set -u
out=${OUT:-gpurun_out/ab}
mkdir -p $out
export TMPDIR=/tmp
: > $out/ab.txt
for r in $(seq 1 ${ROUNDS:-2}); do
  i=0
  for args in "$@"; do
    i=$((i+1))
    timeout -k 10 300 python -u bench.py $args --no-cpu-baseline > $out/run_${r}_${i}.json 2> $out/run_${r}_${i}.err || { echo "run failed: $args"; tail -20 $out/run_${r}_${i}.err; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('$out/run_${r}_${i}.json'))
f=d.get('finalize') or {}
print('%-50s ms/step %.3f value %.4e fin %.3f' % ('$args', d['ms_per_step'], d['value'], f.get('ms_per_call') or 0))" | tee -a $out/ab.txt
  done
done
