#!/bin/bash
# Time the config-2 bench for (parts, chunks) schedules of ParticleSet.advance_pipelined.
set -u
out=${OUT:-gpurun_out/pipe}
mkdir -p $out
for pc in "$@"; do
  p=${pc%x*}; c=${pc#*x}
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 3 --parts $p --chunks $c ${BENCH_ARGS:-} > $out/$pc.json 2> $out/$pc.err || { echo "$pc failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$pc.json')); print('$pc', round(d['ms_per_step'],3), round(d['roofline']['avg_launch_ms'],3), '%.4e' % d['value'])"
done
