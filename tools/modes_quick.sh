#!/bin/bash
# Time bench.py (no CPU baseline) in the four kernel modes on the config-2 mesh; one line each.
set -u
out=${OUT:-gpurun_out/modes}
mkdir -p "$out"
for m in "se|" "sr|--method rk4" "pe|--mode pathline" "pr|--mode pathline --method rk4"; do
  n=${m%%|*}; a=${m#*|}
  timeout -k 10 240 python3 bench.py --no-cpu-baseline $a ${BENCH_ARGS:-} > "$out/$n.json" 2> "$out/$n.err" || { echo "$n failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$n.json')); print('$n', round(d['roofline']['avg_launch_ms'],2), '%.3e' % d['value'])"
done
