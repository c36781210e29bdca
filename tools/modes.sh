#!/bin/bash
# One-device refresh of the per-mode table: bench.py in the four
# kernel modes on the config-2 mesh, then configs 4 and 5; JSON lines in $1.
set -u
out=${1:-gpurun_out/modes}
mkdir -p "$out"
for m in "se:" "sr:--method rk4" "pe:--mode pathline" "pr:--mode pathline --method rk4"; do
  n=${m%%:*}; a=${m#*:}
  timeout -k 10 240 python3 bench.py --no-cpu-baseline $a > "$out/$n.json" 2> "$out/$n.err" || { echo "$n failed"; exit 1; }
done
timeout -k 10 400 python3 bench.py --config 4 --steps 1 --warmup 0 > "$out/c4.json" 2> "$out/c4.err" || { echo "c4 failed"; exit 1; }
timeout -k 10 400 python3 bench.py --config 5 --steps 1 --warmup 0 > "$out/c5.json" 2> "$out/c5.err" || { echo "c5 failed"; exit 1; }
echo modes ok
