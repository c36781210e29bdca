#!/bin/bash
# Round-3 final-build profiles of configs 4 and 5 (kernel stats, PMC traffic + counters, bench line) and the
# full 30-day config-4 run.
set -u
export TMPDIR=/tmp
o=${OUT:-gpurun_out/r03f}
bash tools/profile_r03.sh $o "c4|orrs18to6_chain4_euler_10000000_seg720|dispatches|--config 4 --pairs 2" \
    "c5|orrs18to6_chain5_euler_12500000_seg4320|dispatches|--config 5 --pairs 1" || exit 1
timeout -k 10 600 python3 bench.py --config 4 --steps 1 --warmup 0 > $o/c4_full.json 2> $o/c4_full.err || { echo "c4 full failed"; exit 1; }
cut -c1-300 $o/c4_full.json
