#!/bin/bash
set -u
export TMPDIR=/tmp
bash tools/profile_r03.sh ${OUT:-gpurun_out/r03p} "c2|ec30to60_streamline_euler_1000000_seg720_p2c6|1|" \
    "c3|ec30to60_chain3_euler_10000000_seg1440|dispatches|--config 3 --pairs 1" || exit 1
timeout -k 10 500 python3 bench.py --config 3 --steps 1 --warmup 1 > ${OUT:-gpurun_out/r03p}/c3_full.json 2> ${OUT:-gpurun_out/r03p}/c3_full.err || { echo "c3 full failed"; exit 1; }
cut -c1-300 ${OUT:-gpurun_out/r03p}/c3_full.json
