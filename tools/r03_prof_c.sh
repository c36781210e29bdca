#!/bin/bash
# Round-3 final-build profiles of the other three kernel modes on the config-2 mesh.
set -u
export TMPDIR=/tmp
o=${OUT:-gpurun_out/r03f}
bash tools/profile_r03.sh $o "sr|ec30to60_streamline_rk4_1000000_seg720_p2c6|1|--method rk4" \
    "pe|ec30to60_pathline_euler_1000000_seg720_p2c6|1|--mode pathline" \
    "pr|ec30to60_pathline_rk4_1000000_seg720_p2c6|1|--mode pathline --method rk4" || exit 1
