#!/bin/bash
# round 5: the config-3 Euler profile of the final build again (the first profiling box ran 6% slow)
set -o pipefail
export TMPDIR=/tmp
bash tools/profile_round.sh gpurun_out/r05x/c3 || exit 3
grep -h "traj_kernel<7, true, true, true>" gpurun_out/r05x/c3/stats/*kernel_stats.csv | cut -c1-120
