#!/bin/bash
# Stall decomposition of the trajectory kernel (round 6): why do the SIMDs idle?
#   BENCH_ARGS="--method rk4" bash tools/pmc_stall.sh OUTDIR
# Three rocprofv3 passes over one bench step (the RK4 companion off), each within the per-block limits
# (8 SQ, 2 GRBM, SQC alone):
#   wait:   wave cycles, cycles waiting for anything / for an instruction's issue, issue-any, ifetch
#   issue:  VALU single and dual issue, SALU issue, in-flight LDS and VMEM levels (latency = level / insts)
#   icache: SQC instruction-cache hits and misses
# Summarise with: python3 tools/pmc_means.py OUTDIR "<kernel name>" STEPS_PER_LAUNCH
set -u
out=${1:-gpurun_out/stall}
mkdir -p "$out"
export TMPDIR=/tmp MOPS_BENCH_NO_RK4=1
run() {  # name seconds counters...
  local name=$1 secs=$2; shift 2
  timeout -s KILL "$secs" rocprofv3 --pmc "$@" --kernel-include-regex traj_kernel --output-format csv -d "$out/$name" -o p -- \
      python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 ${BENCH_ARGS:-} > "$out/$name.log" 2>&1 \
      || { echo "$name pass failed"; tail -5 "$out/$name.log"; exit 1; }
}
run wait ${PASS_SECS:-300} SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH \
    SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
run issue ${PASS_SECS:-300} SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_ACTIVE_INST_SCA SQ_INST_LEVEL_LDS SQ_INST_LEVEL_VMEM \
    SQ_INSTS_LDS SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE
# the SQC block's counter limit is not in the guide: probe it on a short program first
if timeout -s KILL 60 rocprofv3 --pmc SQC_ICACHE_HITS SQC_ICACHE_MISSES GRBM_GUI_ACTIVE --output-format csv -d "$out/icache_probe" \
    -o p -- ./build/fp64bench 1 add_f64 > "$out/icache_probe.log" 2>&1; then
  run icache ${PASS_SECS:-300} SQC_ICACHE_HITS SQC_ICACHE_MISSES GRBM_GUI_ACTIVE
else
  echo "icache probe failed: SQC pass skipped"; tail -3 "$out/icache_probe.log"
fi
echo "stall ok"
