# round 5: (1) the VALU instruction mix of the config-3 tiled Euler kernel (INT32 / INT64 / CVT / TRANS counters);
# (2) the per-lane RK4 kernel (-DMOPS_COOP_PR=0) profiled like the tiled one: the RK4 tile's before counters
set -o pipefail
out=gpurun_out/r05m
mkdir -p $out
export TMPDIR=/tmp MOPS_BENCH_NO_RK4=1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT \
    SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_FMA_F32 --kernel-include-regex traj_kernel --output-format csv \
    -d $out/mix -o p -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > $out/mix.log 2>&1 || exit 2
L=$PWD/build/variants/libmops_nocooppr.so
MOPS_TRAJ_LIB=$L timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $out/rk4plain/stats -o p -- \
    python3 bench.py --no-cpu-baseline --method rk4 --steps 1 --warmup 1 > $out/rk4plain_stats.log 2>&1 || exit 3
MOPS_TRAJ_LIB=$L timeout -s KILL 300 rocprofv3 --pmc TD_TD_BUSY_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum \
    --kernel-include-regex traj_kernel --output-format csv -d $out/rk4plain/td -o p -- \
    python3 bench.py --no-cpu-baseline --method rk4 --steps 1 --warmup 0 > $out/rk4plain_td.log 2>&1 || exit 4
MOPS_TRAJ_LIB=$L timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 \
    SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU --kernel-include-regex traj_kernel --output-format csv -d $out/rk4plain/pmc -o p -- \
    python3 bench.py --no-cpu-baseline --method rk4 --steps 1 --warmup 0 > $out/rk4plain_pmc.log 2>&1 || exit 5
echo mix ok
