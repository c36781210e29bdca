# round 5: TD cost vs distinct lines per wave-instruction (membench mb_l1_scatter); config 4's 30-day line;
# the two-rank gloo rehearsal of config 3 with record gathers (the memory plan in the line)
set -o pipefail
out=gpurun_out/r05i
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 ./build/membench 3 > $out/membench_times.jsonl || exit 2
timeout -s KILL 120 rocprofv3 --pmc TD_TD_BUSY_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum --kernel-include-regex mb_l1 \
    --output-format csv -d $out/membench_td -o p -- ./build/membench 1 > $out/membench_td.log 2>&1 || exit 3
timeout -k 10 900 python -u bench.py --config 4 > $out/bench_c4.json 2> $out/bench_c4.err || exit 4
MOPS_BENCH_ONE_DEVICE=1 timeout -k 10 600 python -u bench.py --gpus 2 --backend gloo --steps 1 --warmup 0 --pairs 2 \
    --particles 2000000 --no-cpu-baseline > $out/rehearsal_2rank_gloo.json 2> $out/rehearsal_2rank_gloo.err || exit 5
grep scatter $out/membench_times.jsonl
tail -c 600 $out/bench_c4.json
