#!/bin/bash
# Record-build tile sweep: rocprofv3 kernel stats of pair_record_fused_kernel per engine variant
# (build/variants/libmops_<v>.so, "base" = the product library) on a 2-pair config-4 chain, after a
# write-bandwidth probe (torch fill_ of 8 GiB, HIP events).
set -u
out=${OUT:-gpurun_out/rec_sweep}
mkdir -p "$out"
export TMPDIR=/tmp MOPS_BENCH_NO_RK4=1
timeout -k 10 120 python3 -c "
import torch
x = torch.empty(2**30, dtype=torch.float64, device='cuda'); y = torch.empty_like(x)
for name, f, b in (('fill 8 GiB', lambda: x.fill_(1.0), 8 * 2**30), ('copy 8 GiB', lambda: y.copy_(x), 16 * 2**30)):
    f(); torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10): f()
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f'{name}: {ms:.3f} ms, {b / ms / 1e6:.0f} GB/s')
" > "$out/write_bw.txt" 2>&1 || { echo "write probe failed"; exit 1; }
for v in "$@"; do
  if [ "$v" = base ]; then L=""; else L=$PWD/build/variants/libmops_$v.so; fi
  MOPS_TRAJ_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/$v" -o p -- \
      python3 bench.py --config 4 --pairs 2 --steps 1 --warmup 0 --no-cpu-baseline > "$out/$v.log" 2>&1 \
      || { echo "$v failed"; exit 1; }
  python3 -c "
import csv
for r in csv.DictReader(open('$out/$v/p_kernel_stats.csv')):
    if 'pair_record_fused' in r['Name']:
        print('%-6s pair_record_fused calls %s avg %.3f ms min %.3f ms' % ('$v', r['Calls'], float(r['AverageNs']) / 1e6, float(r['MinNs']) / 1e6))
" | tee -a "$out/sweep.txt"
done
