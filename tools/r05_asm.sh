#!/bin/bash
# round 5, late: assembly kernel with 16-B record reads and streaming stores (MOPS_ASM_V2) -- parity with the
# variant, then config-3 chains interleaved against the final build, then kernel stats of both
set -o pipefail
out=gpurun_out/r05asm
mkdir -p $out
export TMPDIR=/tmp
B=$PWD/build/variants
MOPS_TRAJ_LIB=$B/libmops_asm2.so timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
    tests/test_gpu_parity.py tests/test_remove_nan_gpu.py tests/test_chain.py > $out/test.txt 2>&1 || { tail -40 $out/test.txt; exit 2; }
tail -2 $out/test.txt
run() {  # name lib args...
  local name=$1 lib=$2; shift 2
  MOPS_BENCH_NO_RK4=1 MOPS_TRAJ_LIB=$lib timeout -k 10 400 python3 -u bench.py --no-cpu-baseline "$@" \
      > $out/$name.json 2> $out/$name.err || { echo "$name failed"; tail -20 $out/$name.err; exit 3; }
  python3 -c "
import json; d=json.load(open('$out/$name.json'))
print('%-14s ms/step %.3f value %.4e' % ('$name', d['ms_per_step'], d['value']))" | tee -a $out/ab.txt
}
for r in 1 2 3; do
  run c3_base_$r $B/libmops_base.so --steps 5 --warmup 1 || exit 3
  run c3_asm2_$r $B/libmops_asm2.so --steps 5 --warmup 1 || exit 3
done
for v in base asm2; do
  MOPS_BENCH_NO_RK4=1 MOPS_TRAJ_LIB=$B/libmops_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $out/stats_$v -o p -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 > $out/stats_$v.log 2>&1 || exit 4
  grep -h "assemble" $out/stats_$v/*kernel_stats.csv | cut -c1-160
done
