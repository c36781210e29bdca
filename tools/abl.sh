#!/bin/bash
# Time bench.py (avg traj_kernel launch) for the default library and each
# build/variants/libmops_<v>.so; BENCH_ARGS selects the mode.  One device, one call.
set -u
out=${OUT:-gpurun_out/abl}
mkdir -p $out
for v in "$@"; do
  if [ "$v" = base ]; then L=""; else L=$PWD/build/variants/libmops_$v.so; fi
  MOPS_TRAJ_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 2 ${BENCH_ARGS:-} > $out/$v.json 2> $out/$v.err || { echo "$v failed"; exit 1; }
  python3 -c "import json; d=json.load(open('$out/$v.json')); print('$v', round(d['roofline']['avg_launch_ms'],3), '%.3e' % d['value'])"
done
