#!/bin/bash
# Time every build/variants/libmops_<v>.so named on the command line (and the
# default library as "base") in the four kernel modes; one device, one call.
set -u
for cfg in se sr pe pr; do
  case $cfg in se) A="";; sr) A="--method rk4";; pe) A="--mode pathline";; pr) A="--mode pathline --method rk4";; esac
  for v in base "$@"; do
    if [ "$v" = base ]; then L=""; else L=$PWD/build/variants/libmops_$v.so; fi
    MOPS_TRAJ_LIB=$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 1 $A > gpurun_out/var_${cfg}_$v.log 2>&1 || { echo "$cfg $v failed"; exit 1; }
  done
done
echo ok
