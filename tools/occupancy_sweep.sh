set -u
for cfg in se sr pe pr; do
  case $cfg in se) A="";; sr) A="--method rk4";; pe) A="--mode pathline";; pr) A="--mode pathline --method rk4";; esac
  for v in all1 all2 all3; do
    MOPS_TRAJ_LIB=$PWD/build/variants/libmops_$v.so timeout -k 10 200 python3 bench.py --no-cpu-baseline --steps 1 $A > gpurun_out/var_${cfg}_$v.log 2>&1 || { echo "$cfg $v failed"; exit 1; }
  done
done
echo ok
