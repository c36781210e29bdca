#!/bin/bash
# Round 6 GPU driver: STAGE selects what runs (one gpurun call per stage).
#   stall   class prices (fp64bench) + stall decomposition of the tiled RK4 and Euler pathline kernels
set -u
export TMPDIR=/tmp
O=gpurun_out/r06${TAG:-}
mkdir -p $O
for st in ${STAGE:-stall}; do
case "$st" in
stall)
  bash tools/fp64bench.sh $O/fp64bench || exit 2
  python3 tools/fp64bench_summary.py $O/fp64bench > $O/fp64bench/summary.txt; cat $O/fp64bench/summary.txt
  BENCH_ARGS="--method rk4" bash tools/pmc_stall.sh $O/stall_rk4 || exit 3
  python3 tools/pmc_means.py $O/stall_rk4 "void traj_kernel<7, true, false, true>" 240 > $O/stall_rk4/summary.txt
  bash tools/pmc_stall.sh $O/stall_euler || exit 4
  python3 tools/pmc_means.py $O/stall_euler "void traj_kernel<7, true, true, true>" 1440 > $O/stall_euler/summary.txt
  tail -12 $O/stall_rk4/summary.txt $O/stall_euler/summary.txt
  ;;
newtests)  # the round's new GPU tests (host delivery, root gather)
  timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
      tests/test_record_density.py::test_host_line_sink_delivers_the_device_lines tests/test_multirank_gpu.py \
      > $O/newtests.log 2>&1
  rc=$?; tail -15 $O/newtests.log; [ $rc -eq 0 ] || exit 5
  ;;
rk4ab)  # code-size variants of the tiled RK4 kernel (tools/build_variant.sh nohexprc / nohexpr)
  BENCH_ARGS="--method rk4 --steps 1 --warmup 1" OUT=$O/rk4ab ROUNDS=2 bash tools/var_ab.sh base ${RK4_VARIANTS:-nohexprc nohexpr} || exit 11
  cat $O/rk4ab/ab.txt
  ;;
pcsamp)  # PC sampling of the config-3 Euler and RK4 launches (2e6 particles, one pair): hot instructions
  export MOPS_BENCH_NO_COMPANIONS=1
  for m in euler rk4; do
    rm -rf /tmp/pcs_$m
    timeout -s KILL 400 rocprofv3 --pc-sampling-beta-enabled 1 --pc-sampling-method ${PCS_METHOD:-stochastic} \
        --pc-sampling-unit ${PCS_UNIT:-cycles} --pc-sampling-interval ${PCS_INTERVAL:-65536} -d /tmp/pcs_$m -o p \
        --output-format csv -- python3 bench.py --no-cpu-baseline --steps 1 --warmup 0 --pairs 1 --particles 2000000 \
        --method $m > $O/pcs_$m.log 2>&1 || { tail -20 $O/pcs_$m.log; exit 9; }
    python3 tools/pcsamp_summary.py /tmp/pcs_$m $O/pcs_$m.txt traj_kernel || exit 10
    du -sh /tmp/pcs_$m
  done
  ;;
gputests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit 6
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 7; }
  tail -1 $O/smoke.log
  ;;
bench)
  timeout -k 10 900 python -u bench.py ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 8; }
  tail -c 1500 $O/bench.json
  ;;
esac
done
