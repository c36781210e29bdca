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
eulerab)  # tiled Euler kernel variants on the driver's default workload (config 3, 7-pair chain)
  MOPS_BENCH_NO_COMPANIONS=1 BENCH_ARGS="--steps 2 --warmup 1" OUT=$O/eulerab ROUNDS=${ROUNDS:-2} bash tools/var_ab.sh base ${EULER_VARIANTS} || exit 12
  cat $O/eulerab/ab.txt
  ;;
prof)  # event counters (-DMOPS_PROF builds): cooperative wave-steps, regroups, walks per variant
  for v in ${PROF_VARIANTS:-prof7 prof8}; do
    MOPS_TRAJ_LIB=$PWD/build/variants/libmops_$v.so MOPS_PROF_SECTIONS=1 MOPS_BENCH_NO_COMPANIONS=1 timeout -k 10 300 \
        python3 -u bench.py --no-cpu-baseline --steps 1 --warmup 0 ${BENCH_ARGS:-} > $O/prof_$v.json 2> $O/prof_$v.err \
        || { tail -20 $O/prof_$v.err; exit 13; }
    grep "prof counters" $O/prof_$v.err | sed "s/^/$v: /"
  done
  ;;
rk4ab)  # code-size variants of the tiled RK4 kernel (tools/build_variant.sh nohexprc / nohexpr)
  BENCH_ARGS="--method rk4 --steps 1 --warmup 1" OUT=$O/rk4ab ROUNDS=${ROUNDS:-2} bash tools/var_ab.sh base ${RK4_VARIANTS:-nohexprc nohexpr} || exit 11
  cat $O/rk4ab/ab.txt
  ;;
profiles)  # PMC profiles of the other configs' launches (their PMC entries for this engine build)
  BENCH_ARGS="--config 2" bash tools/profile_round.sh $O/c2 || exit 18
  BENCH_ARGS="--config 4 --pairs 2" bash tools/profile_round.sh $O/c4 || exit 19
  ;;
profile)  # the round's profile of one workload (tools/profile_round.sh: bench, rocprof stats, PMC passes incl. the class mix)
  bash tools/profile_round.sh $O/${PROF_NAME:-c3} || exit 14
  grep -h "traj_kernel" $O/${PROF_NAME:-c3}/stats/*kernel_stats.csv | cut -c1-110 | head -4
  ;;
stalleuler)
  bash tools/pmc_stall.sh $O/stall_euler || exit 20
  python3 tools/pmc_means.py $O/stall_euler "void traj_kernel<7, true, true, true>" 1440 > $O/stall_euler/summary.txt
  tail -8 $O/stall_euler/summary.txt
  ;;
stallrk4)
  BENCH_ARGS="--method rk4" bash tools/pmc_stall.sh $O/stall_rk4 || exit 15
  python3 tools/pmc_means.py $O/stall_rk4 "void traj_kernel<7, true, false, true>" 240 > $O/stall_rk4/summary.txt
  tail -8 $O/stall_rk4/summary.txt
  ;;
rehearse)  # the N > 1 bench path with both ranks on the one GPU (gloo), default collection (gather to rank 0)
  MOPS_BENCH_ONE_DEVICE=1 MOPS_BENCH_NO_COMPANIONS=1 timeout -k 10 600 python -u bench.py --gpus 2 --backend gloo --steps 1 \
      --warmup 0 --pairs 2 --particles 2000000 --no-cpu-baseline > $O/rehearsal_2rank_gloo_root.json \
      2> $O/rehearsal_2rank_gloo_root.err || { tail -30 $O/rehearsal_2rank_gloo_root.err; exit 16; }
  tail -c 1200 $O/rehearsal_2rank_gloo_root.json
  ;;
configs)  # the other BASELINE configs on the final engine (config 2 call, config 4 30-day run, config 5 year)
  for c in 2 4 5; do
    timeout -k 10 700 python -u bench.py --config $c > $O/bench_c$c.json 2> $O/bench_c$c.err || { tail -20 $O/bench_c$c.err; exit 17; }
    python3 -c "import json; d=json.load(open('$O/bench_c$c.json')); print($c, d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'))"
  done
  ;;
gputests)
  timeout -k 10 1000 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -5 $O/pytest.log; [ $rc -eq 0 ] || exit 6
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; exit 7; }
  tail -1 $O/smoke.log
  ;;
bench)  # the driver's command (LINE_ARGS, default its --steps 20 --warmup 5); BENCH_ARGS stays the config selection
  timeout -k 10 900 python -u bench.py ${LINE_ARGS:---steps 20 --warmup 5} ${BENCH_ARGS:-} > $O/bench.json 2> $O/bench.err \
      || { tail -20 $O/bench.err; exit 8; }
  tail -c 1500 $O/bench.json
  ;;
esac
done
