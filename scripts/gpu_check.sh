#!/bin/bash
# One GPU session: smoke -> parity tests -> bench -> rocprof kernel trace.
# Each GPU step has its own time limit; a crash/abort/timeout (exit >= 124 or a
# signal) ends the session; ordinary test failures (pytest exit 1) do not.
set -u
OUT=gpurun_out
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" ; date
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"; tail -5 $OUT/$name.log
  if [ $rc -ge 124 ] || [ $rc -gt 128 ]; then echo "FATAL in $name (rc=$rc): stopping"; exit $rc; fi
  return $rc
}
STEPS=${STEPS:-"smoke tests bench prof"}
for s in $STEPS; do
  case $s in
    smoke) step smoke 400 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    tests) step pytest_gpu 1500 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} ; [ $? -le 1 ] || exit 1 ;;
    bench) step bench 600 python bench.py ${BENCH_ARGS:-} || exit $? ;;
    prof)  step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python bench.py --no-cpu-baseline ${BENCH_ARGS:-} || exit $?
           python scripts/trace_mean.py $OUT/prof 50 > $OUT/prof/timed_mean.txt; cat $OUT/prof/timed_mean.txt ;;
    traffic)
      for c in ${TRAFFIC_CFGS:-c2 c3 c4 c5}; do
        for ctr in FETCH_SIZE WRITE_SIZE; do
          step pmc_${c}_$ctr 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/pmc_${c}_$ctr -o run -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline || exit $?
        done
        python scripts/pmc_traffic.py $c $OUT/pmc_${c}_FETCH_SIZE $OUT/pmc_${c}_WRITE_SIZE $OUT/pmc_traffic.json || exit 1
      done ;;
    counters) step counters 300 rocprofv3 -L ;;
    pmc)
      i=0
      GROUPS_STR=${PMC_GROUPS:-"WRITE_SIZE;FETCH_SIZE;GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU"}
      IFS=';' read -ra GRPS <<< "$GROUPS_STR"
      for grp in "${GRPS[@]}"; do
        i=$((i+1))
        step pmc$i 300 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/pmc$i -o run -- ${PMC_CMD:-python bench.py --steps 3 --warmup 1 --no-cpu-baseline}
        rc=$?; [ $rc -ge 124 ] && exit $rc
      done ;;
    c3|c4|c5) step bench_$s 600 python bench.py --config $s --steps 5 --warmup 2 --no-cpu-baseline || exit $? ;;
    profcfg) step prof_$PCFG 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$PCFG -o run -- python bench.py --config $PCFG --steps 10 --warmup 3 --no-cpu-baseline || exit $? ;;
    profc3) step profc3 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profc3 -o run -- python bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline || exit $? ;;
    profall) step profall 900 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/profall -o run -- python scripts/profile_all.py || exit $? ;;
  esac
done
echo ALLDONE
