#!/bin/bash
# One GPU session producing the judged artifacts of a round (run via gpurun):
#   1. PMC FETCH_SIZE / WRITE_SIZE passes per config -> gpurun_out/pmc_traffic.json
#      (copied into profiles/$ROUND/ on the box so the bench lines carry "traffic")
#   2. rocprofv3 --kernel-trace --stats per config   -> gpurun_out/prof_<cfg>/
#   3. bench.py per config (CPU baseline included)   -> gpurun_out/bench_<cfg>.json
#   4. (r03) a VALU PMC pass per config + the traces -> gpurun_out/kernel_roofline.json
#      (per-kernel binding resource; copied into profiles/$ROUND/ like pmc_traffic.json);
#      (r04) plus an LDS pass (array cycles, bank conflicts, LDS issue stalls)
#   PARTS selects the parts: "pmc prof roof bench" (default all).
# Every GPU step has its own time limit; a crash / abort / timeout ends the session.
set -u
ROUND=${ROUND:-r06}
PARTS=${PARTS:-"pmc prof roof bench"}
CFGS=${CFGS:-"c2 c3 c4 c5"}
OUT=gpurun_out
mkdir -p $OUT profiles/$ROUND
export TMPDIR=/tmp
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name $(date +%T)"
  timeout -k 10 $t "$@" > $OUT/$name.log 2>&1
  local rc=$?
  echo "   rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/$name.log; echo "FATAL in $name"; exit $rc; fi
}
has() { case " $PARTS " in *" $1 "*) return 0;; esac; return 1; }
if has pmc; then
  for c in $CFGS; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      run pmc_${c}_$ctr 400 rocprofv3 --pmc $ctr --kernel-trace --output-format csv -d $OUT/pmc_${c}_$ctr -o run -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-gather
    done
    python scripts/pmc_traffic.py $c $OUT/pmc_${c}_FETCH_SIZE $OUT/pmc_${c}_WRITE_SIZE $OUT/pmc_traffic.json > /dev/null || exit 1
  done
  cp $OUT/pmc_traffic.json profiles/$ROUND/pmc_traffic.json
fi
if has prof; then
  for c in $CFGS; do
    STEPS_K=10
    [ $c = c2 ] && STEPS_K=50
    run prof_$c 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$c -o run -- python bench.py --config $c --steps $STEPS_K --warmup 5 --no-cpu-baseline --no-gather
    python scripts/trace_mean.py $OUT/prof_$c $STEPS_K > $OUT/prof_$c/timed_mean.txt
  done
fi
if has roof; then
  for c in $CFGS; do
    TR=$OUT/prof_$c
    if [ $c = c4 ]; then  # per-kernel durations from a one-stream trace (each kernel's own time)
      WTMI_WCT_SIDE_STREAM=0 run prof_c4_serial 500 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_c4_serial -o run -- python bench.py --config c4 --steps 10 --warmup 5 --no-cpu-baseline --no-gather
      python scripts/trace_mean.py $OUT/prof_c4_serial 10 > $OUT/prof_c4_serial/timed_mean.txt
      TR=$OUT/prof_c4_serial
    fi
    run valu_$c 400 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/valu_$c -o run -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-gather
    run lds_$c 400 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/lds_$c -o run -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-gather
    STEPS_K=10
    [ $c = c2 ] && STEPS_K=50
    python scripts/kernel_roofline.py $c $TR $OUT/pmc_${c}_FETCH_SIZE $OUT/pmc_${c}_WRITE_SIZE $OUT/valu_$c $OUT/kernel_roofline.json $STEPS_K $OUT/lds_$c > $OUT/roof_$c.txt || exit 1
    head -4 $OUT/roof_$c.txt
  done
  cp $OUT/kernel_roofline.json profiles/$ROUND/kernel_roofline.json
fi
if has bench; then
  for c in $CFGS; do
    ARGS=""
    [ $c = c2 ] && ARGS="--steps 20 --warmup 5"
    [ $c = c2 ] || ARGS="--steps 10 --warmup 3"
    run bench_$c 600 python bench.py --config $c $ARGS
    grep '^{' $OUT/bench_$c.log | tail -1 > $OUT/bench_$c.json
    cut -c1-200 $OUT/bench_$c.json
  done
fi
echo ALLDONE
