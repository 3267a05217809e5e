#!/bin/bash
# C3 synthesis: chain levels from dq >= CG groups read W_j from L2, below it through LDS.
# FETCH_SIZE per variant (modwt_syn 1/2/3 = CG 4/8/16) and an in-process timing A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in 3 4 5 6; do
  WTMI_MODWT_SYN=$v timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/c3cg_$v -o run -- python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c3cg_$v.log 2>&1 || { tail -5 gpurun_out/c3cg_$v.log; exit 1; }
  python scripts/pmc_summary.py gpurun_out/c3cg_$v | grep -i imodwt
done
timeout -k 10 300 python scripts/ab_option.py c3s modwt_syn 1 3 4 5 6 --rounds 4 > gpurun_out/c3cg_ab.log 2>&1; rc=$?; cat gpurun_out/c3cg_ab.log; exit $rc
