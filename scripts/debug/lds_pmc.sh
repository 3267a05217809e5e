#!/bin/bash
# LDS / issue counters for the CWT and WCT kernels of C2, C4, C5 (diagnostic).
set -u
export TMPDIR=/tmp
OUT=gpurun_out/lds_pmc
mkdir -p $OUT
for c in c2 c4 c5; do
  timeout -k 10 200 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d $OUT/$c -o run -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $OUT/$c.log 2>&1 || exit 1
done
echo done
