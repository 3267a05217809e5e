#!/bin/bash
# PMC passes over the C3 MODWT kernels (diagnostic): SQ issue/wait split + clocks.
set -u
export TMPDIR=/tmp
OUT=gpurun_out/imodwt_pmc
mkdir -p $OUT
for syn in 0 2; do
  WTMI_MODWT_SYN=$syn timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d $OUT/syn$syn -o run -- python scripts/debug/imodwt_once.py > $OUT/syn$syn.log 2>&1 || exit 1
  WTMI_MODWT_SYN=$syn timeout -k 10 120 rocprofv3 --pmc SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAVES --kernel-trace --output-format csv -d $OUT/syn${syn}b -o run -- python scripts/debug/imodwt_once.py >> $OUT/syn$syn.log 2>&1 || exit 1
done
echo done
