#!/bin/bash
# r04: decimation classes under a work counter (wct_dec_merge 3) vs per class (0) / static merged (2).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
WTMI_WCT_DEC_MERGE=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_wct_app.py tests/test_gpu_fullsize.py tests/test_gpu_stores_graphs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_wct.log 2>&1
rc=$?; tail -2 gpurun_out/t_wct.log; [ $rc -eq 0 ] || exit $rc
for B in 64 128 256 512; do
  timeout -k 10 200 python scripts/ab_option.py c4 wct_dec_merge 0 2 3 --batch $B --rounds 4 > gpurun_out/ab_dyn_$B.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_dyn_$B.log; [ $rc -eq 0 ] || exit $rc
done
