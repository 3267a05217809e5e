#!/bin/bash
# r04: merged decimation-class launch -- WCT GPU tests, A/B at shard sizes (bitwise check inside).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wct_app.py tests/test_gpu_fullsize.py tests/test_gpu_stores_graphs.py tests/test_gpu_threads.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_wct.log 2>&1
rc=$?; tail -3 gpurun_out/t_wct.log; [ $rc -eq 0 ] || exit $rc
for B in 64 128 512; do
  timeout -k 10 200 python scripts/ab_option.py c4 wct_dec_merge 0 1 --batch $B --rounds 4 > gpurun_out/ab_merge_$B.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_merge_$B.log; [ $rc -eq 0 ] || exit $rc
done
