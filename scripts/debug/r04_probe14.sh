#!/bin/bash
# r04: phase B with all K window rows' loads in flight (wct_b_deep).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
WTMI_WCT_B_DEEP=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_wct_app.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_wct.log 2>&1
rc=$?; tail -2 gpurun_out/t_wct.log; [ $rc -eq 0 ] || exit $rc
for B in 64 128 512; do
  timeout -k 10 200 python scripts/ab_option.py c4 wct_b_deep 0 1 2 3 --batch $B --rounds 4 > gpurun_out/ab_bdeep_$B.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_bdeep_$B.log; [ $rc -eq 0 ] || exit $rc
done
for v in 0 3; do
  WTMI_WCT_B_DEEP=$v WTMI_WCT_SIDE_STREAM=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trb_$v -o run -- python scripts/debug/c4_shard_trace.py 64 30 > gpurun_out/trb_$v.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/trb_$v.log; exit $rc; }
  echo "deep=$v 64 pairs serial:"; python scripts/trace_mean.py gpurun_out/trb_$v 10 | grep 'phase_b\|boxcar'
done
