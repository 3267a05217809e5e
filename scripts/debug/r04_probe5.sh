#!/bin/bash
# r04: side stream at the greatest stream priority (A/B at shard sizes) + timeline with it.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_stores_graphs.py tests/test_gpu_threads.py tests/test_gpu_fullsize.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_wct.log 2>&1
rc=$?; tail -2 gpurun_out/t_wct.log; [ $rc -eq 0 ] || exit $rc
for B in 64 128 256 512; do
  timeout -k 10 200 python scripts/ab_option.py c4 wct_side_prio 0 1 --batch $B --rounds 4 > gpurun_out/ab_prio_$B.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_prio_$B.log; [ $rc -eq 0 ] || exit $rc
done
WTMI_WCT_SIDE_PRIO=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlp_64 -o run -- python scripts/debug/c4_shard_trace.py 64 30 > gpurun_out/tlp_64.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/tlp_64.log; exit $rc; }
python scripts/debug/trace_timeline.py gpurun_out/tlp_64 wct_spectra_plan 2
