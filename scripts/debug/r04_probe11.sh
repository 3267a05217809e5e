#!/bin/bash
# r04: phase B on the third stream after the decimated time-domain rows (wct_b_third), side
# streams at the least priority (wct_side_prio) -- WCT parity tests first.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_wct_app.py tests/test_gpu_fullsize.py tests/test_gpu_stores_graphs.py tests/test_gpu_threads.py tests/test_gpu_edges.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_wct.log 2>&1
rc=$?; tail -2 gpurun_out/t_wct.log; [ $rc -eq 0 ] || exit $rc
for B in 64 128 256; do
  timeout -k 10 200 python scripts/ab_option.py c4 wct_b_third 0 1 --batch $B --rounds 4 > gpurun_out/ab_b3_$B.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_b3_$B.log; [ $rc -eq 0 ] || exit $rc
done
for B in 64 128 512; do
  timeout -k 10 200 python scripts/ab_option.py c4 wct_side_prio 0 2 3 --batch $B --rounds 3 > gpurun_out/ab_lprio_$B.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_lprio_$B.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlb_64 -o run -- python scripts/debug/c4_shard_trace.py 64 30 > gpurun_out/tlb_64.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/tlb_64.log; exit $rc; }
python scripts/debug/trace_timeline.py gpurun_out/tlb_64 wct_spectra_plan 2
