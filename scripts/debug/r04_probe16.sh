#!/bin/bash
# r04: the N = 8192 tail's permlane swaps batched 8 per wait-state block -- parity, then A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_cwt.py tests/test_gpu_wct_app.py tests/test_gpu_long.py tests/test_gpu_stores_graphs.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_sw.log 2>&1
rc=$?; tail -2 gpurun_out/t_sw.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh c4 wavelet-transformer_amd/wtmi/_ab/libwtmi_head.so wavelet-transformer_amd/wtmi/libwtmi.so 4 > gpurun_out/ab_sw4.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/ab_sw4.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh c5 wavelet-transformer_amd/wtmi/_ab/libwtmi_head.so wavelet-transformer_amd/wtmi/libwtmi.so 2 > gpurun_out/ab_sw5.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/ab_sw5.log; [ $rc -eq 0 ] || exit $rc
