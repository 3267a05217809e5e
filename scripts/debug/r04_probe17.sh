#!/bin/bash
# r04: degree-6 atan2 polynomial -- full GPU suite, then C4 A/B against the degree-7 library and
# the one-stream trace.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; tail -2 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh c4 wavelet-transformer_amd/wtmi/_ab/libwtmi_head.so wavelet-transformer_amd/wtmi/libwtmi.so 4 > gpurun_out/ab_atan6.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/ab_atan6.log; [ $rc -eq 0 ] || exit $rc
WTMI_WCT_SIDE_STREAM=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trs_a6 -o run -- python scripts/debug/c4_shard_trace.py 512 30 > gpurun_out/trs_a6.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/trs_a6.log; exit $rc; }
python scripts/trace_mean.py gpurun_out/trs_a6 10 | head -4
