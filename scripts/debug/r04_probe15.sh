#!/bin/bash
# r04: band phasor folded into the N = 8192 radix-2 tail -- GPU suite, then C4 A/B against HEAD.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; tail -2 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh c4 wavelet-transformer_amd/wtmi/_ab/libwtmi_head.so wavelet-transformer_amd/wtmi/libwtmi.so 4 > gpurun_out/ab_ph.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/ab_ph.log; [ $rc -eq 0 ] || exit $rc
WTMI_WCT_SIDE_STREAM=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trs_ph -o run -- python scripts/debug/c4_shard_trace.py 512 30 > gpurun_out/trs_ph.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/trs_ph.log; exit $rc; }
python scripts/trace_mean.py gpurun_out/trs_ph 10 | head -6
