#!/bin/bash
# r04: phase C q windows entered at their union smoothed band (plan bits ec) -- WCT parity tests,
# A/B against the HEAD library, full-band rows' own chunking A/B, smoke + default bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_wct_app.py tests/test_gpu_fullsize.py tests/test_gpu_wct_sig.py tests/test_gpu_stores_graphs.py tests/test_gpu_cwt.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_wct.log 2>&1
rc=$?; tail -2 gpurun_out/t_wct.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh c4 wavelet-transformer_amd/wtmi/_ab/libwtmi_head.so wavelet-transformer_amd/wtmi/libwtmi.so 4 > gpurun_out/ab_ec.log 2>&1
rc=$?; grep -v amdgpu gpurun_out/ab_ec.log; [ $rc -eq 0 ] || exit $rc
for B in 64 128; do
  timeout -k 10 200 python scripts/ab_option.py c4 wct_k0_rows 0 1 2 --batch $B --rounds 4 > gpurun_out/ab_k0rows_$B.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_k0rows_$B.log; [ $rc -eq 0 ] || exit $rc
done
WTMI_WCT_SIDE_STREAM=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trs_ec -o run -- python scripts/debug/c4_shard_trace.py 512 30 > gpurun_out/trs_ec.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/trs_ec.log; exit $rc; }
python scripts/trace_mean.py gpurun_out/trs_ec 10 | head -8
