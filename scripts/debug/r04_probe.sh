#!/bin/bash
# r04 probe session: GPU suite, atan A/B on C4, serial per-kernel traces of C4 shards.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; tail -3 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
bash scripts/ab_bench.sh c4 wavelet-transformer_amd/wtmi/_ab/libwtmi_atan_r03.so wavelet-transformer_amd/wtmi/libwtmi.so 4 > gpurun_out/ab_atan.log 2>&1
rc=$?; cat gpurun_out/ab_atan.log; [ $rc -eq 0 ] || exit $rc
for B in 64 512; do
  WTMI_WCT_SIDE_STREAM=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trs_$B -o run -- python scripts/debug/c4_shard_trace.py $B 30 > gpurun_out/trs_$B.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/trs_$B.log; exit $rc; }
  python scripts/trace_mean.py gpurun_out/trs_$B 10 > gpurun_out/trs_$B.txt; echo "== B=$B serial"; head -12 gpurun_out/trs_$B.txt
done
for B in 64 128 512; do
  timeout -k 10 200 python scripts/ab_option.py c4 wct_a2_order 0 1 --batch $B --rounds 4 > gpurun_out/ab_order_$B.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_order_$B.log; [ $rc -eq 0 ] || exit $rc
done
