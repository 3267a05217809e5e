#!/bin/bash
# r04: rows per workgroup for tiny WCT batches (the app's single-pair calls) -- WCT tests,
# app latencies, and C4-shaped A/B at 1 / 8 / 32 pairs.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_wct_app.py tests/test_gpu_stores_graphs.py tests/test_gpu_wct_sig.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_wct.log 2>&1
rc=$?; tail -2 gpurun_out/t_wct.log; [ $rc -eq 0 ] || exit $rc
for B in 1 8 32; do
  timeout -k 10 200 python scripts/ab_option.py c4 wct_min_rows 1 4 --batch $B --rounds 4 > gpurun_out/ab_mr_$B.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_mr_$B.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 500 python scripts/app_latency.py --out gpurun_out/app_latency.json > gpurun_out/app_latency.log 2>&1
rc=$?; python -c "
import json;d=json.load(open('gpurun_out/app_latency.json'))
print({k:round(v['median_ms'],3) for k,v in d['gpu'].items() if isinstance(v,dict) and 'median_ms' in v})"; exit $rc
