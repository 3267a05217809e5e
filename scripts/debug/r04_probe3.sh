#!/bin/bash
# r04: full GPU suite with the merged decimation launch; shard sweeps at 64 / 128 pairs.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_all.log 2>&1
rc=$?; tail -3 gpurun_out/t_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u scripts/shard_graph.py c4 40 > gpurun_out/shard_c4.log 2>&1; rc=$?; grep -v amdgpu.ids gpurun_out/shard_c4.log; [ $rc -eq 0 ] || exit $rc
for B in 64 128; do
  timeout -k 10 200 python scripts/ab_option.py c4 wct_dec_rows 2 3 4 6 --batch $B --rounds 3 > gpurun_out/ab_decrows_$B.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_decrows_$B.log; [ $rc -eq 0 ] || exit $rc
  timeout -k 10 200 python scripts/ab_option.py c4 wct_min_rows 1 2 3 --batch $B --rounds 3 > gpurun_out/ab_minrows_$B.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_minrows_$B.log; [ $rc -eq 0 ] || exit $rc
done
