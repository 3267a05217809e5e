#!/bin/bash
# r04: stream policy at the full batch with the final kernels (side stream on/off, phase C's third stream).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 256 512; do
  timeout -k 10 200 python scripts/ab_option.py c4 wct_side_stream 0 1 --batch $B --rounds 4 > gpurun_out/ab_side_$B.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_side_$B.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python scripts/ab_option.py c4 wct_pc_early 0 1 --batch 512 --rounds 4 > gpurun_out/ab_pce_512.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/ab_pce_512.log; [ $rc -eq 0 ] || exit $rc
