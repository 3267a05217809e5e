#!/bin/bash
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 64 128 256 512; do
  timeout -k 10 200 python scripts/debug/c4_graph_ab.py $B 5 > gpurun_out/graph_ab_$B.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/graph_ab_$B.log; [ $rc -eq 0 ] || exit $rc
done
