#!/bin/bash
# r04: C4 64-pair timeline (streams on) and a rows-per-workgroup sweep at shard sizes.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl_64 -o run -- python scripts/debug/c4_shard_trace.py 64 30 > gpurun_out/tl_64.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/tl_64.log; exit $rc; }
python scripts/debug/trace_timeline.py gpurun_out/tl_64 wct_spectra_plan 2
python scripts/debug/trace_timeline.py gpurun_out/tl_64 wct_spectra_plan 3
for B in 64 128 256 512; do
  timeout -k 10 200 python scripts/ab_option.py c4 wct_min_rows 1 2 3 4 --batch $B --rounds 3 > gpurun_out/ab_minrows_$B.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_minrows_$B.log; [ $rc -eq 0 ] || exit $rc
done
