#!/bin/bash
# r04: side streams at the least stream priority (the caller's decimated chain is critical at 64 pairs).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for B in 64 128 256 512; do
  timeout -k 10 200 python scripts/ab_option.py c4 wct_side_prio 0 2 3 --batch $B --rounds 4 > gpurun_out/ab_lprio_$B.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_lprio_$B.log; [ $rc -eq 0 ] || exit $rc
done
WTMI_WCT_SIDE_PRIO=2 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tll_64 -o run -- python scripts/debug/c4_shard_trace.py 64 30 > gpurun_out/tll_64.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/tll_64.log; exit $rc; }
python scripts/debug/trace_timeline.py gpurun_out/tll_64 wct_spectra_plan 2
