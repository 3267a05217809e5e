#!/bin/bash
# r04: 64-pair timelines with the current library (streams on).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlg_64 -o run -- python scripts/debug/c4_shard_trace.py 64 30 > gpurun_out/tlg_64.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/tlg_64.log; exit $rc; }
for it in 2 3 4; do python scripts/debug/trace_timeline.py gpurun_out/tlg_64 wct_spectra_plan $it; done
