#!/bin/bash
# r04: smoke + default bench (as the driver runs them), full-band rows' own chunking A/B, 64-pair timeline.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE OK')" > gpurun_out/smoke.log 2>&1
rc=$?; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; tail -1 gpurun_out/bench_default.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
for B in 64 128; do
  timeout -k 10 200 python scripts/ab_option.py c4 wct_k0_rows 0 1 2 --batch $B --rounds 4 > gpurun_out/ab_k0rows_$B.log 2>&1
  rc=$?; grep -v amdgpu.ids gpurun_out/ab_k0rows_$B.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tlf_64 -o run -- python scripts/debug/c4_shard_trace.py 64 30 > gpurun_out/tlf_64.log 2>&1
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/tlf_64.log; exit $rc; }
python scripts/debug/trace_timeline.py gpurun_out/tlf_64 wct_spectra_plan 2
python scripts/debug/trace_timeline.py gpurun_out/tlf_64 wct_spectra_plan 3
