#!/bin/bash
# A/B/C... of several builds of libwtmi.so on one box, alternating bench runs (separate processes):
#   bash scripts/debug/ab_libs.sh CONFIG ROUNDS LIB_1 LIB_2 ...
set -u
cfg=$1; rounds=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 "$rounds"); do
  for lib in "$@"; do
    WTMI_LIB_PATH=$lib timeout -k 10 200 python bench.py --config "$cfg" --steps 20 --warmup 5 \
      --no-cpu-baseline > gpurun_out/ab_lib.log 2>&1 || { tail -5 gpurun_out/ab_lib.log; exit 1; }
    python -c "import json;d=json.loads([l for l in open('gpurun_out/ab_lib.log') if l[0]=='{'][-1]);print('$cfg', '$lib', round(d['ms_per_step'],4), d.get('check'))"
  done
done
