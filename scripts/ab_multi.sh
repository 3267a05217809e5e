#!/bin/bash
# A/B/C... of launch options on one box: alternate bench runs (separate processes) over
# several environment settings.   bash scripts/ab_multi.sh CONFIG ROUNDS "ENV_1" "ENV_2" ...
set -u
cfg=$1; rounds=$2; shift 2
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  i=0
  for e in "$@"; do
    i=$((i+1))
    env $e timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_$i.log 2>&1 || { tail -5 gpurun_out/ab_$i.log; exit 1; }
    python -c "import json;d=json.loads([l for l in open('gpurun_out/ab_$i.log') if l[0]=='{'][-1]);print('[$e]', round(d['ms_per_step'],4), d['check'])"
  done
done
