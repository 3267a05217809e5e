#!/bin/bash
# A/B of launch options on one box: alternate bench runs (separate processes) between two
# environment settings.   bash scripts/ab_env.sh CONFIG "ENV_A" "ENV_B" [ROUNDS]
set -u
cfg=$1; ea=$2; eb=$3; rounds=${4:-3}
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for tag in A B; do
    e=$ea; [ $tag = B ] && e=$eb
    env $e timeout -k 10 200 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/ab_$tag.log 2>&1 || { tail -5 gpurun_out/ab_$tag.log; exit 1; }
    python -c "import json;d=json.loads([l for l in open('gpurun_out/ab_$tag.log') if l[0]=='{'][-1]);print('$tag [$e]', round(d['ms_per_step'],4), d['check'])"
  done
done
