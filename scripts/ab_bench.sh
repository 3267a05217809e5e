#!/bin/bash
# A/B of two builds of libwtmi.so on one box: alternate bench runs (separate processes).
#   bash scripts/ab_bench.sh CONFIG LIB_A LIB_B [ROUNDS]
set -u
cfg=$1; la=$2; lb=$3; rounds=${4:-3}
mkdir -p gpurun_out
for r in $(seq 1 $rounds); do
  for tag in A B; do
    lib=$la; [ $tag = B ] && lib=$lb
    WTMI_LIB_PATH=$lib timeout -k 10 200 python bench.py --config $cfg --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_$tag.json || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_$tag.json'));print('$tag', round(d['ms_per_step'],4))"
  done
done
