# C5 chunk-size / workgroup-target sweep (one box, alternating runs)
#   bash scripts/debug/c5_chunks.sh
set -u
mkdir -p gpurun_out
for r in 1 2; do
  for ch in 256 512 1024; do
    for wg in 0 2048; do
      if [ $wg = 0 ]; then E="WTMI_DUMMY=0"; else E="WTMI_CWT_TARGET_WG=$wg"; fi
      env WTMI_C5_CHUNK=$ch $E timeout -k 10 200 python bench.py --config c5 --steps 4 --warmup 2 --no-cpu-baseline > gpurun_out/c5.json || exit 1
      python -c "import json;d=json.load(open('gpurun_out/c5.json'));print('chunk $ch wg $wg', round(d['ms_per_step'],3))"
    done
  done
done
