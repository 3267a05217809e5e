# C4 phase-A workgroup-count sweep (WTMI_WCT_TARGET_WG, WTMI_WCT_MIN_ROWS), alternating runs
#   bash scripts/debug/c4_target_wg.sh
set -u
mkdir -p gpurun_out
for r in 1 2; do
  for cfg in "8192 4" "100000 4" "100000 3" "100000 2"; do
    set -- $cfg
    WTMI_WCT_TARGET_WG=$1 WTMI_WCT_MIN_ROWS=$2 timeout -k 10 200 python bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c4.json || exit 1
    python -c "import json;d=json.load(open('gpurun_out/c4.json'));print('target $1 min_rows $2', round(d['ms_per_step'],4))"
  done
done
