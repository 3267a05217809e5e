# Per-kernel SQ / TA / TCP / TCC counters of one bench config, three separate --pmc passes.
#   bash scripts/debug/pmc_detail.sh [c2|c3|c4|c5]  ->  gpurun_out/pmcx_<cfg>/summary.txt
set -u
export TMPDIR=/tmp
CFG=${1:-c3}
mkdir -p gpurun_out/pmcx_$CFG
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmcx_$CFG/counters_list.txt 2>&1 || echo "list rc=$?"
B="python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmcx_$CFG/p1 -o run -- $B > gpurun_out/pmcx_$CFG/p1.log 2>&1 || { echo p1 fail; tail -5 gpurun_out/pmcx_$CFG/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmcx_$CFG/p2 -o run -- $B > gpurun_out/pmcx_$CFG/p2.log 2>&1 || { echo p2 fail; tail -5 gpurun_out/pmcx_$CFG/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_FLAT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcx_$CFG/p3 -o run -- $B > gpurun_out/pmcx_$CFG/p3.log 2>&1 || { echo p3 fail; tail -5 gpurun_out/pmcx_$CFG/p3.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmcx_$CFG/p1 gpurun_out/pmcx_$CFG/p2 gpurun_out/pmcx_$CFG/p3 > gpurun_out/pmcx_$CFG/summary.txt
cat gpurun_out/pmcx_$CFG/summary.txt | grep -i wtmi
