set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcx
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmcx/counters_list.txt 2>&1 || echo "list rc=$?"
B="python bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_VALU SQ_BUSY_CYCLES --kernel-trace --output-format csv -d gpurun_out/pmcx/p1 -o run -- $B > gpurun_out/pmcx/p1.log 2>&1 || { echo p1 fail; tail -5 gpurun_out/pmcx/p1.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d gpurun_out/pmcx/p2 -o run -- $B > gpurun_out/pmcx/p2.log 2>&1 || { echo p2 fail; tail -5 gpurun_out/pmcx/p2.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_FLAT GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d gpurun_out/pmcx/p3 -o run -- $B > gpurun_out/pmcx/p3.log 2>&1 || { echo p3 fail; tail -5 gpurun_out/pmcx/p3.log; exit 1; }
python scripts/pmc_summary.py gpurun_out/pmcx/p1 gpurun_out/pmcx/p2 gpurun_out/pmcx/p3 > gpurun_out/pmcx/summary.txt
cat gpurun_out/pmcx/summary.txt | grep -i modwt
