set -o pipefail
mkdir -p gpurun_out
for w in t64; do
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD --output-format csv -d gpurun_out/pmc_${w}_sq2 -- python3 tools/single_loop.py $w 3 > gpurun_out/pmc_${w}_sq2.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAVES SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_ANY SQ_INSTS_SMEM --output-format csv -d gpurun_out/pmc_${w}_sq3 -- python3 tools/single_loop.py $w 3 > gpurun_out/pmc_${w}_sq3.log 2>&1 || exit 1
done
