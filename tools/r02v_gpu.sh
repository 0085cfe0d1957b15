set -o pipefail
mkdir -p gpurun_out
for w in c1 head; do for win in 4096 8192; do
  WIN=$win timeout -k 10 120 python -u tools/single_loop.py $w 50 || exit 1
done; done
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmc_c1_sq -- python3 tools/single_loop.py c1 5 > gpurun_out/pmc_c1_sq.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmc_head_sq -- python3 tools/single_loop.py head 5 > gpurun_out/pmc_head_sq.log 2>&1 || exit 1
