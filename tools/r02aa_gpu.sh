set -o pipefail
mkdir -p gpurun_out
for w in t64 t1; do
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/pmc_${w}_sq -- python3 tools/single_loop.py $w 3 > gpurun_out/pmc_${w}_sq.log 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_${w} -- python3 tools/single_loop.py $w 10 > /dev/null 2>&1 || exit 1
python tools/kt_gaps.py gpurun_out/kt_${w}/*/*_kernel_trace.csv | grep "dur" | grep -v fill
done
