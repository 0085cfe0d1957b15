set -o pipefail
mkdir -p gpurun_out
for w in head c1; do for u in 3 0; do
  WSC_UNMASK_BUF=$u timeout -k 10 120 python -u tools/single_loop.py $w || exit 1
  WSC_UNMASK_BUF=$u timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_single_${w}_$u -- python3 tools/single_loop.py $w > /dev/null 2>&1 || exit 1
  python tools/kt_gaps.py gpurun_out/kt_single_${w}_$u/*/*_kernel_trace.csv | grep -v fillBuffer
done; done
