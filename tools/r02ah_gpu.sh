set -o pipefail
mkdir -p gpurun_out
for w in c1 head c2; do
  timeout -k 10 120 python -u tools/single_loop.py $w 30 || exit 1
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_h_$w -- python3 tools/single_loop.py $w 10 > /dev/null 2>&1 || exit 1
  python tools/kt_gaps.py gpurun_out/kt_h_$w/*/*_kernel_trace.csv | grep "dur q" | grep wsc
done
