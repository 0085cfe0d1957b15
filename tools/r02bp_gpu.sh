set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/kt_c11 -o kt -- python3 tools/single_loop.py c11 20 > gpurun_out/c11.log 2>&1 || { tail -20 gpurun_out/c11.log; exit 1; }
grep "c11:" gpurun_out/c11.log
f=$(find gpurun_out/kt_c11 -name '*kernel_stats.csv' | head -1); cut -d, -f1-4 "$f" | head -12
