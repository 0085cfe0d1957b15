set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_utf8.py > gpurun_out/pytest_u8.log 2>&1 || { tail -30 gpurun_out/pytest_u8.log; exit 1; }
tail -2 gpurun_out/pytest_u8.log
for w in t64 t1; do timeout -k 10 120 python -u tools/single_loop.py $w 20 || exit 1; done
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_t64 -- python3 tools/single_loop.py t64 10 > /dev/null 2>&1 || exit 1
python tools/kt_gaps.py gpurun_out/kt_t64/*/*_kernel_trace.csv | grep "dur" | grep -v fill
