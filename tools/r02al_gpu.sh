set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_utf8.py tests/test_gpu_parity.py > gpurun_out/pytest_agg.log 2>&1 || { tail -30 gpurun_out/pytest_agg.log; exit 1; }
tail -1 gpurun_out/pytest_agg.log
for w in t1 t64 c2; do timeout -k 10 120 python -u tools/single_loop.py $w 30 || exit 1; done
timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt_t1 -- python3 tools/single_loop.py t1 10 > /dev/null 2>&1 || exit 1
