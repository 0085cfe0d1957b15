set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_utf8.py > gpurun_out/pytest_u8.log 2>&1 || { tail -30 gpurun_out/pytest_u8.log; exit 1; }
tail -1 gpurun_out/pytest_u8.log
for rep in 1 2; do for w in t64 t1 c2; do timeout -k 10 120 python -u tools/single_loop.py $w 30 || exit 1; done; done
