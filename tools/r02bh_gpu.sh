set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_utf8.py > gpurun_out/pytest_u8.log 2>&1 || { tail -40 gpurun_out/pytest_u8.log; exit 1; }
tail -1 gpurun_out/pytest_u8.log
