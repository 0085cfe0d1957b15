set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_encode.py tests/test_echo.py > gpurun_out/pytest_enc.log 2>&1 || { tail -30 gpurun_out/pytest_enc.log; exit 1; }
tail -1 gpurun_out/pytest_enc.log
timeout -k 10 120 python -u tools/encode_loop.py || exit 1
timeout -k 10 120 python -u tools/encode_loop.py || exit 1
