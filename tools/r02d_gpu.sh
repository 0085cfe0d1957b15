set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_session.py tests/test_echo.py tests/test_gpu_parity.py -m gpu -x -v --timeout 120 --timeout-method thread -k "session or echo or decode_packet" > gpurun_out/pytest_session.log 2>&1 || exit 1
for a in "--conns 1 --frames 4000 --size 65536" "--conns 64 --frames 200 --size 65536 --client-threads 4" "--conns 64 --frames 2000 --size 1024 --client-threads 4"; do
  timeout -k 10 120 tools/ws_echo $a >> gpurun_out/echo.log 2>&1 || exit 1
  timeout -k 10 120 tools/ws_echo $a --sync >> gpurun_out/echo.log 2>&1 || exit 1
  timeout -k 10 120 oracle/_build/ws_echo_cpu $a >> gpurun_out/echo.log 2>&1 || exit 1
done
