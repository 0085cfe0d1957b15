set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_long_frames.py > gpurun_out/pytest_long.log 2>&1 || { tail -40 gpurun_out/pytest_long.log; exit 1; }
tail -8 gpurun_out/pytest_long.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ > gpurun_out/pytest_gpu_all.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_all.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_all.log
