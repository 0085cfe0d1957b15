set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_long_frames.py -k "text_frame_over_1gib" > gpurun_out/pytest_long.log 2>&1 || { tail -40 gpurun_out/pytest_long.log; exit 1; }
tail -5 gpurun_out/pytest_long.log
