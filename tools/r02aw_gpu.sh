set -o pipefail
mkdir -p gpurun_out
WSC_DEBUG_SPLIT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_long_frames.py tests/test_gpu_parity.py tests/test_gpu_session.py -k "long or overflow or config4 or fuzz" > gpurun_out/pytest_dbg.log 2>&1 || { grep -a "decode_sync_part\|passed\|failed" gpurun_out/pytest_dbg.log | tail -40; exit 1; }
tail -2 gpurun_out/pytest_dbg.log
