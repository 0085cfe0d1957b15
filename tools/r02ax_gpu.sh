set -o pipefail
mkdir -p gpurun_out
WSC_DEBUG_SPLIT=1 timeout -k 10 600 python -u -m pytest -x -q -s --timeout 200 --timeout-method thread tests -m gpu > gpurun_out/pytest_dbg2.log 2>&1 || { grep -a "decode_sync_part\|passed\|failed\|FAILED" gpurun_out/pytest_dbg2.log | tail -40; exit 1; }
tail -2 gpurun_out/pytest_dbg2.log
