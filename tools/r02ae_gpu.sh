set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_utf8.py tests/test_gpu_parity.py -k "utf8 or U8 or text or fuzz or close or golden" > gpurun_out/pytest_u8.log 2>&1 || { tail -30 gpurun_out/pytest_u8.log; exit 1; }
tail -1 gpurun_out/pytest_u8.log
for w in t64 t1 c1 head; do timeout -k 10 120 python -u tools/single_loop.py $w 20 || exit 1; done
