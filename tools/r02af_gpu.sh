set -o pipefail
mkdir -p gpurun_out
WSC_U8_INLINE_MAX=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_utf8.py > gpurun_out/pytest_u8.log 2>&1 || { tail -30 gpurun_out/pytest_u8.log; exit 1; }
tail -1 gpurun_out/pytest_u8.log
for rs in 0 1; do for w in t64 t1 c1 head; do echo "restage $rs"; WSC_U8_RESTAGE=$rs timeout -k 10 120 python -u tools/single_loop.py $w 20 || exit 1; done; done
