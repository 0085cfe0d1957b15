set -o pipefail
mkdir -p gpurun_out
WSC_U8_WPB=10 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_utf8.py > gpurun_out/pytest_u8.log 2>&1 || { tail -30 gpurun_out/pytest_u8.log; exit 1; }
tail -1 gpurun_out/pytest_u8.log
for rep in 1 2; do for wpb in 4 10; do for w in c2 c1 t64 t1; do echo -n "wpb $wpb "; WSC_U8_WPB=$wpb timeout -k 10 120 python -u tools/single_loop.py $w 30 || exit 1; done; done; done
