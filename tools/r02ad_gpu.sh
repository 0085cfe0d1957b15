set -o pipefail
mkdir -p gpurun_out
for ch in 4 2; do
WSC_U8_CHAINS=$ch timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_utf8.py > gpurun_out/pytest_u8_$ch.log 2>&1 || { tail -30 gpurun_out/pytest_u8_$ch.log; exit 1; }
tail -1 gpurun_out/pytest_u8_$ch.log
done
for ch in 1 2 4; do for w in t64 t1; do echo "chains $ch"; WSC_U8_CHAINS=$ch timeout -k 10 120 python -u tools/single_loop.py $w 20 || exit 1; done; done
