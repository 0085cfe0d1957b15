set -o pipefail
mkdir -p gpurun_out
WSC_STAGE_CHECK=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "staged" > gpurun_out/pytest_sc.log 2>&1 || { tail -30 gpurun_out/pytest_sc.log; exit 1; }
tail -1 gpurun_out/pytest_sc.log
for w in t64 t1; do for sc in 0 1; do for wc in 16 128 256; do
  echo -n "stage_check $sc "; WSC_STAGE_CHECK=$sc timeout -k 10 120 python -u tools/staged_probe.py $w $wc 0 30 || exit 1
done; done; done
