#!/bin/bash
# UTF-8 chain counts: the unmask's fold with 8 / 16 chains (tools/build_variant.sh foldN
# -DWSC_FOLD_NCH=N) and the check with 8 (WSC_U8_CHAINS=8), against the in-tree library (fold 4,
# check 4): UTF-8 parity, then the TEXT configs twice; then the check's trace and SQ pass.
for v in fold8 fold16; do
  WSC_LIB=$PWD/tools/_var/libwscodec_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_utf8.py > gpurun_out/${v}_pytest.log 2>&1 || { echo "$v FAILED"; tail -15 gpurun_out/${v}_pytest.log; exit 1; }
  echo "$v utf8: $(tail -1 gpurun_out/${v}_pytest.log)"
done
WSC_U8_CHAINS=8 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_utf8.py > gpurun_out/chk8_pytest.log 2>&1 || { echo "chk8 FAILED"; tail -15 gpurun_out/chk8_pytest.log; exit 1; }
echo "chk8 utf8: $(tail -1 gpurun_out/chk8_pytest.log)"
for rep in 1 2; do
  for v in default fold8 fold16 chk8; do
    unset WSC_LIB WSC_U8_CHAINS
    case $v in fold*) export WSC_LIB=$PWD/tools/_var/libwscodec_$v.so ;; chk8) export WSC_U8_CHAINS=8 ;; esac
    echo "=== $v rep $rep"
    timeout -k 10 300 python3 tools/cfg_bench.py "TEXT" || exit $?
  done
done
unset WSC_LIB WSC_U8_CHAINS
bash tools/pmc_check.sh
