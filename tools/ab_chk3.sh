#!/bin/bash
# k_u8_check built for 3 waves per SIMD (141 VGPRs, no scratch) against 4 (128 VGPRs + 20 B of
# spills): UTF-8 parity through WSC_LIB, the TEXT configs twice, one-batch traces of both.
V=$PWD/tools/_var/libwscodec_chk3.so
WSC_LIB=$V timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_utf8.py tests/test_gpu_pong_eof.py > gpurun_out/chk3_pytest.log 2>&1 || { echo "chk3 FAILED"; tail -15 gpurun_out/chk3_pytest.log; exit 1; }
echo "chk3 utf8: $(tail -1 gpurun_out/chk3_pytest.log)"
for rep in 1 2; do
  for v in default chk3; do
    if [ $v = default ]; then unset WSC_LIB; else export WSC_LIB=$V; fi
    echo "=== $v rep $rep"
    timeout -k 10 300 python3 tools/cfg_bench.py "TEXT" || exit $?
  done
done
export WSC_LIB=$V
bash tools/kt_configs.sh t64 t1
