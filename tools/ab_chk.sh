#!/bin/bash
# k_u8_check builds (tools/build_variant.sh): p0w4 = no next-unit prefetch (127 VGPRs, no spills),
# p0w5 / p1w5 = 5 waves per SIMD (96 VGPRs, 112 / 188 B of spills); UTF-8 parity through WSC_LIB,
# then the TEXT configs twice, interleaved with the in-tree library (prefetch, 4 waves, 20 B spills).
for v in p0w4 p0w5 p1w5; do
  WSC_LIB=$PWD/tools/_var/libwscodec_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_utf8.py > gpurun_out/${v}_pytest.log 2>&1 || { echo "$v FAILED"; tail -15 gpurun_out/${v}_pytest.log; exit 1; }
  echo "$v utf8: $(tail -1 gpurun_out/${v}_pytest.log)"
done
for rep in 1 2; do
  for v in default p0w4 p0w5 p1w5; do
    if [ $v = default ]; then unset WSC_LIB; else export WSC_LIB=$PWD/tools/_var/libwscodec_$v.so; fi
    echo "=== $v rep $rep"
    timeout -k 10 300 python3 tools/cfg_bench.py "TEXT" || exit $?
  done
done
