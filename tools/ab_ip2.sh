#!/bin/bash
# In-place unmask variants through WSC_LIB (tools/build_variant.sh): ip2 = edge windows in two
# passes, ip2w5 = the same built for 5 waves per SIMD; parity first, then the headline and the
# in-place configs, twice, interleaved with the in-tree library.
HL="--steps 200 --warmup 10 --no-cpu --no-host-inclusive --no-echo --no-other-configs --no-config3"
for v in ip2 ip2w5; do
  WSC_LIB=$PWD/tools/_var/libwscodec_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "not True" > gpurun_out/${v}_pytest.log 2>&1 || { echo "$v parity FAILED"; tail -15 gpurun_out/${v}_pytest.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/${v}_pytest.log)"
done
for rep in 1 2; do
  for v in default ip2 ip2w5; do
    if [ $v = default ]; then unset WSC_LIB; else export WSC_LIB=$PWD/tools/_var/libwscodec_$v.so; fi
    echo "=== $v rep $rep"
    timeout -k 10 120 python3 bench.py $HL || exit $?
    timeout -k 10 300 python3 tools/cfg_bench.py "configs[1] 1M x 1 KiB BIN, 16" "configs[2] 256k mixed 125" "configs[3]" || exit $?
  done
done
