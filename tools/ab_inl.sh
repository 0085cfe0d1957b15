#!/bin/bash
# The unmask's general window inlined (no call: in place 84 VGPRs, COMPACT 72, no spills) with the
# P = 4 kernels built for 4 (inl4) or 5 (inl5) waves per SIMD, through WSC_LIB: parity, then the
# headline and every other_configs line, twice, interleaved with the in-tree library.
HL="--steps 200 --warmup 10 --no-cpu --no-host-inclusive --no-echo --no-other-configs --no-config3"
for v in inl4 inl5; do
  WSC_LIB=$PWD/tools/_var/libwscodec_$v.so timeout -k 10 420 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_utf8.py tests/test_gpu_long_frames.py > gpurun_out/${v}_pytest.log 2>&1 || { echo "$v FAILED"; tail -15 gpurun_out/${v}_pytest.log; exit 1; }
  echo "$v parity: $(tail -1 gpurun_out/${v}_pytest.log)"
done
for rep in 1 2; do
  for v in default inl4 inl5; do
    if [ $v = default ]; then unset WSC_LIB; else export WSC_LIB=$PWD/tools/_var/libwscodec_$v.so; fi
    echo "=== $v rep $rep"
    timeout -k 10 120 python3 bench.py $HL || exit $?
    timeout -k 10 400 python3 tools/cfg_bench.py || exit $?
  done
done
