#!/bin/bash
# COMPACT unmask without the UTF-8 fold: aligned 16-byte stores at 7 (ca7) or 8 (ca8) waves per
# SIMD vs the default byte-aligned stores at 7: COMPACT tests on ca8, configs[4] legs.
o=gpurun_out/r05ab19; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 3 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
V=$PWD/tools/_var
step tests_ca8 500 env WSC_LIB=$V/libwscodec_ca8.so python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_session.py tests/test_gpu_long_frames.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for rep in 1 2 3; do
  step c4_default_$rep 200 python3 tools/cfg_bench.py "configs[4]"
  step c4_ca7_$rep 200 env WSC_LIB=$V/libwscodec_ca7.so python3 tools/cfg_bench.py "configs[4]"
  step c4_ca8_$rep 200 env WSC_LIB=$V/libwscodec_ca8.so python3 tools/cfg_bench.py "configs[4]"
done
echo done
