#!/bin/bash
# Round 5 set 6: the encode scan (wave-strided rounds, messages per thread chosen per batch) and
# the copy's frame preload; the echo's read size per connection and round at 8 pollers.
o=gpurun_out/r05ab6; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 2 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
step enc_tests 300 python3 -u -m pytest tests/test_encode.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step enc_tests_pre 300 env WSC_LIB=$PWD/tools/_var/libwscodec_pre.so python3 -u -m pytest tests/test_encode.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
V=$PWD/tools/_var
for rep in 1 2; do
  step enc_r4_$rep 200 env WSC_LIB=$V/libwscodec_encipt.so WSC_ENC_IPT=16 python3 tools/enc_only.py
  step enc_ipt_$rep 200 env WSC_LIB=$V/libwscodec_encipt.so python3 tools/enc_only.py
  step enc_new_$rep 200 python3 tools/enc_only.py
  step enc_new16_$rep 200 env WSC_ENC_IPT=16 python3 tools/enc_only.py
  step enc_pre_$rep 200 env WSC_LIB=$V/libwscodec_pre.so python3 tools/enc_only.py
done
E="--conns 64 --frames 200 --size 65536 --client-threads 4 --pollers 8"
for rep in 1 2 3; do
  for rb in 4194304 1048576 262144; do
    step echo_gpu_${rb}_$rep 120 env ECHO_READ_BYTES=$rb tools/ws_echo $E
    step echo_cpu_${rb}_$rep 120 env ECHO_READ_BYTES=$rb oracle/_build/ws_echo_cpu $E
  done
done
echo done
