#!/bin/bash
# Round 5 set 7: the encode scan as adopted (tests + timing); the echo's read size per connection
# and round at 1 / 4 / 8 pollers (GPU session vs CPU port); PMC passes over the encode kernels.
o=gpurun_out/r05ab7; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 2 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
step enc_tests 300 python3 -u -m pytest tests/test_encode.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step enc_1 200 python3 tools/enc_only.py
step enc_2 200 python3 tools/enc_only.py
for rep in 1 2 3; do
  for P in 1 4 8; do
    E="--conns 64 --frames 200 --size 65536 --client-threads 4 --pollers $P"
    for rb in 4194304 1048576 524288; do
      step echo_gpu_P${P}_${rb}_$rep 120 tools/ws_echo $E --read-bytes $rb
    done
    for rb in 4194304 1048576; do
      step echo_cpu_P${P}_${rb}_$rep 120 oracle/_build/ws_echo_cpu $E --read-bytes $rb
    done
  done
  E="--conns 64 --frames 2000 --size 1024 --client-threads 4 --pollers 8"
  for rb in 4194304 1048576; do
    step echo1k_gpu_P8_${rb}_$rep 120 tools/ws_echo $E --read-bytes $rb
    step echo1k_cpu_P8_${rb}_$rep 120 oracle/_build/ws_echo_cpu $E --read-bytes $rb
  done
done
step pmc_enc 400 bash tools/pmc_enc.sh $o/pmc
echo done
