#!/bin/bash
# Round 5 set 8: encode copy variants at 1 KiB (frames loaded into 16 lanes first; nt loads in the
# lane-parallel windows) with their HBM reads; the echo server sending round r before waiting
# for round r+1 (old harness binary vs new), by read size.
o=gpurun_out/r05ab8; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 2 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
V=$PWD/tools/_var
step enc_tests_nl16 300 env WSC_LIB=$V/libwscodec_nl16nte.so python3 -u -m pytest tests/test_encode.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for rep in 1 2; do
  step enc_base_$rep 200 python3 tools/enc_only.py
  for v in nl16 nte nl16nte; do step enc_${v}_$rep 200 env WSC_LIB=$V/libwscodec_$v.so python3 tools/enc_only.py; done
done
for v in base nl16 nte; do
  L=""; [ $v = base ] || L="WSC_LIB=$V/libwscodec_$v.so"
  step fetch_$v 90 env $L rocprofv3 --pmc FETCH_SIZE -d $o/pmc_$v -o run --output-format csv -- python3 tools/enc_loop.py 3
done
for rep in 1 2 3; do
  for P in 4 8; do
    E="--conns 64 --frames 200 --size 65536 --client-threads 4 --pollers $P"
    for rb in 4194304 524288; do
      step echo_old_P${P}_${rb}_$rep 120 env LD_LIBRARY_PATH=$PWD/netman_amd $V/ws_echo_old $E --read-bytes $rb
      step echo_new_P${P}_${rb}_$rep 120 tools/ws_echo $E --read-bytes $rb
      step echo_cpu_P${P}_${rb}_$rep 120 oracle/_build/ws_echo_cpu $E --read-bytes $rb
    done
  done
done
echo done
