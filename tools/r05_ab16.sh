#!/bin/bash
# Round 5 set 16: encode copy driven by the scan's window bitmaps (edge pieces and each piece's
# frame by popcount) vs the binary search: encode tests, timing, SQ counters.
o=gpurun_out/r05ab16; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 3 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
V=$PWD/tools/_var
step enc_tests 300 python3 -u -m pytest tests/test_encode.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for rep in 1 2 3; do
  step enc_old_$rep 200 env WSC_LIB=$V/libwscodec_encold.so python3 tools/enc_only.py
  step enc_bm_$rep 200 python3 tools/enc_only.py
done
step pmc_bm 300 bash tools/pmc_enc.sh $o/pmc_bm
echo done
