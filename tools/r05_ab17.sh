#!/bin/bash
# Round 5 set 17: the sequential encode copy (waves own runs of windows, frames kept in lanes;
# WSC_ENC_SEQ=1) vs one window per wave: encode tests both ways, timing, SQ counters.
o=gpurun_out/r05ab17; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 3 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
step enc_tests 300 python3 -u -m pytest tests/test_encode.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step enc_tests_seq 300 env WSC_ENC_SEQ=1 python3 -u -m pytest tests/test_encode.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for rep in 1 2 3; do
  step enc_base_$rep 200 python3 tools/enc_only.py
  step enc_seq_$rep 200 env WSC_ENC_SEQ=1 python3 tools/enc_only.py
done
step pmc_seq 300 env WSC_ENC_SEQ=1 bash tools/pmc_enc.sh $o/pmc_seq
echo done
