#!/bin/bash
# Round 5 set 2: the GPU suite on the edge-table build, then UTF-8 edge tables on/off (TEXT lines),
# the host-inclusive copy layouts again, and the other_configs lines with the serial candidate.
o=gpurun_out/r05ab2; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -2 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
step utf8 400 python3 -u -m pytest tests/test_gpu_utf8.py tests/test_gpu_pong_eof.py tests/test_gpu_stream.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step pytest 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
for rep in 1 2; do
  step text_edge1_$rep 200 python3 tools/cfg_bench.py TEXT
  step text_edge0_$rep 200 env WSC_U8_EDGE=0 python3 tools/cfg_bench.py TEXT
done
step hi 300 python3 tools/hi_probe.py
step cfg 500 python3 tools/cfg_bench.py "configs[1]" "configs[2]" "configs[3]" "configs[4]"
echo done
