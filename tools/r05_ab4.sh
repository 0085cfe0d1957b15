#!/bin/bash
# Round 5 set 4: the check's next-unit prefetch (fits 128 VGPRs again), host-inclusive copy layouts
# (own contexts, copy streams per direction), persistent unmask grids on the small configs[2] batch.
o=gpurun_out/r05ab4; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 2 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
for rep in 1 2; do
  step text_pf0_$rep 200 python3 tools/cfg_bench.py TEXT
  step text_pf1_$rep 200 env WSC_LIB=$PWD/tools/_var/libwscodec_pf1.so python3 tools/cfg_bench.py TEXT
done
for rep in 1 2; do step hi_$rep 240 python3 tools/hi_probe.py; done
for w in 0 20 40; do step c2_wpc$w 200 env WSC_UNMASK_WPC=$w python3 tools/cfg_bench.py "configs[2] 256k mixed 125"; done
echo done
