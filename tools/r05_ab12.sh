#!/bin/bash
# Round 5 set 12: the whole GPU suite on the current tree; the other configs' legs.
o=gpurun_out/r05ab12; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 3 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
step pytest 700 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step cfg 500 python3 tools/cfg_bench.py "configs"
echo done
