#!/bin/bash
# Round 5 set 14: host-inclusive pieces with the copies done by kernels (wsc_kcopy).
o=gpurun_out/r05ab14; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 12 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
step hi 400 python3 -u tools/hi_probe.py
echo done
