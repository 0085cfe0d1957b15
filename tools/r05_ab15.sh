#!/bin/bash
# Round 5 set 15: wsc_kcopy's reachability guard (session tests) and the echo with it.
o=gpurun_out/r05ab15; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 3 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
step tests 400 python3 -u -m pytest tests/test_gpu_session.py tests/test_echo.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step echo_P8 120 tools/ws_echo --conns 64 --frames 200 --size 65536 --client-threads 4 --pollers 8
echo done
