#!/bin/bash
# Round 5 set 9: where a GPU poller's submit goes (session launch timing) at 4 / 8 pollers; the
# pipelined leg's serial order on one context.
o=gpurun_out/r05ab9; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 3 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
for P in 8 4 1; do
  step timing_P$P 120 env ECHO_TIMING=1 WSC_SESSION_TIMING=1 tools/ws_echo --conns 64 --frames 200 --size 65536 --client-threads 4 --pollers $P
done
step timing_P8_512k 120 env ECHO_TIMING=1 WSC_SESSION_TIMING=1 tools/ws_echo --conns 64 --frames 200 --size 65536 --client-threads 4 --pollers 8 --read-bytes 524288
step cfg 400 python3 tools/cfg_bench.py "configs[1]"
echo done
