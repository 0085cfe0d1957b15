#!/bin/bash
# Round 5 set 8: encode copy variants at 1 KiB (frames loaded into 16 lanes first; nt loads in the
# lane-parallel windows) with their HBM reads; the echo server sending round r before waiting
# for round r+1 (old harness binary vs new), by read size.
o=gpurun_out/r05ab8b; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 2 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
V=$PWD/tools/_var
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
