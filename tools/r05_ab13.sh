#!/bin/bash
# Round 5 set 13: replies sent straight from the decoders' message data (sendmsg of views) vs
# copied into an out buffer first, both servers; session/echo tests; the two-buffer decode leg.
o=gpurun_out/r05ab13; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 3 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
V=$PWD/tools/_var
step tests 400 python3 -u -m pytest tests/test_gpu_session.py tests/test_gpu_tls.py tests/test_gpu_pong_eof.py tests/test_echo.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step timing_P8 120 env ECHO_TIMING=1 WSC_SESSION_TIMING=1 tools/ws_echo --conns 64 --frames 200 --size 65536 --client-threads 4 --pollers 8
for rep in 1 2 3; do
  for P in 1 4 8; do
    E="--conns 64 --frames 200 --size 65536 --client-threads 4 --pollers $P"
    for rb in 4194304 524288; do
      step echo_gcopy_P${P}_${rb}_$rep 120 $V/ws_echo_copy $E --read-bytes $rb
      step echo_gzc_P${P}_${rb}_$rep 120 tools/ws_echo $E --read-bytes $rb
      step echo_ccopy_P${P}_${rb}_$rep 120 $V/ws_echo_cpu_copy $E --read-bytes $rb
      step echo_czc_P${P}_${rb}_$rep 120 oracle/_build/ws_echo_cpu $E --read-bytes $rb
    done
  done
  E="--conns 64 --frames 2000 --size 1024 --client-threads 4 --pollers 8"
  step echo1k_gzc_P8_$rep 120 tools/ws_echo $E
  step echo1k_czc_P8_$rep 120 oracle/_build/ws_echo_cpu $E
  step echo1c_gzc_$rep 120 tools/ws_echo --conns 1 --frames 4000 --size 65536
  step echo1c_czc_$rep 120 oracle/_build/ws_echo_cpu --conns 1 --frames 4000 --size 65536
done
step cfg 400 python3 tools/cfg_bench.py "configs[1]"
echo done
