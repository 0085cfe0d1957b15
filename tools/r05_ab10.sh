#!/bin/bash
# Round 5 set 10: the session's wire staged by the fetch kernel (wsc_fetch) vs hipMemcpyAsync:
# session tests, then the echo at 1 / 4 / 8 pollers by read size, interleaved, and the timings.
o=gpurun_out/r05ab10; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 3 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
step tests 400 python3 -u -m pytest tests/test_gpu_session.py tests/test_gpu_tls.py tests/test_echo.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
step timing_P8 120 env ECHO_TIMING=1 WSC_SESSION_TIMING=1 tools/ws_echo --conns 64 --frames 200 --size 65536 --client-threads 4 --pollers 8
for rep in 1 2 3; do
  for P in 1 4 8; do
    E="--conns 64 --frames 200 --size 65536 --client-threads 4 --pollers $P"
    for rb in 4194304 524288; do
      step echo_memcpy_P${P}_${rb}_$rep 120 env WSC_SESSION_FETCH=0 tools/ws_echo $E --read-bytes $rb
      step echo_fetch_P${P}_${rb}_$rep 120 tools/ws_echo $E --read-bytes $rb
      step echo_cpu_P${P}_${rb}_$rep 120 oracle/_build/ws_echo_cpu $E --read-bytes $rb
    done
  done
  E="--conns 64 --frames 2000 --size 1024 --client-threads 4 --pollers 8"
  step echo1k_memcpy_P8_$rep 120 env WSC_SESSION_FETCH=0 tools/ws_echo $E
  step echo1k_fetch_P8_$rep 120 tools/ws_echo $E
  step echo1k_cpu_P8_$rep 120 oracle/_build/ws_echo_cpu $E
  step echo1c_memcpy_$rep 120 env WSC_SESSION_FETCH=0 tools/ws_echo --conns 1 --frames 4000 --size 65536
  step echo1c_fetch_$rep 120 tools/ws_echo --conns 1 --frames 4000 --size 65536
done
echo done
