#!/bin/bash
# Round 5 set 11: every session staging copy by a kernel (wsc_kcopy, WSC_SESSION_KCOPY=2) vs the
# wire's H2D only (1) vs copy engines (0): session tests, launch timings, echo by pollers / read size.
o=gpurun_out/r05ab11; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 3 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
step tests 400 python3 -u -m pytest tests/test_gpu_session.py tests/test_gpu_tls.py tests/test_gpu_pong_eof.py tests/test_echo.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for L in 2 1 0; do
  step timing_P8_k$L 120 env WSC_SESSION_KCOPY=$L ECHO_TIMING=1 WSC_SESSION_TIMING=1 tools/ws_echo --conns 64 --frames 200 --size 65536 --client-threads 4 --pollers 8
done
for rep in 1 2 3; do
  for P in 1 4 8; do
    E="--conns 64 --frames 200 --size 65536 --client-threads 4 --pollers $P"
    for rb in 4194304 524288; do
      for L in 0 2; do step echo_k${L}_P${P}_${rb}_$rep 120 env WSC_SESSION_KCOPY=$L tools/ws_echo $E --read-bytes $rb; done
      step echo_cpu_P${P}_${rb}_$rep 120 oracle/_build/ws_echo_cpu $E --read-bytes $rb
    done
  done
  E="--conns 64 --frames 2000 --size 1024 --client-threads 4 --pollers 8"
  for L in 0 2; do step echo1k_k${L}_P8_$rep 120 env WSC_SESSION_KCOPY=$L tools/ws_echo $E; done
  step echo1k_cpu_P8_$rep 120 oracle/_build/ws_echo_cpu $E
  for L in 0 2; do step echo1c_k${L}_$rep 120 env WSC_SESSION_KCOPY=$L tools/ws_echo --conns 1 --frames 4000 --size 65536; done
  step echo1c_cpu_$rep 120 oracle/_build/ws_echo_cpu --conns 1 --frames 4000 --size 65536
done
echo done
