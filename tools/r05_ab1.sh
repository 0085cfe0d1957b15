#!/bin/bash
# Round 5 A/B set 1 (one box): walk issue priority (s_setprio) and the high-priority walk stream
# in the pipelines; the 1024-thread UTF-8 check; host-inclusive copy-stream layouts.
# Results in gpurun_out/r05ab1/; stops at the first failing step.
o=gpurun_out/r05ab1; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -2 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
step tls 300 python3 -u -m pytest tests/test_gpu_tls.py tests/test_gpu_pong_eof.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
HL="--steps 100 --warmup 5 --no-cpu --no-host-inclusive --no-echo --no-other-configs --no-config3"
for rep in 1 2; do
  step hl_default_$rep 120 python3 bench.py $HL
  step hl_noprio_$rep 120 env WSC_WALK_PRIO=0 python3 bench.py $HL
  step hl_priostream_$rep 120 python3 bench.py $HL --walk-prio 1
done
step cfg_prio 400 python3 tools/cfg_bench.py "configs[1]" "configs[2]" "configs[3]" "configs[4]"
step cfg_noprio 400 env WSC_WALK_PRIO=0 python3 tools/cfg_bench.py "configs[1]" "configs[2]" "configs[3]" "configs[4]"
step text_wpb4 200 python3 tools/cfg_bench.py TEXT "configs[2] 256k mixed 125"
step text_wpb16 200 env WSC_U8_WPB=16 python3 tools/cfg_bench.py TEXT "configs[2] 256k mixed 125"
step hi 300 python3 tools/hi_probe.py
echo done
