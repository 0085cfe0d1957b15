#!/bin/bash
# Round 5 set 3: echo decoders (per-poller sessions, --blocking-wait, --batcher) at 1/4/8 pollers,
# interleaved, 3 reps; host-inclusive copy layouts x3; other_configs with the serial candidate;
# configs[1] with the quad pre-pass walk geometry (mode 65).
o=gpurun_out/r05ab3; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 2 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
step echo 600 python3 tools/echo_ab.py
for rep in 1 2; do step hi_$rep 200 python3 tools/hi_probe.py; done
step cfg 500 python3 tools/cfg_bench.py "configs[1]" "configs[2]" "configs[3]" "configs[4]"
step cfg_mode65 300 env WSC_WALK_MODE=65 python3 tools/cfg_bench.py "configs[1] 1M x 1 KiB BIN, 16"
for rep in 1 2; do
  step text_pf0_$rep 200 python3 tools/cfg_bench.py TEXT
  step text_pf1_$rep 200 env WSC_LIB=$PWD/tools/_var/libwscodec_pf1.so python3 tools/cfg_bench.py TEXT
done
echo done
