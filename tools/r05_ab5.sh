#!/bin/bash
# Round 5 set 5: walk mode 257 (one segment per lane, 3 blocks per CU) vs the tiled walk at 1 M
# one-frame segments, really pinned this time; the encode copy's buffer stores.
o=gpurun_out/r05ab5; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 2 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
for rep in 1 2; do
  step c11_tiled_$rep 200 python3 tools/cfg_bench.py "configs[1] 1M x 1 KiB BIN, 1 frame"
  step c11_m257_$rep 200 env WSC_WALK_MODE=257 python3 tools/cfg_bench.py "configs[1] 1M x 1 KiB BIN, 1 frame"
  step enc0_$rep 200 python3 tools/enc_only.py
  step enc1_$rep 200 env WSC_ENC_BUF=1 python3 tools/enc_only.py
done
step ca_tests 400 env WSC_LIB=$PWD/tools/_var/libwscodec_ca.so python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_utf8.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
for rep in 1 2; do
  step c4_default_$rep 200 python3 tools/cfg_bench.py "configs[4]"
  step c4_aligned_$rep 200 env WSC_LIB=$PWD/tools/_var/libwscodec_ca.so python3 tools/cfg_bench.py "configs[4]"
done
step echo_timing_gpu 120 env ECHO_TIMING=1 WSC_SESSION_TIMING=1 tools/ws_echo --conns 64 --frames 200 --size 65536 --client-threads 4 --pollers 8
step echo_timing_cpu 120 env ECHO_TIMING=1 oracle/_build/ws_echo_cpu --conns 64 --frames 200 --size 65536 --client-threads 4 --pollers 8
step echo_timing_gpu4 120 env ECHO_TIMING=1 WSC_SESSION_TIMING=1 tools/ws_echo --conns 64 --frames 200 --size 65536 --client-threads 4 --pollers 4
for rep in 1 2; do
  step text_base_$rep 200 python3 tools/cfg_bench.py TEXT
  step text_cls_$rep 200 env WSC_LIB=$PWD/tools/_var/libwscodec_cls.so python3 tools/cfg_bench.py TEXT
done
step n2_rehearsal 300 env WSC_BENCH_BACKEND=gloo python3 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu --no-host-inclusive --no-echo --no-other-configs
echo done
