#!/bin/bash
# COMPACT two-pass edge windows (tools/build_variant.sh edge2 -DWSC_COMPACT_EDGE2=1): parity suites
# through WSC_LIB, then configs[4] against the in-tree library (twice) and the unmask's
# instructions per wave (SQ pass, tools/single_loop.py c4).
export TMPDIR=/tmp
V=$PWD/tools/_var/libwscodec_edge2.so
WSC_LIB=$V timeout -k 10 420 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_gpu_stream.py tests/test_gpu_pong_eof.py -k "compact or True or config4 or fragmented" > gpurun_out/edge2_pytest.log 2>&1 || { tail -20 gpurun_out/edge2_pytest.log; exit 1; }
tail -2 gpurun_out/edge2_pytest.log
for rep in 1 2; do
  for lib in default edge2; do
    if [ $lib = default ]; then unset WSC_LIB; else export WSC_LIB=$V; fi
    echo "=== $lib rep $rep"
    timeout -k 10 300 python3 tools/cfg_bench.py "configs[4]" "TEXT 16384" || exit $?
  done
done
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"
mkdir -p gpurun_out/edge2
for lib in default edge2; do
  if [ $lib = default ]; then unset WSC_LIB; else export WSC_LIB=$V; fi
  rm -rf gpurun_out/edge2/t_$lib
  timeout -s KILL 90 rocprofv3 --pmc $SQ -d gpurun_out/edge2/t_$lib -o run --output-format csv -- python3 tools/single_loop.py c4 3 > gpurun_out/edge2/log_$lib.txt 2>&1 || exit 1
  f=$(find gpurun_out/edge2/t_$lib -name '*counter_collection.csv' | head -1)
  cp "$f" gpurun_out/edge2/sq_$lib.csv && rm -rf gpurun_out/edge2/t_$lib
  echo "sq $lib ok"
done
