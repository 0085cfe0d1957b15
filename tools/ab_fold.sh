#!/bin/bash
# The unmask's UTF-8 window fold with 1 / 2 (default) / 4 DFA chains per lane chunk
# (tools/build_variant.sh foldN -DWSC_FOLD_NCH=N): UTF-8 parity through WSC_LIB, then the TEXT
# configs, twice, interleaved with the in-tree library.
for v in fold4 fold1; do
  WSC_LIB=$PWD/tools/_var/libwscodec_$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_utf8.py > gpurun_out/${v}_pytest.log 2>&1 || { echo "$v FAILED"; tail -15 gpurun_out/${v}_pytest.log; exit 1; }
  echo "$v utf8: $(tail -1 gpurun_out/${v}_pytest.log)"
done
for rep in 1 2; do
  for v in default fold4 fold1; do
    if [ $v = default ]; then unset WSC_LIB; else export WSC_LIB=$PWD/tools/_var/libwscodec_$v.so; fi
    echo "=== $v rep $rep"
    timeout -k 10 300 python3 tools/cfg_bench.py "TEXT" || exit $?
  done
done
