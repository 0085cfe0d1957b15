#!/bin/bash
# A/B: non-temporal header loads in the walk (tools/build_variant.sh hdrnt -DWSC_HDR_NT=1) against
# the default build: FETCH_SIZE of the walk kernels at configs[2] / configs[1] 1 frame/segment, then
# the configs the walk bounds, twice.
export TMPDIR=/tmp
V=tools/_var/libwscodec_hdrnt.so
mkdir -p gpurun_out/hdrnt
for lib in default hdrnt; do
  if [ $lib = hdrnt ]; then export WSC_LIB=$PWD/$V; else unset WSC_LIB; fi
  for c in c2 c11; do
    rm -rf gpurun_out/hdrnt/t_$lib_$c
    timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/hdrnt/t_${lib}_$c -o run --output-format csv -- python3 tools/single_loop.py $c 3 > gpurun_out/hdrnt/log_${lib}_$c.txt 2>&1 || exit 1
    f=$(find gpurun_out/hdrnt/t_${lib}_$c -name '*counter_collection.csv' | head -1)
    cp "$f" gpurun_out/hdrnt/fetch_${lib}_$c.csv && rm -rf gpurun_out/hdrnt/t_${lib}_$c
    echo "fetch $lib $c ok"
  done
done
for rep in 1 2; do
  for lib in default hdrnt; do
    if [ $lib = hdrnt ]; then export WSC_LIB=$PWD/$V; else unset WSC_LIB; fi
    echo "=== $lib rep $rep"
    timeout -k 10 300 python3 tools/cfg_bench.py "configs[1] 1M x 1 KiB BIN, 1" "configs[2]" "configs[4]" || exit $?
  done
done
