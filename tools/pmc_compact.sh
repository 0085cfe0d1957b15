#!/bin/bash
# configs[4] COMPACT store-policy variants: time (tools/compact_probe.py) and, per variant, a
# WRITE_SIZE pass (its own rocprofv3 run under a kill timer)
out=gpurun_out/pmc_c4; mkdir -p $out; export TMPDIR=/tmp
timeout -k 10 240 python3 tools/compact_probe.py 20 > $out/probe.log 2>&1 || exit $?
for v in 0 1 4 5; do
  rm -rf $out/tmp_$v
  WSC_PROBE_VARIANT=$v timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $out/tmp_$v -o run --output-format csv -- python3 tools/compact_probe.py 3 > $out/log_$v.txt 2>&1 || exit $?
  f=$(find $out/tmp_$v -name '*counter_collection.csv' | head -1); cp "$f" $out/write_$v.csv; rm -rf $out/tmp_$v
done
echo done
