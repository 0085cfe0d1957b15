#!/bin/bash
# PMC passes over the encode kernels (tools/enc_loop.py), one counter group per run under its own
# kill timer; summarised by tools/pmc_enc.py.  usage: bash tools/pmc_enc.sh <outdir>
out="$1"; mkdir -p "$out"; export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
for pass in fetch write sq; do
  case $pass in fetch) ctr="FETCH_SIZE" ;; write) ctr="WRITE_SIZE" ;; sq) ctr="$SQ" ;; esac
  rm -rf "$out/tmp_$pass"
  timeout -s KILL 90 rocprofv3 --pmc $ctr -d "$out/tmp_$pass" -o run --output-format csv -- python3 tools/enc_loop.py 3 > "$out/log_$pass.txt" 2>&1
  rc=$?; if [ $rc -ne 0 ]; then echo "pass $pass rc=$rc"; tail -5 "$out/log_$pass.txt"; exit $rc; fi
  f=$(find "$out/tmp_$pass" -name '*counter_collection.csv' | head -1)
  cp "$f" "$out/$pass.csv" && rm -rf "$out/tmp_$pass"
  echo "pass $pass ok"
done
