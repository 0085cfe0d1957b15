#!/bin/bash
# PMC passes (one counter group per run, each under its own kill timer) of tools/single_loop.py for
# the walk / unmask kernels; summarised by tools/pmc_walk.py.  usage: bash tools/pmc_walk.sh <outdir> <cfg>...
out="$1"; shift
mkdir -p "$out"
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
for c in "$@"; do
  for pass in fetch write sq; do
    case $pass in
      fetch) ctr="FETCH_SIZE" ;;
      write) ctr="WRITE_SIZE" ;;
      sq) ctr="$SQ" ;;
    esac
    rm -rf "$out/tmp_${pass}_$c"
    timeout -s KILL 90 rocprofv3 --pmc $ctr -d "$out/tmp_${pass}_$c" -o run --output-format csv -- python3 tools/single_loop.py "$c" 3 > "$out/log_${pass}_$c.txt" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "pass $pass $c rc=$rc"; tail -5 "$out/log_${pass}_$c.txt"; exit $rc; fi
    f=$(find "$out/tmp_${pass}_$c" -name '*counter_collection.csv' | head -1)
    cp "$f" "$out/${pass}_$c.csv" && rm -rf "$out/tmp_${pass}_$c"
    echo "pass $pass $c ok"
  done
done
