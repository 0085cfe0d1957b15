#!/bin/bash
# The UTF-8 check at TEXT 64 KiB / 1 KiB: kernel trace (tools/kt_configs.sh) and one SQ pass
# (tools/single_loop.py t64 / t1).  -> gpurun_out/kt/<cfg>.txt, gpurun_out/pmc_check/sq_<cfg>.csv
export TMPDIR=/tmp
bash tools/kt_configs.sh t64 t1 || exit 1
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
mkdir -p gpurun_out/pmc_check
for c in t64 t1; do
  rm -rf gpurun_out/pmc_check/t_$c
  timeout -s KILL 90 rocprofv3 --pmc $SQ -d gpurun_out/pmc_check/t_$c -o run --output-format csv -- python3 tools/single_loop.py $c 3 > gpurun_out/pmc_check/log_$c.txt 2>&1 || exit 1
  f=$(find gpurun_out/pmc_check/t_$c -name '*counter_collection.csv' | head -1)
  cp "$f" gpurun_out/pmc_check/sq_$c.csv && rm -rf gpurun_out/pmc_check/t_$c
  echo "sq $c ok"
done
