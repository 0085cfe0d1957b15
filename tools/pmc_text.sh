#!/bin/bash
# SQ passes (instruction mix, waits, LDS conflicts) for the TEXT decodes (tools/single_loop.py t1 / t64)
out=gpurun_out/pmctext; mkdir -p $out; export TMPDIR=/tmp
A="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
B="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
for c in t1 t64; do
  for p in A B; do
    ctr=${!p}
    timeout -s KILL 90 rocprofv3 --pmc $ctr -d $out/tmp_${p}_$c -o run --output-format csv -- python3 tools/single_loop.py $c 3 > $out/log_${p}_$c.txt 2>&1 || exit 1
    cp $(find $out/tmp_${p}_$c -name '*counter_collection.csv' | head -1) $out/${p}_$c.csv && rm -rf $out/tmp_${p}_$c
  done
done
