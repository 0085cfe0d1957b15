#!/bin/bash
# SQ passes of the TEXT 1 KiB decode (tools/single_loop.py t1) for two builds of the library:
#   bash tools/pmc_text_ab.sh <libA.so> <libB.so>  -> gpurun_out/pmctab/{A,B}_{p1,p2}.csv
out=gpurun_out/pmctab; mkdir -p $out; export TMPDIR=/tmp
P1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
P2="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
i=0
for lib in "$@"; do
  tag=$(echo AB | cut -c$((i+1))); i=$((i+1))
  for p in P1 P2; do
    rm -rf $out/tmp
    timeout -s KILL 90 rocprofv3 --pmc ${!p} -d $out/tmp -o run --output-format csv -- python3 tools/single_loop.py t1 3 --lib $lib > $out/log_${tag}_$p.txt 2>&1 || exit 1
    cp $(find $out/tmp -name '*counter_collection.csv' | head -1) $out/${tag}_$p.csv && rm -rf $out/tmp
    echo "$tag $p ok"
  done
done
