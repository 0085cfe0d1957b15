#!/bin/bash
# PMC passes (FETCH, WRITE, SQ) and a kernel trace of the encode batches (tools/enc_time.py)
set -e
mkdir -p gpurun_out/pmcenc
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmcenc/f -o run --output-format csv -- python3 tools/enc_time.py > gpurun_out/pmcenc/f.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmcenc/w -o run --output-format csv -- python3 tools/enc_time.py > gpurun_out/pmcenc/w.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc $SQ -d gpurun_out/pmcenc/s -o run --output-format csv -- python3 tools/enc_time.py > gpurun_out/pmcenc/s.log 2>&1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d gpurun_out/pmcenc/k -o run -- python3 tools/enc_time.py > gpurun_out/pmcenc/k.log 2>&1
