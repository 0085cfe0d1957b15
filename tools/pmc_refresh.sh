#!/bin/bash
# PMC passes (FETCH / WRITE / SQ, each its own run) of the decode kernels for the BASELINE configs on
# the current tree: gpurun_out/pmc_r06/ -> python tools/pmc_walk.py gpurun_out/pmc_r06
export TMPDIR=/tmp
timeout -k 10 900 bash tools/pmc_walk.sh gpurun_out/pmc_r06 head c1 c11 c2 c4
