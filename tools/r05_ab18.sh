#!/bin/bash
# COMPACT unmask at configs[4]: SQ counters and traffic, byte-aligned dwordx4 stores (default) vs
# aligned 16-byte stores through a lane funnel (WSC_COMPACT_ALIGNED)
o=gpurun_out/r05ab18; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 3 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
step pmc_default 400 bash tools/pmc_walk.sh $o/default c4
step pmc_aligned 400 env WSC_LIB=$PWD/tools/_var/libwscodec_ca.so bash tools/pmc_walk.sh $o/aligned c4
echo done
