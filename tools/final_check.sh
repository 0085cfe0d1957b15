#!/bin/bash
# A second pass of the GPU suite and smoke on the final tree (stability), plus the N=2 control path
# rehearsed with gloo ranks sharing the box's one GPU.
o=gpurun_out/final2; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -n 3 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
step pytest 560 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 120 python3 -c "import __graft_entry__ as g; g.smoke()"
step n2 300 env WSC_BENCH_BACKEND=gloo python3 bench.py --gpus 2 --steps 20 --warmup 3 --no-cpu --no-host-inclusive --no-echo --no-other-configs
echo done
