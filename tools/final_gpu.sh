#!/bin/bash
# End-of-round evidence on one box: GPU suite, smoke, the default bench, a kernel trace of the
# bench, and the headline's PMC traffic passes (FETCH_SIZE / WRITE_SIZE, separate runs).
# Results in gpurun_out/final/; stops at the first failure.
o=gpurun_out/final; mkdir -p $o; export TMPDIR=/tmp
step() { name=$1; secs=$2; shift 2; echo "=== $name"; timeout -k 10 $secs "$@" > $o/$name.log 2>&1; rc=$?; tail -3 $o/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; exit $rc; }; }
[ -n "$NO_PYTEST" ] || step pytest 560 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider
step smoke 120 python3 -c "import __graft_entry__ as g; g.smoke()"
step bench 400 python3 -u bench.py
step trace 300 rocprofv3 --kernel-trace --stats -d $o/trace -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu --no-host-inclusive --no-echo
HL="--steps 5 --warmup 2 --no-cpu --no-host-inclusive --no-echo --no-other-configs --no-config3"
step fetch 120 rocprofv3 --pmc FETCH_SIZE -d $o/fetch -o run --output-format csv -- python3 bench.py $HL
step write 120 rocprofv3 --pmc WRITE_SIZE -d $o/write -o run --output-format csv -- python3 bench.py $HL
echo done
