#!/bin/bash
# GPU-box driver: runs each step under its own time limit; stops at the first fault/abort/timeout.
# usage: bash tools/gpu_run.sh <name>:<seconds>:<command> ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%:*}"; rest="${spec#*:}"; secs="${rest%%:*}"; cmd="${rest#*:}"
  echo "=== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "$name rc=$rc" | tee -a "gpurun_out/$name.log"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then echo "fatal rc=$rc in $name: stopping"; exit $rc; fi
done
