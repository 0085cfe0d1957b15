#!/bin/bash
# kernel trace of one-batch-in-flight decode loops, one config per trace (kernel durations and the
# gaps between them without other configs' launches mixed in):
#   bash tools/kt_configs.sh c2 c21 c11 ...   -> gpurun_out/kt/<cfg>/, gaps in gpurun_out/kt/<cfg>.txt
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/kt
for x in "$@"; do
  timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/kt/$x -o run -- python3 tools/single_loop.py $x 100 > gpurun_out/kt/$x.log 2>&1
  f=$(find gpurun_out/kt/$x -name 'run_kernel_trace.csv' | head -1)
  python3 tools/kt_gaps.py "$f" > gpurun_out/kt/$x.txt
  echo "== $x"; cat gpurun_out/kt/$x.txt
done
