#!/bin/bash
# unmask blocks per XCD run (WSC_XCD_RUN: 1 = the hardware's round-robin deal): headline, configs[3],
# configs[4] COMPACT, configs[1]
HL="--steps 200 --warmup 10 --no-cpu --no-host-inclusive --no-echo --no-other-configs --no-config3"
for rep in 1 2; do
  for x in ${RUNS:-1 4 8 16 32}; do
    echo "=== WSC_XCD_RUN=$x rep $rep"
    WSC_XCD_RUN=$x timeout -k 10 200 python3 tools/cfg_bench.py "configs[4]" "configs[3]" "configs[1] 1M x 1 KiB BIN, 16" || exit $?
    WSC_XCD_RUN=$x timeout -k 10 120 python3 bench.py $HL || exit $?
  done
done
