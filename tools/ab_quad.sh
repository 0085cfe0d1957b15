#!/bin/bash
# A/B of the fused walk's quad pre-pass (WSC_QUAD_PRE=0 / 1): the bench.py other_configs lines it
# touches and the headline, twice each, same box.
HL="--steps 200 --warmup 10 --no-cpu --no-host-inclusive --no-echo --no-other-configs --no-config3"
for rep in 1 2; do
  for q in 0 1; do
    echo "=== WSC_QUAD_PRE=$q rep $rep"
    WSC_QUAD_PRE=$q timeout -k 10 300 python3 tools/cfg_bench.py "configs[1] 1M x 1 KiB BIN, 16" "configs[2]" "configs[4]" "TEXT 262144" || exit $?
    WSC_QUAD_PRE=$q timeout -k 10 120 python3 bench.py $HL || exit $?
  done
done
