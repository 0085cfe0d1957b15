#!/bin/bash
# A/B of the walk's look-back order: ticket atomic (WSC_WALK_HW_ORDER=0, default) against the
# hardware workgroup index (=1): walk stamps (launch spread) and the configs the walk bounds, twice.
for o in 0 1; do
  echo "=== stamps WSC_WALK_HW_ORDER=$o"
  WSC_WALK_HW_ORDER=$o timeout -k 10 120 python3 tools/walk_stamps.py mixed || exit $?
  WSC_WALK_HW_ORDER=$o timeout -k 10 120 python3 tools/walk_stamps.py 1k1 || exit $?
done
for rep in 1 2; do
  for o in 0 1; do
    echo "=== WSC_WALK_HW_ORDER=$o rep $rep"
    WSC_WALK_HW_ORDER=$o timeout -k 10 300 python3 tools/cfg_bench.py "configs[1] 1M x 1 KiB BIN, 1" "configs[2]" "configs[4]" "TEXT 262144" || exit $?
  done
done
