#!/bin/bash
# A/B of the UTF-8 check merged into the unmask launch (WSC_U8_MERGE=1, default) against its own
# launch (WSC_U8_MERGE=0): every other_configs line, twice each, same box.  (Historical: the merge
# was reverted after this A/B, profiles/r04_u8_merge_ab.log; WSC_U8_MERGE no longer exists.)
for rep in 1 2; do
  for m in 0 1; do
    echo "=== WSC_U8_MERGE=$m rep $rep"
    WSC_U8_MERGE=$m timeout -k 10 400 python3 tools/cfg_bench.py || exit $?
  done
done
