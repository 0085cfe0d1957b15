#!/bin/bash
# A/B of environment settings on one library: each setting (A then B) runs the named other_configs
# lines, twice, interleaved.   bash tools/ab_env.sh "A settings" "B settings" [config fragments ...]
A="$1"; B="$2"; shift 2
for rep in 1 2; do
  for set in "$A" "$B"; do
    echo "=== [$set] rep $rep"
    env $set timeout -k 10 300 python3 tools/cfg_bench.py "$@" || exit $?
  done
done
