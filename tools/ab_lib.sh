#!/bin/bash
# A/B of an experiment build (tools/build_variant.sh <name>) against the in-tree library, through
# WSC_LIB: walk stamps (tiled 1 M segments, mixed) and the named other_configs lines, twice each.
#   bash tools/ab_lib.sh <name> [config name fragments ...]
name=$1; shift
V=$PWD/tools/_var/libwscodec_$name.so
for lib in default $name; do
  if [ $lib = default ]; then unset WSC_LIB; else export WSC_LIB=$V; fi
  echo "=== stamps $lib"
  timeout -k 10 120 python3 tools/walk_stamps.py 1k1 || exit $?
  timeout -k 10 120 python3 tools/walk_stamps.py mixed || exit $?
done
for rep in 1 2; do
  for lib in default $name; do
    if [ $lib = default ]; then unset WSC_LIB; else export WSC_LIB=$V; fi
    echo "=== $lib rep $rep"
    timeout -k 10 300 python3 tools/cfg_bench.py "$@" || exit $?
  done
done
