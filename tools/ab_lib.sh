#!/bin/bash
# A/B of an experiment build (tools/build_variant.sh <name>) against the in-tree library: walk
# stamps (tiled 1 M segments, mixed) and the named other_configs lines, twice each.
#   bash tools/ab_lib.sh <name> [config name fragments ...]
name=$1; shift
V=$PWD/tools/_var/libwscodec_$name.so
D=$PWD/netman_amd/libwscodec.so
for lib in $D $V; do
  echo "=== stamps $lib"
  timeout -k 10 120 python3 tools/walk_stamps.py 1k1 --lib $lib || exit $?
  timeout -k 10 120 python3 tools/walk_stamps.py mixed --lib $lib || exit $?
done
for rep in 1 2; do
  for lib in $D $V; do
    echo "=== $lib rep $rep"
    timeout -k 10 300 python3 tools/lib_ab.py $lib configs "$@" || exit $?
  done
done
