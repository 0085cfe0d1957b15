#!/bin/bash
# An experiment build of libwscodec.so with extra -D flags, for A/B runs (tools/lib_ab.py, ab_lib.sh):
#   bash tools/build_variant.sh <name> -DFLAG ...   -> tools/_var/libwscodec_<name>.so
set -e
name=$1; shift
cd "$(dirname "$0")/../netman_amd/csrc"
out=../../tools/_var; mkdir -p $out
objs=()
for s in wsc_kernels.hip wsc_unmask_inplace.hip wsc_unmask_compact.hip wsc_encode.hip wsc_api.cpp wsc_session.cpp; do
  o=/tmp/var_${name}_$s.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall "$@" -x hip -c $s -o $o &
  objs+=($o)
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libwscodec_$name.so "${objs[@]}"
echo "$out/libwscodec_$name.so"
