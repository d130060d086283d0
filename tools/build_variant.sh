#!/bin/bash
# Build reed-solomon-simd_amd/lib/variants/librs_mi355x_<name>.so: the given sources
# recompiled with extra hipcc flags, linked with the main build's other objects
# (A/B of kernel variants: tools/ab_common.sh puts it in place of the main build).
#   bash tools/build_variant.sh <name> "<src> [src...]" -DFOO ...
set -euo pipefail
NAME=$1; SRCS=$2; shift 2
PKG=reed-solomon-simd_amd
B=$PKG/build/variant_$NAME
mkdir -p "$B" $PKG/lib/variants
objs=()
for src in rs_kernels.hip rs_mono.hip rs_lane.hip rs_chunks.hip rs_eval.hip rs_codec.cpp gf_tables.cpp; do
  if [[ " $SRCS " == *" $src "* ]]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC "$@" -c $PKG/csrc/$src -o $B/$src.o
    objs+=($B/$src.o)
  else
    objs+=($PKG/build/$src.o)
  fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $PKG/lib/variants/librs_mi355x_$NAME.so "${objs[@]}"
echo built $PKG/lib/variants/librs_mi355x_$NAME.so
