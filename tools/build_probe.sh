#!/bin/bash
# Build a column-kernel probe binary tools/probe_bin/<name> from tools/mono_probe.hip
# (A/B tooling).  SRC: kernel source to include (default: the in-tree rs_mono.hip);
# extra hipcc flags follow, e.g. -DRS_MONO_ONLY_L=11 -DRS_MONO_ONLY_MODE=2 for a
# decode-only build in a fraction of the compile time.
#   bash tools/build_probe.sh <name> [SRC=path] [flags...]
set -euo pipefail
NAME=$1; shift
SRC=""
if [[ "${1:-}" == SRC=* ]]; then SRC=$(realpath "${1#SRC=}"); shift; fi
mkdir -p tools/probe_bin
args=(--offload-arch=gfx950 -O3 -std=c++17 -Ireed-solomon-simd_amd/csrc "$@")
if [ -n "$SRC" ]; then args+=("-DRS_MONO_SRC=\"$SRC\""); fi
/opt/rocm/bin/hipcc "${args[@]}" tools/mono_probe.hip reed-solomon-simd_amd/csrc/gf_tables.cpp -o tools/probe_bin/$NAME
echo built tools/probe_bin/$NAME
