#!/bin/bash
# Build tools/_probe/chunks_probe (k_chunks timing + stamps) from tools/chunks_probe.hip;
# extra hipcc flags follow (e.g. -DRS_CHUNK_NO_STAMPS for the plain kernel).
#   bash tools/build_chunks_probe.sh [name] [flags...]
set -euo pipefail
NAME=${1:-chunks_probe}; shift || true
mkdir -p tools/_probe
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ireed-solomon-simd_amd/csrc "$@" tools/chunks_probe.hip \
    reed-solomon-simd_amd/csrc/gf_tables.cpp -o tools/_probe/$NAME
echo built tools/_probe/$NAME
