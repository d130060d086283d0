#!/bin/bash
# Build a lane-kernel probe binary tools/_probe/<name> from tools/lane_probe.hip
# (A/B tooling); extra hipcc flags follow (e.g. -DRS_LANE_SKIP_LAYERS).
set -euo pipefail
NAME=$1; shift
mkdir -p tools/_probe
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -Ireed-solomon-simd_amd/csrc "$@" tools/lane_probe.hip \
  reed-solomon-simd_amd/csrc/gf_tables.cpp -o tools/_probe/$NAME
echo built tools/_probe/$NAME
