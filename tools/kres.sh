#!/bin/bash
# Register / occupancy summary of the column kernels (development aid).
# Usage: tools/kres.sh [extra hipcc flags...]   (run from the repo root)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 "$@" -c reed-solomon-simd_amd/csrc/rs_mono.hip \
  -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "Function Name|VGPRs:|Spill|Occupancy" | sed -E 's/.*remark: +//; s/ \[-Rpass.*//' |
  paste - - - - - | sed -E 's/Function Name: _ZN2rs12_GLOBAL__N_16k_monoILi([0-9]+)ELi([0-9]+)ELi([0-9]+)ELb([01])ELb([01])ELb([01])ELi([0-9])E[^\t]*/k_mono<\1,\2,\3,\4,\5,\6,\7>/'
