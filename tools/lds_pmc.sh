#!/bin/bash
# LDS counters of the column kernel (tools/_build/mp_base, headline encode and
# the 1 % decode): one rocprofv3 --pmc pass each; CSVs under gpurun_out/<tag>/lds.
set -euo pipefail
TAG=${1:-lds}
OUT=gpurun_out/$TAG/lds
mkdir -p "$OUT"
C="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
timeout -s KILL 60 rocprofv3 --pmc $C -f csv -d "$OUT/enc" -o run -- tools/_build/mp_base 1024 1024 > "$OUT/enc.txt" 2>&1
timeout -s KILL 60 rocprofv3 --pmc $C -f csv -d "$OUT/dec" -o run -- tools/_build/mp_base 2048 1024 d1 > "$OUT/dec.txt" 2>&1
