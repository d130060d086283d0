#!/bin/bash
# LDS / VALU SQ counters (one rocprofv3 --pmc pass) over a bench config:
#   bash tools/pmc_lds_bench.sh <tag> <bench args...>
set -euo pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG/lds_bench
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
C="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_ACTIVE_INST_LDS SQ_BUSY_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $C -f csv -d "$OUT" -o run -- python3 bench.py "$@" > "$OUT/run.log" 2>&1
