#!/bin/bash
# Alternate probe binaries tools/_probe/<bin> over R rounds on the given modes
# (args "n S mode"), printing "<bin> <mode> <us/launch>" lines (A/B tooling).
#   bash tools/ab_bins.sh <out> <rounds> "<n S mode>;<n S mode>" bin...
set -uo pipefail
OUT=$1; R=$2; MODES=$3; shift 3
mkdir -p "$(dirname "$OUT")"
IFS=';' read -ra MS <<< "$MODES"
for ((i = 0; i < R; ++i)); do
  for b in "$@"; do
    for m in "${MS[@]}"; do
      t=$(timeout -k 5 60 tools/_probe/$b $m 2>&1) || { echo "$b $m FAILED: $t"; exit 1; }
      echo "$b $m $(echo "$t" | grep -m1 '^mono' | sed -E 's/.*: ([0-9.]+) us.*/\1/')"
    done
  done
done | tee "$OUT"
