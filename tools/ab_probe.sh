#!/bin/bash
# A/B of column-kernel probe binaries (tools/_probe/<name>, built from tools/mono_probe.hip):
# back-to-back launch time of the headline encode (1024:1024 x 1 KiB) and decodes
# (2048 work rows, 1 % and 100 % loss, split plan), alternating the binaries R times.
#   bash tools/ab_probe.sh <tag> <rounds> <bin> [bin...]     (output: gpurun_out/<tag>/ab_probe.txt)
set -euo pipefail
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p "$OUT"
for ((i = 0; i < R; ++i)); do
  for b in "$@"; do
    for a in "1024 1024" "2048 1024 d1s" "2048 1024 ds"; do
      echo "== $b $a (round $i)" >> "$OUT/ab_probe.txt"
      timeout -k 5 60 tools/_probe/$b $a >> "$OUT/ab_probe.txt" 2>&1 || echo "rc=$?" >> "$OUT/ab_probe.txt"
    done
  done
done
grep -E "^==|us/launch" "$OUT/ab_probe.txt"
