#!/bin/bash
# Column-kernel ablation set (tools/_build/mp_* built from tools/mono_probe.hip with
# RS_MONO_SKIP_* / RS_MONO_FAKE_TABS variants); output under gpurun_out/<tag>/.
set -euo pipefail
TAG=${1:-probe}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for b in tools/_build/mp_*; do
  n=$(basename "$b")
  { echo "== $n encode"; timeout -k 5 60 "$b" 1024 1024; echo "== $n decode 1%"; timeout -k 5 60 "$b" 2048 1024 d1;
    echo "== $n decode 100%"; timeout -k 5 60 "$b" 2048 1024 d;
    echo "== $n decode 1% split"; timeout -k 5 60 "$b" 2048 1024 d1s;
    echo "== $n decode 100% split"; timeout -k 5 60 "$b" 2048 1024 ds; } >> "$OUT/probe.txt" 2>&1
done
cat "$OUT/probe.txt"
