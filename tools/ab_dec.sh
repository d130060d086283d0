#!/bin/bash
# GPU box: parity tests, then alternating back-to-back launch timings of column-kernel probe
# variants (tools/probe_bin/<prefix>_<variant>), then per-workgroup stamps of <prefix>_stamps.
# Usage: tools/ab_dec.sh <out-dir> <prefix> <n> <S> "<variants>" "<modes>" [rounds]
set -uo pipefail
OUT=$1; P=$2; N=$3; S=$4; VARS=$5; MODES=$6; ROUNDS=${7:-3}
mkdir -p "$OUT"
if [ "${SKIP_TESTS:-0}" != "1" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$OUT/pytest.log" 2>&1 || { tail -5 "$OUT/pytest.log"; exit 1; }
  tail -1 "$OUT/pytest.log"
fi
for r in $(seq "$ROUNDS"); do
  for v in $VARS; do
    for m in $MODES; do
      t=$(timeout -k 5 30 "tools/probe_bin/${P}_$v" "$N" "$S" "$m") || exit 1
      echo "$v $m $(echo "$t" | grep -m1 '^mono' | sed -E 's/.*: ([0-9.]+) us.*/\1/')"
    done
  done
done | tee "$OUT/ab.txt"
if [ -x "tools/probe_bin/${P}_stamps" ]; then
  for m in $MODES; do timeout -k 5 30 "tools/probe_bin/${P}_stamps" "$N" "$S" "$m" || exit 1; done > "$OUT/stamps.txt"
fi
