#!/bin/bash
# The round-5 half-split parity failure, made deterministic.
# kMonoHalfFEnc read the shared twiddle region (the FFT's first layers) with no
# barrier after every wave's writes to it.  Both variants below poison that
# region and hold back all waves but wave 0 before they write their pieces
# (-DRS_MONO_HALF_RACE_PROBE, rs_mono.hip):
#   race_nofix  also -DRS_MONO_NO_HALF_BARRIER (the round-5 code): wave 0 reads poison
#   race_fix    the committed barrier: every read waits for the writers
# Build here (CPU):  bash tools/build_variant.sh race_nofix rs_mono.hip -DRS_MONO_HALF_RACE_PROBE -DRS_MONO_NO_HALF_BARRIER
#                    bash tools/build_variant.sh race_fix rs_mono.hip -DRS_MONO_HALF_RACE_PROBE
# Run on the box:    bash tools/half_race_demo.sh <outdir>
set -uo pipefail
OUT=${1:-gpurun_out/half_race}
mkdir -p "$OUT"
source tools/ab_common.sh
for v in race_nofix race_fix; do
  use_lib $v
  timeout -k 10 240 python -u -m pytest tests/test_gpu_parity.py -k "half_split_encode or half_split_decode" \
    -q -p no:cacheprovider --timeout 120 --timeout-method thread > "$OUT/$v.log" 2>&1
  rc=$?
  echo "$v: pytest exit $rc" | tee -a "$OUT/summary.txt"
  tail -3 "$OUT/$v.log" >> "$OUT/summary.txt"
  # 0 = all passed, 1 = test failures (the expected outcome of race_nofix); anything
  # else (a timeout, a crash) ends the script
  if [ $rc -gt 1 ]; then exit $rc; fi
done
use_lib main
