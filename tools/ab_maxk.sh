#!/bin/bash
# Level size A/B (RS_MI355X_MAX_K: caps encode and decode pass levels) on configs 3 and 4
set -euo pipefail
mkdir -p gpurun_out/abk
for i in 1 2; do
  for k in 5 6 7 8; do
    RS_MI355X_MAX_K=$k timeout -k 10 100 python -u bench.py --no-cpu --no-host --no-copy --batch 1 --config 32768x32768x1k --steps 200 --warmup 10 > gpurun_out/abk/c3_k${k}_$i.json
    RS_MI355X_MAX_K=$k timeout -k 10 100 python -u bench.py --no-cpu --no-host --no-copy --batch 1 --config 8192x8192x64k --steps 10 --warmup 2 > gpurun_out/abk/c4_k${k}_$i.json
  done
done
