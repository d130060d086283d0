#!/bin/bash
# Alternating A/B of the decode pruning on config 3 only (no other workload between runs)
set -euo pipefail
mkdir -p gpurun_out/ab3
for i in 1 2 3; do
  for m in 0 1; do
    RS_MI355X_DECODE_PRUNE=$m timeout -k 10 100 python -u bench.py --no-cpu --no-host --no-copy --batch 1 --config 32768x32768x1k --steps 400 --warmup 20 > gpurun_out/ab3/c3_m${m}_$i.json
  done
done
