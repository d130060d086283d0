#!/bin/bash
# A/B of the decode pruning modes (RS_MI355X_DECODE_PRUNE: 0 all, 1 none, 2 store masks only)
set -euo pipefail
mkdir -p gpurun_out/ab
for i in 1 2; do
  for m in 0 1; do
    RS_MI355X_DECODE_PRUNE=$m timeout -k 10 100 python -u bench.py --no-cpu --no-host --batch 1 --config 32768x32768x1k --steps 200 --warmup 10 > gpurun_out/ab/c3_m${m}_$i.json
    RS_MI355X_DECODE_PRUNE=$m timeout -k 10 100 python -u bench.py --no-cpu --no-host --batch 1 --config 8192x8192x64k --steps 10 --warmup 2 > gpurun_out/ab/c4_m${m}_$i.json
  done
done
