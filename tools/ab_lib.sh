#!/bin/bash
# Alternating A/B of library variants on the headline bench (encode + decode 1 % / 100 %):
#   bash tools/ab_lib.sh <tag> <rounds> main <variant> ...   (variant: lib/variants/librs_mi355x_<v>.so)
set -euo pipefail
source "$(dirname "$0")/ab_common.sh"
TAG=$1; R=$2; shift 2
OUT=gpurun_out/$TAG; mkdir -p $OUT
ARGS="--no-cpu --no-host --no-copy --batch 1 --steps 200 --warmup 20"
for r in $(seq 1 $R); do
  for v in "$@"; do
    use_lib $v
    timeout -k 10 120 python -u bench.py $ARGS > $OUT/${v}_$r.json
    python3 -c "import json; d=json.load(open('$OUT/${v}_$r.json')); x=d['decode_GiBps']; print('$v', $r, d['value'], d['roofline']['avg_us'], x['1pct_us_per_step']['gpu_events'], x['100pct_us_per_step']['gpu_events'])"
  done
done
