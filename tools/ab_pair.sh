#!/bin/bash
# A/B of the pair encode (two workgroups per pack) against one workgroup per pack
# on the headline encode: alternating bench runs + one kernel-trace pass each.
set -euo pipefail
TAG=${1:-ab_pair}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
ARGS="--no-cpu --no-host --no-copy --batch 1 --no-decode --steps 200 --warmup 20"
for r in 1 2; do
  RS_MI355X_PAIR=1 timeout -k 10 120 python -u bench.py $ARGS > "$OUT/pair_$r.json"
  RS_MI355X_PAIR=0 timeout -k 10 120 python -u bench.py $ARGS > "$OUT/nopair_$r.json"
done
timeout -k 10 120 python -u bench.py --no-cpu --no-host --no-copy --batch 1 --no-decode --steps 20 --warmup 5 > "$OUT/pair_steps20.json"
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d "$OUT/kt_pair" -o run -- python3 bench.py $ARGS > "$OUT/kt_pair.log" 2>&1
python3 tools/ab_show.py "$OUT" 2>/dev/null || true
for f in "$OUT"/*.json; do echo "$f $(python3 -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['avg_us'], d['roofline']['kernel'])")"; done
