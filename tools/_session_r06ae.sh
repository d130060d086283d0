# r06ae: the default line's configs[4] (sharded) encode step read 4.9-5.1 ms in r06w / r06ad
# against 4.1-4.2 before; default lines with RS_MI355X_BFLY_PRUNE=0 / 1, alternating
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ae
mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    RS_MI355X_BFLY_PRUNE=$v timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu > $O/line_p${v}_r$r.json 2>> $O/bench.err || exit 1
    python3 -c "import json;d=json.load(open('$O/line_p${v}_r$r.json'));s=d['sharded'];print('round $r prune $v', s['step_ms'], s['GiBps'], s['per_gpu_roofline']['achieved'], s['decode_1pct']['step_ms'])"
  done
done
