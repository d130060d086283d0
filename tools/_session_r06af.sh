# r06af: the default line with 4 warmup steps in the sharded block (2 before), twice
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06af
mkdir -p $O
for r in 1 2 3; do
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu > $O/line_r$r.json 2>> $O/bench.err || exit 1
  python3 -c "import json;d=json.load(open('$O/line_r$r.json'));s=d['sharded'];print('round $r', d['value'], s['step_ms'], s['GiBps'], s['per_gpu_roofline']['achieved'], s['decode_1pct']['step_ms'])"
done
