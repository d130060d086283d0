# r06d: the decode's destination narrowed to the erased rows' span -- probe A/B, GPU suite, bench
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06d
mkdir -p $O
for r in 1 2 3; do
  for m in d1s2 d1s2n ds2; do
    t=$(timeout -k 5 30 tools/probe_bin/vd_time 2048 1024 $m) || exit 1
    echo "$r $m $(echo "$t" | grep -m1 '^mono')"
  done
done | tee $O/ab_narrow.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-configs --no-sharded > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "
import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('encode', d['value'], d['us_per_step'], 'decode', d['decode_GiBps']['1pct'], d['decode_GiBps']['100pct'], d['decode_GiBps']['roofline_1pct']['avg_us'], 'obj', d['object_api'])"
