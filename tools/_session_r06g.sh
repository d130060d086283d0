# r06g: the quad encode -- its parity tests, then a same-box A/B against the 2-element column kernel
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "quad" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_quad.log 2>&1
rc=$?; tail -15 $O/pytest_quad.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for q in 0 1; do
    RS_MI355X_QUAD=$q timeout -k 10 120 python -u tools/route_time.py 1024:1024:1024 1024:1024:512 1000:1000:576 1024:1024:256 --iters 300 > $O/route_q${q}_$r.jsonl 2>&1 || exit $?
  done
done
python3 - <<'PY' | tee gpurun_out/r06g/quad_ab.txt
import json, glob, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/r06g/route_q*_*.jsonl")):
    q = f.split("route_q")[1][0]
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            e = d["encode"]
            acc[(d["shape"], q)].append((e["wall_us"], [(k["name"], k["avg_us"]) for k in e["kernels"]]))
for k in sorted(acc):
    print(k[0], "quad" if k[1] == "1" else "e2  ", "wall us", [w for w, _ in acc[k]], "kernel us", [ks for _, ks in acc[k]][0])
PY
