# r06u: block pruning of the multi-pass decode's fused top pass (RS_MI355X_BFLY_PRUNE=1)
# against none (=0): GPU suite, then configs 3 and 4 alternating
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06u
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 1; do
    RS_MI355X_BFLY_PRUNE=$v timeout -k 10 200 python -u bench.py --no-cpu --config 8192x8192x64k --steps 10 --warmup 2 > $O/c4_p${v}_r$r.json 2>> $O/bench.err || exit 1
    RS_MI355X_BFLY_PRUNE=$v timeout -k 10 200 python -u bench.py --no-cpu --config 32768x32768x1k --steps 50 --warmup 5 > $O/c3_p${v}_r$r.json 2>> $O/bench.err || exit 1
    echo "round $r prune $v done"
  done
done
