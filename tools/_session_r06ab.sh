# r06ab: configs[3] decode levels with the pruned top pass: default (6-bit, 3 levels) against
# RS_MI355X_MAX_K=7 (2 levels, top pass K = 7: no butterfly pruning there) and 8
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ab
mkdir -p $O
for r in 1 2; do
  for k in def 7; do
    echo "== round $r max_k $k"
    if [ $k = def ]; then timeout -k 10 200 python -u tools/route_time.py 8192:8192:65536 --iters 8 || exit 1
    else RS_MI355X_MAX_K=$k timeout -k 10 200 python -u tools/route_time.py 8192:8192:65536 --iters 8 || exit 1; fi
  done
done > $O/route_maxk.txt 2>&1
