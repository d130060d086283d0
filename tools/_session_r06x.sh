# r06x: the top-pass pruning at 8192:8192 x 1 KiB (the shape table's one regression) and
# neighbours: per-kernel times with RS_MI355X_BFLY_PRUNE=0 / 1, alternating
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06x
mkdir -p $O
for r in 1 2; do
  for v in 0 1; do
    echo "== round $r prune $v"
    RS_MI355X_BFLY_PRUNE=$v timeout -k 10 200 python -u tools/route_time.py 8192:8192:1024 16384:16384:1024 4096:4096:1024 --iters 50 || exit 1
  done
done > $O/route_prune.txt 2>&1
