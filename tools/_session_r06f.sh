# r06f: feasibility of a 4-rows-per-lane headline encode: k_mono<9, E=4> on 256 workgroups
# (512:512 x 2 KiB = the quad layout's transform core) against the headline k_mono<10, E=2>
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06f
mkdir -p $O
for r in 1 2 3; do
  for a in "1024 1024 e2" "512 2048 e4" "512 1024 e4" "512 1024 e2" "1024 2048 e4"; do
    t=$(timeout -k 5 30 tools/probe_bin/ve_all $a) || exit 1
    echo "$r [$a] $(echo "$t" | grep -m1 '^mono')"
  done
done | tee $O/quad_feasibility.txt
