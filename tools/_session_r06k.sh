# r06k: one-shot copies in on the pool or on the calling thread (copies out always on the pool)
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06k
mkdir -p $O
for r in 1 2 3; do
  for c in 1 0; do
    echo "copyin_pool=$c $(RS_MI355X_COPYIN_POOL=$c timeout -k 5 120 reed-solomon-simd_amd/lib/rs_object_bench 1024 1024 1024 300 20)" || exit 1
  done
done | tee $O/oneshot_copyin.txt
