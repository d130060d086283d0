# r06j: one-shot encode: direct pageable D2H into the caller's buffer vs pinned staging + CopyPool
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06j
mkdir -p $O
for r in 1 2 3; do
  for d in 0 1; do
    echo "direct=$d $(RS_MI355X_ONESHOT_DIRECT=$d timeout -k 5 120 reed-solomon-simd_amd/lib/rs_object_bench 1024 1024 1024 300 20)" || exit 1
  done
done | tee $O/oneshot_direct.txt
RS_MI355X_ONESHOT_DIRECT=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "c_oneshot" -q --timeout 120 --timeout-method thread -p no:cacheprovider 2>&1 | tail -2
