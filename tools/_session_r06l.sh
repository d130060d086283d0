# r06l: one-shot encode with the recovery rows back in 1 / 2 / 4 / 8 pieces (copy-out overlapped)
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "c_oneshot" -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_oneshot.log 2>&1
rc=$?; tail -2 $O/pytest_oneshot.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for k in 1 2 4 8; do
    echo "pieces=$k $(RS_MI355X_ONESHOT_PIECES=$k timeout -k 5 120 reed-solomon-simd_amd/lib/rs_object_bench 1024 1024 1024 300 20)" || exit 1
  done
done | tee $O/oneshot_pieces.txt
