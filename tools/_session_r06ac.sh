# r06ac (library: tools/build_variant.sh k7 with the K = 7 pruning patch): configs[3] decode levels with the top-pass pruning extended to K = 7: default
# (6-bit, 3 levels) against RS_MI355X_MAX_K=7 (2 levels, pruned K = 7 top pass); GPU suite first
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
cp reed-solomon-simd_amd/lib/variants/librs_mi355x_k7.so reed-solomon-simd_amd/lib/librs_mi355x.so  # the K = 7 pruning build
O=gpurun_out/r06ac
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
RS_MI355X_MAX_K=7 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "pruned or large or baseline_decode or decode_device" > $O/pytest_maxk7.log 2>&1
rc=$?; tail -2 $O/pytest_maxk7.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for k in def 7; do
    echo "== round $r max_k $k"
    if [ $k = def ]; then timeout -k 10 200 python -u tools/route_time.py 8192:8192:65536 8192:8192:1024 4096:4096:65536 --iters 8 || exit 1
    else RS_MI355X_MAX_K=$k timeout -k 10 200 python -u tools/route_time.py 8192:8192:65536 8192:8192:1024 4096:4096:65536 --iters 8 || exit 1; fi
  done
done > $O/route_maxk7.txt 2>&1
