# r06ag: the randomised GPU sweep on two more seeds, on the final build (top-pass pruning on)
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06ag
mkdir -p $O
for seed in 606 707; do
  RS_TEST_SEED=$seed timeout -k 10 500 python -u -m pytest tests/test_gpu_random.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/random_$seed.log 2>&1
  rc=$?; echo "seed $seed: $(tail -1 $O/random_$seed.log)"; [ $rc -eq 0 ] || exit $rc
done
