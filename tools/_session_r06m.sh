# r06m: the random sweep on three more seeds (narrowed decode destination, quad route, all routes)
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06m
mkdir -p $O
for sd in 0x51 0xA2 0xF3; do
  RS_TEST_SEED=$sd timeout -k 10 400 python -u -m pytest tests/test_gpu_random.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/random_$sd.log 2>&1
  rc=$?; echo "seed $sd: $(tail -1 $O/random_$sd.log)"; [ $rc -eq 0 ] || exit $rc
done
