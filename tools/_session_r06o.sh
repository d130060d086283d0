# r06o: eval_poly with two LDS remaps (RS_MONO_EVAL_REMAP=1) against the four exchange rounds
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06o
mkdir -p $O
for r in 1 2 3; do
  for v in vd2_r0 vd2_r1; do
    for a in "2048 1024 d1s2n" "2048 1024 ds2" "1024 1024 d1s2n" "1024 1024 d2"; do
      t=$(timeout -k 5 30 tools/probe_bin/$v $a) || exit 1
      echo "$r $v [$a] $(echo "$t" | grep -m1 '^mono' | sed -E 's/.*: ([0-9.]+ us).*hash ([0-9a-f]+)/\1 \2/')"
    done
  done
done | tee $O/eval_remap_ab.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_random.py -k "decode or random" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_decode.log 2>&1
rc=$?; tail -2 $O/pytest_decode.log; exit $rc
