# r06q: per-layer table addresses computed once up front (RS_MONO_PRE_ADDR=1) against
# the per-layer slot arithmetic (=0), 2^10-row encode and decode probes
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06q
mkdir -p $O
for r in 1 2 3; do
  for p in pa0 pa1; do
    for a in "e 1024 1024 e2" "e 1024 512 e2" "d 1024 1024 d1s2n" "d 1024 1024 d2"; do
      set -- $a
      t=$(timeout -k 5 30 tools/probe_bin/${1}_$p $2 $3 $4) || exit 1
      echo "$r ${1}_$p [$2 $3 $4] $(echo "$t" | grep -m1 '^mono' | sed -E 's/.*: ([0-9.]+ us).*hash ([0-9a-f]+)/\1 \2/')"
    done
  done
done | tee $O/pre_addr_ab.txt
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for p in e_pa0 e_pa1; do
  timeout -s KILL 60 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU -f csv -d $O/pmc_$p -o run -- tools/probe_bin/$p 1024 1024 e2 > $O/pmc_$p.log 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; exit $rc
