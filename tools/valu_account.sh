#!/bin/bash
# VALU accounting of the headline column kernels: SQ counters per
# launch of tools/mono_probe.hip builds with one part ablated each (RS_MONO_SKIP_*,
# tools/build_probe.sh; vd_* = the 2^11-row decode, ve_* = the 2^10-row encode, 2-element
# packs, 1 KiB shards).  One rocprofv3 --pmc pass per (variant, mode); summary by
# tools/valu_account.py.
#   bash tools/valu_account.sh <outdir>
set -uo pipefail
OUT=${1:-gpurun_out/valu}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # run <variant> <n> <mode>
  local v=$1 n=$2 m=$3
  timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU -f csv -d "$OUT/$v.$m" -o run \
    -- tools/probe_bin/$v $n 1024 $m > "$OUT/$v.$m.log" 2>&1
}
for v in vd_full vd_noeval vd_nolayers vd_noxpose vd_noremap vd_nostage vd_noio vd_noscale vd_nosplittop vd_noscalemul vd_noreveal vd_skeleton; do
  for m in d1s2 ds2; do run $v 2048 $m || exit $?; done
done
for v in ve_full ve_nolayers ve_noxpose ve_noremap ve_nostage ve_noio ve_skeleton; do
  run $v 1024 e2 || exit $?
done
python3 tools/valu_account.py "$OUT" > "$OUT/summary.txt"
cat "$OUT/summary.txt"
