# r06i: per-workgroup stamps of the headline decode (1 %, split plan), destination narrowed or not
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06i
mkdir -p $O
for m in d1s2n d1s2 ds2; do
  echo "== $m"; timeout -k 5 60 tools/probe_bin/vd_stamps 2048 1024 $m || exit 1
done > $O/decode_stamps.txt 2>&1
cat $O/decode_stamps.txt
