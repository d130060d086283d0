# r06t: host enqueue cost against GPU time per call, C loop (tools/api_probe.cpp), small to headline shapes
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06t
mkdir -p $O
for s in "32 32 1024" "128 128 1024" "256 256 1024" "1024 1024 1024" "1000 100 1024" "4096 4096 1024"; do
  timeout -k 5 60 tools/probe_bin/api_probe $s || exit 1
done 2>&1 | grep -v amdgpu.ids | tee $O/api_probe.txt
