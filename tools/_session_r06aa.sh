# r06aa: per-kernel composition of the configs[2] / configs[3] decodes (route_time)
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06aa
mkdir -p $O
timeout -k 10 300 python -u tools/route_time.py 8192:8192:65536 32768:32768:1024 --iters 10 > $O/route_c34.txt 2>&1
