# r06v: kernel trace of the configs[3] bench (decode 1 % / 100 %) with the top-pass pruning
set -uo pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06v
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 bench.py --no-cpu --no-host --no-copy --batch 1 --config 8192x8192x64k --steps 5 --warmup 2 > $O/kt.log 2>&1
