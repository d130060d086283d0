# r06b: the bench line (configs 2-5), its kernel trace, and the column kernels' VALU accounting
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06b
mkdir -p $O
t0=$SECONDS
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || exit $?
echo "bench wall s: $((SECONDS - t0))" | tee $O/bench_wall.txt
tail -c 2300 $O/bench.json
bash tools/valu_account.sh $O/valu || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $O/kt -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu > $O/kt.log 2>&1 || exit $?
echo done
