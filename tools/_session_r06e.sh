# r06e: one-shot copy threads
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06e
mkdir -p $O
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count())" | tee $O/cpus.txt
for r in 1 2; do
  for t in 0 1 3 7; do
    echo "threads=$t $(RS_MI355X_COPY_THREADS=$t timeout -k 5 120 reed-solomon-simd_amd/lib/rs_object_bench 1024 1024 1024 200 10)" || exit 1
  done
done | tee $O/oneshot_threads.txt
