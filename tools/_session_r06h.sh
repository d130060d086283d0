# r06h: SQ counters of the quad encode against the 2-element column kernel (headline shape)
set -uo pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r06h
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for q in 0 1; do
  RS_MI355X_QUAD=$q timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM -f csv -d $O/pmc_q$q -o run \
    -- python3 tools/route_time.py 1024:1024:1024 --iters 100 > $O/pmc_q$q.log 2>&1 || exit $?
done
python3 - <<'PY' | tee $O/quad_sq.txt
import csv, glob, collections
for q in ("0", "1"):
    acc = collections.defaultdict(lambda: [0.0, set()])
    for f in glob.glob(f"gpurun_out/r06h/pmc_q{q}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "k_mono" not in r["Kernel_Name"] or ", 2>" in r["Kernel_Name"] and "k_mono<11" in r["Kernel_Name"]:
                continue
            key = (r["Kernel_Name"][:60], r["Counter_Name"])
            acc[key][0] += float(r["Counter_Value"]); acc[key][1].add(r["Dispatch_Id"])
    for k in sorted(acc):
        print("quad" if q == "1" else "e2", k[0], k[1], round(acc[k][0] / len(acc[k][1])))
PY
# world 8 rehearsal of bench.py --gpus 8 on this one GPU (gloo collectives; numbers meaningless)
RS_BENCH_REHEARSE=1 timeout -k 10 600 python -u bench.py --gpus 8 --steps 3 --warmup 1 --no-cpu --no-host --no-object --no-copy --batch 1 > $O/rehearse8.log 2>&1
rc=$?; grep -E '^\{"metric|"rank"' $O/rehearse8.log | cut -c1-400; exit $rc
