"""Summarise tools/valu_account.sh: mean SQ counters per launch of the k_mono kernel in
each (variant, mode) pass, and the difference of every ablation from the full kernel."""
import csv
import glob
import os
import sys
from collections import defaultdict

out = sys.argv[1]
rows = {}
for d in sorted(glob.glob(os.path.join(out, "v?_*.*"))):
    if not os.path.isdir(d):
        continue
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        continue
    acc = defaultdict(lambda: [0.0, set()])
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if "k_mono" not in r.get("Kernel_Name", ""):
                    continue
                a = acc[r["Counter_Name"]]
                a[0] += float(r["Counter_Value"])
                a[1].add(r.get("Dispatch_Id", r.get("Correlation_Id")))
    rows[os.path.basename(d)] = {k: v[0] / max(1, len(v[1])) for k, v in acc.items()}
ctr = ["SQ_INSTS_VALU", "SQ_WAVES", "SQ_INSTS_LDS", "SQ_INSTS_SALU"]
print("# SQ counters per k_mono launch (mean over the probe's launches); VALU/wave = SQ_INSTS_VALU / SQ_WAVES")
print(f"{'variant.mode':24s} " + " ".join(f"{c:>14s}" for c in ctr) + f" {'VALU/wave':>10s} {'dVALU vs full':>14s}")
for name in sorted(rows):
    r = rows[name]
    v, m = name.split(".")
    full = rows.get(f"{v[:2]}_full.{m}", {})
    dv = r.get("SQ_INSTS_VALU", 0) - full.get("SQ_INSTS_VALU", 0) if full else 0
    vw = r.get("SQ_INSTS_VALU", 0) / max(1.0, r.get("SQ_WAVES", 1))
    print(f"{name:24s} " + " ".join(f"{r.get(c, 0):14.0f}" for c in ctr) + f" {vw:10.1f} {dv:14.0f}")
