#!/usr/bin/env python3
"""Summarise a gpu_round.sh run into profiles/<tag>/.

Reads gpurun_out/<tag>/{kt,pmc_fetch,pmc_write} (rocprofv3 CSV output) and
writes
  profiles/<tag>/kernel_stats.csv   -- rocprofv3 --kernel-trace --stats summary
  profiles/<tag>/traffic.json       -- per-kernel average HBM-side bytes per launch
  profiles/<tag>/bench.json         -- the bench line of the same session
HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE (KiB) come from separate --pmc passes; on gfx950 FETCH_SIZE counts
half the bytes of a streaming read, so it is doubled.
"""
import collections
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def short(name):
    """'void rs::(anonymous namespace)::k_mono<10, 1, 0, true>(rs::MonoArgs)' -> 'k_mono<10, 1, 0, true>'"""
    m = re.search(r"(k_[a-z_]+(?:<[^()]*>)?)\(", name)
    return m.group(1) if m else name[:80]


def counter_means(path, counter):
    acc = collections.defaultdict(list)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    for f in ("bench.json", "bench_config3.json", "bench_config4.json", "bench_config5_n1.json"):
        if os.path.exists(os.path.join(src, f)) and os.path.getsize(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f))
    fetch = counter_means(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counter_means(os.path.join(src, "pmc_write", "run_counter_collection.csv"), "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) & set(write)):
        if not k.startswith("k_"):
            continue
        fb = fetch[k][0] * 1024 * 2  # KiB, gfx950 half-count correction
        wb = write[k][0] * 1024
        out[k] = {"fetch_bytes": round(fb), "write_bytes": round(wb), "hbm_bytes": round(fb + wb),
                  "launches": fetch[k][1]}
    with open(os.path.join(dst, "traffic.json"), "w") as f:
        json.dump({"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes ({tag})",
                   "correction": "FETCH_SIZE x2 (gfx950 half count; calibrated for the column kernel's 4-byte paired-lane "
                                 "pack reads by tools/fetch_calib.hip, profiles/r01j/fetch_calib_*.csv: a 512 MiB read "
                                 "reports 262,155 KiB, the 16 B/lane stream 262,147 KiB), KiB -> bytes",
                   "note": "FETCH counts L2 misses per XCD (Infinity-Cache hits included): tables read by every "
                           "workgroup are fetched once per XCD, 8x their size",
                   "kernels": out}, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
