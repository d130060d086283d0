#!/usr/bin/env python3
"""Summarise a gpu_round.sh run into profiles/<tag>/.

Reads gpurun_out/<tag>/ (rocprofv3 CSV output of tools/gpu_round.sh) and writes
  profiles/<tag>/kernel_stats.csv       -- rocprofv3 --kernel-trace --stats summary (headline bench)
  profiles/<tag>/kernel_stats_<cfg>.csv -- the same for the other configs' benches, when run
  profiles/<tag>/traffic.json           -- per config and kernel: average HBM-side bytes and VALU
                                           wave-instructions per launch
  (the SQ pass is summarised per kernel into traffic.json: mean of each counter per launch;
   the raw per-dispatch CSV stays in gpurun_out/)
  profiles/<tag>/bench*.json            -- the bench lines of the same session
HBM bytes follow /opt/skills/guides/MI355X_MICROARCH.md "HBM": FETCH_SIZE and
WRITE_SIZE (KiB) come from separate --pmc passes; on gfx950 FETCH_SIZE counts
half the bytes of a streaming read, so it is doubled.  SQ_INSTS_VALU (a third
pass with the other SQ counters) is the sum over all waves of a dispatch.
"""
import collections
import csv
import json
import os
import re
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADLINE = "1024x1024x1k"


def short(name):
    """'void rs::(anonymous namespace)::k_mono<10, 1, 0, true>(rs::MonoArgs)' -> 'k_mono<10, 1, 0, true>'"""
    m = re.search(r"(k_[a-z_]+(?:<[^()]*>)?)\(", name)
    return m.group(1) if m else name[:80]


def counter_means(path, counter):
    acc = collections.defaultdict(list)
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                acc[short(r["Kernel_Name"])].append(float(r["Counter_Value"]))
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def summarise(d):
    """d: directory holding fetch/, write/, sq/ rocprofv3 outputs of one bench command."""
    fetch = counter_means(os.path.join(d, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write = counter_means(os.path.join(d, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    sq = os.path.join(d, "sq", "run_counter_collection.csv")
    valu = counter_means(sq, "SQ_INSTS_VALU")
    names = set()
    if os.path.exists(sq):
        with open(sq) as f:
            names = {r["Counter_Name"] for r in csv.DictReader(f)}
    sq_all = {c: counter_means(sq, c) for c in sorted(names)}
    out = {}
    for k in sorted(set(fetch) | set(valu)):
        if not k.startswith("k_"):
            continue
        e = {}
        if k in fetch and k in write:
            fb = fetch[k][0] * 1024 * 2  # KiB, gfx950 half-count correction
            wb = write[k][0] * 1024
            e.update(fetch_bytes=round(fb), write_bytes=round(wb), hbm_bytes=round(fb + wb), launches=fetch[k][1])
        if k in valu:
            e.update(valu_insts=round(valu[k][0]), valu_launches=valu[k][1])
            e["sq"] = {c: round(m[k][0]) for c, m in sq_all.items() if k in m}
        out[k] = e
    return out


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", tag)
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    for f in sorted(os.listdir(src)):
        if f.startswith("bench") and f.endswith(".json") and os.path.getsize(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f))
    configs = {}
    pmc = os.path.join(src, "pmc")
    for cfg in sorted(os.listdir(pmc)) if os.path.isdir(pmc) else []:
        configs[cfg] = summarise(os.path.join(pmc, cfg))
    kt = os.path.join(src, "kt")
    for cfg in sorted(os.listdir(kt)) if os.path.isdir(kt) else []:
        f = os.path.join(kt, cfg, "run_kernel_stats.csv")
        if os.path.exists(f):
            shutil.copy(f, os.path.join(dst, "kernel_stats.csv" if cfg == HEADLINE else f"kernel_stats_{cfg}.csv"))
    with open(os.path.join(dst, "traffic.json"), "w") as f:
        json.dump({"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ counters, separate passes per bench "
                             f"config ({tag})",
                   "correction": "FETCH_SIZE x2 (gfx950 half count; calibrated for the column kernel's 4-byte "
                                 "paired-lane pack reads by tools/fetch_calib.hip, profiles/r01j/fetch_calib_*.csv: "
                                 "a 512 MiB read reports 262,155 KiB, the 16 B/lane stream 262,147 KiB), KiB -> bytes",
                   "note": "FETCH counts L2 misses per XCD (Infinity-Cache hits included); valu_insts = SQ_INSTS_VALU "
                           "per launch, summed over all waves",
                   "configs": configs, "kernels": configs.get(HEADLINE, {})}, f, indent=1)
    print(json.dumps(configs, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r02")
