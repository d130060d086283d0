#!/usr/bin/env python3
"""Decode time of 8192:8192 x 64 KiB for loss patterns (tail / random, 1 % and 100 %):
how much the pruned FFT passes save when losses are contiguous vs scattered.
Run it under RS_MI355X_DECODE_PRUNE=0 / 1 (tools/ab_prune.sh semantics). One JSON line."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))
import reed_solomon_simd as rs  # noqa: E402

N = M = 8192
S = 65536
dev = torch.device("cuda", 0)
g = torch.Generator(device=dev).manual_seed(0)
orig = torch.randint(0, 256, (N, S), dtype=torch.uint8, device=dev, generator=g)
rec = torch.empty((M, S), dtype=torch.uint8, device=dev)
out = torch.empty_like(orig)
rs.encode_device(N, M, S, orig, rec)
res = {}
rng = np.random.default_rng(1)
for name, L, random in (("tail_1pct", 82, False), ("random_1pct", 82, True), ("random_10pct", 820, True),
                        ("all_100pct", N, False)):
    op = np.ones(N, np.uint8)
    op[rng.choice(N, L, replace=False) if random else np.arange(N - L, N)] = 0
    rp = np.zeros(M, np.uint8)
    rp[:L] = 1
    call = rs.decode_device_call(N, M, S, orig, op, rec, rp, out)
    for _ in range(2):
        call()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        call()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    miss = torch.from_numpy(op == 0).to(dev)
    assert torch.equal(out[miss], orig[miss]), name
    res[name] = {"ms": round(ms, 3), "GiBps": round((N + M) * S / (ms / 1e3) / 2**30, 1)}
print(json.dumps({"prune_mode": os.environ.get("RS_MI355X_DECODE_PRUNE", "0"), "decode_8192x8192x64k": res}))
