"""2-element vs 4-element column kernel (development tool): per-launch time of the
headline-shaped encode / decode over several shard sizes (grid = shard_bytes / 4
or / 8 workgroups), through pre-bound C-ABI calls."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "reed-solomon-simd_amd"))
import reed_solomon_simd as rs  # noqa: E402

N = M = 1024


def t_us(fn, steps=300):
    for _ in range(30):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / steps * 1e6


for S in (512, 768, 896, 960, 1024, 1280, 1536):
    d_o = torch.randint(0, 256, (N, S), dtype=torch.uint8, device="cuda")
    d_r = torch.empty((M, S), dtype=torch.uint8, device="cuda")
    enc = rs.encode_device_call(N, M, S, d_o, d_r)
    L = 10
    op = np.ones(N, np.uint8)
    op[:L] = 0
    rp = np.zeros(M, np.uint8)
    rp[:L] = 1
    d_out = torch.empty_like(d_o)
    dec = rs.decode_device_call(N, M, S, d_o, op, d_r, rp, d_out)
    row = [f"S={S:5d}"]
    for flag, name in ((1 | 8, "e4"), (1 | 16, "e2")):
        rs.mono_enable(flag)
        row.append(f"{name} enc {t_us(enc):6.2f} dec {t_us(dec):6.2f}")
    rs.mono_enable(1)
    print("  ".join(row), flush=True)
