"""Column-slice probe (development tool): the config-5 encode (32768:32768 x 64 KiB) as
one call vs k calls on column slices of w = S / k bytes (each slice's work rows fit
the Infinity Cache, so passes 2 and 3 re-read them from there instead of HBM)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "reed-solomon-simd_amd"))
import reed_solomon_simd as rs  # noqa: E402

N = M = int(sys.argv[1]) if len(sys.argv) > 1 else 32768
S = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
d_o = torch.randint(0, 256, (N, S), dtype=torch.uint8, device="cuda")
d_r = torch.empty((M, S), dtype=torch.uint8, device="cuda")
ref = None
for k in (1, 2, 4, 8, 16, 32, 64):
    w = S // k
    calls = [rs.encode_device_call(N, M, w, d_o[:, i * w:(i + 1) * w], d_r[:, i * w:(i + 1) * w]) for i in range(k)]
    for _ in range(2):
        for c in calls:
            c()
    torch.cuda.synchronize()
    if ref is None:
        ref = d_r.clone()
    else:
        assert torch.equal(ref, d_r), k
    steps = 5
    t = time.perf_counter()
    for _ in range(steps):
        for c in calls:
            c()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    print(f"slices {k:3d} (w = {w:6d} B, work {N * w / 2**20:7.1f} MiB): {dt * 1e3:7.3f} ms  "
          f"{(N + M) * S / dt / 2**30:8.1f} GiB/s", flush=True)
