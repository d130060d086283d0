"""E=2 vs E=4 column-kernel encode A/B (development aid): python tools/e2_encode_ab.py N M S
Alternates rs_mono_enable(1 | 8) (4-element packs) and (1 | 16) (2-element packs), 500 encodes
each, and asserts the recovery rows are identical."""
import os, sys, time
sys.path.insert(0, os.path.join(os.getcwd(), "reed-solomon-simd_amd"))
import torch
import reed_solomon_simd as rs
N, M, S = (int(a) for a in sys.argv[1:4])
d_orig = torch.randint(0, 256, (N, S), dtype=torch.uint8, device="cuda")
outs = {}
for mode in (1 | 8, 1 | 16, 1 | 8, 1 | 16):
    rs.mono_enable(mode)
    d_rec = torch.empty((M, S), dtype=torch.uint8, device="cuda")
    call = rs.encode_device_call(N, M, S, d_orig, d_rec)
    for _ in range(20): call()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(500): call()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 500
    outs.setdefault(mode, []).append(dt * 1e6)
    if mode != (1 | 8):
        assert torch.equal(d_rec, ref), "E=2 encode differs"
    else:
        ref = d_rec.clone()
print(N, M, S, {("e4" if k == (1 | 8) else "e2"): [round(x, 2) for x in v] for k, v in outs.items()})
