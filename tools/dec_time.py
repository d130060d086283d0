"""Time one decode shape on the device (development aid): python tools/dec_time.py N M S [loss|enc]
Prints the mean us per decode of `iters` back-to-back calls (1 % loss pattern of
benches/benchmarks.rs:113-118 by default; "enc": the encode instead).  Environment knobs
(RS_MI355X_*) apply."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402
import reed_solomon_simd as rs  # noqa: E402

N, M, S = (int(a) for a in sys.argv[1:4])
enc = len(sys.argv) > 4 and sys.argv[4] == "enc"
loss = float(sys.argv[4]) if len(sys.argv) > 4 and not enc else 0.01
iters = 50
d_orig = torch.randint(0, 256, (N, S), dtype=torch.uint8, device="cuda")
d_rec = torch.empty((M, S), dtype=torch.uint8, device="cuda")
rs.encode_device(N, M, S, d_orig, d_rec)
if enc:
    call = rs.encode_device_call(N, M, S, d_orig, d_rec)
    for _ in range(5):
        call()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        call()
    torch.cuda.synchronize()
    print(f"{N}:{M}x{S} encode: {(time.perf_counter() - t0) / iters * 1e6:.2f} us")
    sys.exit(0)
L = max(1, -(-int(min(N, M) * loss * 100) // 100))
op = np.ones(N, np.uint8)
op[N - L:] = 0
rp = np.zeros(M, np.uint8)
rp[:L] = 1
d_out = torch.zeros_like(d_orig)
call = rs.decode_device_call(N, M, S, d_orig, op, d_rec, rp, d_out)
for _ in range(5):
    call()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(iters):
    call()
torch.cuda.synchronize()
dt = (time.perf_counter() - t0) / iters
miss = torch.from_numpy(op == 0).cuda()
ok = torch.equal(d_out[miss], d_orig[miss])
print(f"{N}:{M}x{S} loss {loss}: {dt * 1e6:.2f} us  restored_ok={ok}")
