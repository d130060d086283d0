"""Per-launch GPU time of one call's kernels (development aid): for each shape, the
kernels one encode / decode call launches (rs_profile_enable: HIP events around
every launch on the call's stream) averaged over `iters` calls, and the wall time
per call of back-to-back calls.  Decode: the 1 % / 100 % loss pattern of
benches/benchmarks.rs:113-138.  Usage: python tools/route_time.py N:M[:S] ... [--iters K]"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))
import torch  # noqa: E402
import reed_solomon_simd as rs  # noqa: E402


def profile(call, iters):
    call()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        call()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / iters
    rs.profile_enable(True)
    for _ in range(iters):
        call()
    torch.cuda.synchronize()
    recs = rs.profile_collect()
    rs.profile_enable(False)
    per = {}
    order = []
    for name, ms, _ in recs:
        if name not in per:
            per[name] = [0.0, 0]
            order.append(name)
        per[name][0] += ms
        per[name][1] += 1
    return {"wall_us": round(wall * 1e6, 2),
            "kernels": [{"name": k, "per_call": per[k][1] / iters, "avg_us": round(1e3 * per[k][0] / per[k][1], 2)}
                        for k in order]}


def main():
    iters = 50
    args = [a for a in sys.argv[1:]]
    if "--iters" in args:
        i = args.index("--iters")
        iters = int(args[i + 1])
        del args[i:i + 2]
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    for shape in args:
        p = [int(x) for x in shape.split(":")]
        N, M = p[0], p[1]
        S = p[2] if len(p) > 2 else 1024
        d_o = torch.randint(0, 256, (N, S), dtype=torch.uint8, device=dev)
        d_r = torch.empty((M, S), dtype=torch.uint8, device=dev)
        d_x = torch.empty((N, S), dtype=torch.uint8, device=dev)
        enc = rs.encode_device_call(N, M, S, d_o, d_r, stream=stream)
        out = {"shape": f"{N}:{M}x{S}", "encode": profile(enc, iters)}
        for pct in (1, 100):
            L = -(-min(N, M) * pct // 100)
            op = rs.present_mask([1] * (N - L) + [0] * L)
            rp = rs.present_mask([1] * L + [0] * (M - L))
            dec = rs.decode_device_call(N, M, S, d_o, op, d_r, rp, d_x, stream=stream)
            out[f"decode_{pct}pct"] = profile(dec, iters)
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
