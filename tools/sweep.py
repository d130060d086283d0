#!/usr/bin/env python3
"""Path sweep (development tool): time device-resident encode / decode for a
list of (N, M, S) under each kernel path (column kernel off / default / all)
to choose the routing thresholds in rs_codec.cpp.

    python3 tools/sweep.py [--iters 100] [--decode]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))

CONFIGS = [
    (128, 128, 1024), (512, 512, 1024), (1024, 1024, 1024), (1024, 1024, 4096), (1024, 1024, 16384),
    (1024, 1024, 65536), (1024, 1024, 2048), (512, 512, 2048), (2048, 2048, 1024), (4096, 4096, 1024), (3000, 1024, 1024), (256, 256, 65536),
    (32768, 32768, 1024), (8192, 8192, 65536),
]
PATHS = {"pass": 0, "mono1": 1, "mono2": 2}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--decode", action="store_true")
    args = ap.parse_args()
    import torch
    import reed_solomon_simd as rs

    s = torch.cuda.Stream()
    for N, M, S in CONFIGS:
        d_orig = torch.randint(0, 256, (N, S), dtype=torch.uint8, device="cuda")
        d_rec = torch.empty((M, S), dtype=torch.uint8, device="cuda")
        d_out = torch.empty((N, S), dtype=torch.uint8, device="cuda")
        row = {"N": N, "M": M, "S": S}
        iters = max(3, min(args.iters, int(2e9 // ((N + M) * S))))
        for name, mono in PATHS.items():
            rs.mono_enable(mono)

            def enc():
                rs.encode_device(N, M, S, d_orig, d_rec, stream=s)

            fns = {"enc": enc}
            if args.decode:
                L = min(N, M)
                op = rs.present_mask([1] * (N - L) + [0] * L)
                rp = rs.present_mask([1] * L + [0] * (M - L))

                def dec():
                    rs.decode_device(N, M, S, d_orig, op, d_rec, rp, d_out, stream=s)

                fns["dec100"] = dec
            for k, fn in fns.items():
                with torch.cuda.stream(s):
                    for _ in range(3):
                        fn()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                with torch.cuda.stream(s):
                    for _ in range(iters):
                        fn()
                torch.cuda.synchronize()
                dt = (time.perf_counter() - t0) / iters
                row[f"{name}_{k}_us"] = round(dt * 1e6, 2)
                row[f"{name}_{k}_GiBps"] = round((N + M) * S / dt / 2**30, 1)
        rs.mono_enable(1)
        print(json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
