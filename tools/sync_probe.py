#!/usr/bin/env python3
"""Where does the fixed per-batch overhead of bench.py's timed region go?

Times K back-to-back headline encodes (1024:1024 x 1 KiB) several ways and
prints one JSON line per variant: wall / K, GPU-event time / K.
  base      : bench.py's timed() as of r01 (stream context + events inside)
  plain     : no `with torch.cuda.stream` (the call is bound to its stream anyway)
  streamsync: stream.synchronize() before torch.cuda.synchronize()
  noevents  : no events in the timed region
Run with SPIN=1 to set hipDeviceScheduleSpin before the device is initialised.
"""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))

if os.environ.get("SPIN") == "1":
    hip = ctypes.CDLL("libamdhip64.so")
    print("hipSetDeviceFlags(spin) ->", hip.hipSetDeviceFlags(ctypes.c_uint(1)), file=sys.stderr)

import torch  # noqa: E402

import reed_solomon_simd as rs  # noqa: E402


def main():
    K = int(os.environ.get("K", "20"))
    reps = int(os.environ.get("REPS", "5"))
    N = M = S = 1024
    dev = torch.device("cuda", 0)
    ctx = rs.Context(0)
    d_o = torch.randint(0, 256, (N, S), dtype=torch.uint8, device=dev)
    d_r = torch.empty((M, S), dtype=torch.uint8, device=dev)
    st = torch.cuda.Stream(device=dev)
    enc = rs.encode_device_call(N, M, S, d_o, d_r, stream=st, ctx=ctx)
    for _ in range(50):
        enc()
    torch.cuda.synchronize()

    def run(variant):
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if variant == "base":
            t0 = time.perf_counter()
            with torch.cuda.stream(st):
                e0.record(st)
                for _ in range(K):
                    enc()
                e1.record(st)
            torch.cuda.synchronize()
            w = time.perf_counter() - t0
        elif variant == "plain":
            t0 = time.perf_counter()
            e0.record(st)
            for _ in range(K):
                enc()
            e1.record(st)
            torch.cuda.synchronize()
            w = time.perf_counter() - t0
        elif variant == "streamsync":
            t0 = time.perf_counter()
            e0.record(st)
            for _ in range(K):
                enc()
            e1.record(st)
            st.synchronize()
            torch.cuda.synchronize()
            w = time.perf_counter() - t0
        else:  # noevents
            t0 = time.perf_counter()
            for _ in range(K):
                enc()
            torch.cuda.synchronize()
            w = time.perf_counter() - t0
            e0.record(st)
            e1.record(st)
            torch.cuda.synchronize()
            return w, None
        return w, e0.elapsed_time(e1) / 1e3

    for v in ("base", "plain", "streamsync", "noevents"):
        ws, gs = [], []
        for _ in range(reps):
            w, g = run(v)
            ws.append(w)
            if g is not None:
                gs.append(g)
        print(json.dumps({"variant": v, "spin": os.environ.get("SPIN") == "1", "K": K,
                          "wall_us_per_step": [round(x / K * 1e6, 2) for x in ws],
                          "gpu_us_per_step": [round(x / K * 1e6, 2) for x in gs]}))
    # host cost of one call (no GPU wait): enqueue 200 and time the loop only
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(200):
        enc()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(json.dumps({"host_enqueue_us_per_call": round((t1 - t0) / 200 * 1e6, 2)}))


if __name__ == "__main__":
    main()
