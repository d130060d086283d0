"""A/B of the one-row-per-lane encode kernel (rs_lane.hip) against the column
kernel (rs_mono.hip) on single-chunk 2-element encodes: per shape, alternating
rounds of `steps` back-to-back rs_encode_device calls on one stream, GPU time
from events around each round (mode bits: rs_mono_enable 1 | 32 / 1 | 64).
Also checks both outputs are identical.  Usage: python tools/lane_ab.py [rounds] [steps]"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))
import torch  # noqa: E402
import reed_solomon_simd as rs  # noqa: E402

SHAPES = [(1024, 1024, 1024), (512, 512, 1024), (256, 256, 1024), (1024, 1024, 512), (1024, 1024, 256),
          (700, 513, 1024), (256, 256, 512)]


def main():
    rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    dev = torch.device("cuda", 0)
    stream = torch.cuda.Stream(device=dev)
    out = []
    for N, M, S in SHAPES:
        g = torch.Generator(device=dev)
        g.manual_seed(N + M + S)
        d_o = torch.randint(0, 256, (N, S), dtype=torch.uint8, device=dev, generator=g)
        res = {}
        outs = {}
        for mode in (32, 64):
            d_r = torch.empty((M, S), dtype=torch.uint8, device=dev)
            rs.mono_enable(1 | mode)
            rs.encode_device_call(N, M, S, d_o, d_r, stream=stream)()
            torch.cuda.synchronize()
            outs[mode] = d_r.clone()
        same = bool(torch.equal(outs[32], outs[64]))
        times = {32: [], 64: []}
        for r in range(rounds):
            for mode in (32, 64):
                rs.mono_enable(1 | mode)
                d_r = outs[mode]
                call = rs.encode_device_call(N, M, S, d_o, d_r, stream=stream)
                call()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(stream)
                for _ in range(steps):
                    call()
                e1.record(stream)
                torch.cuda.synchronize()
                times[mode].append(e0.elapsed_time(e1) * 1e3 / steps)
        rs.mono_enable(1)
        res = {"shape": f"{N}:{M}x{S}", "identical": same,
               "lane_us": sorted(round(t, 2) for t in times[32]), "mono_us": sorted(round(t, 2) for t in times[64])}
        res["lane_median"] = res["lane_us"][len(times[32]) // 2]
        res["mono_median"] = res["mono_us"][len(times[64]) // 2]
        print(json.dumps(res), flush=True)
        out.append(res)


if __name__ == "__main__":
    main()
