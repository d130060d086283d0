#!/usr/bin/env python3
"""bench.py -- device-resident Reed-Solomon GF(2^16) encode/decode on MI355X.

Metric (BASELINE.json): GiB/s of (original + recovery) bytes, device-resident,
at 1024:1024 x 1024 B shards (BASELINE.json configs[1]).  A "step" is one
encode of one 1024:1024 x 1 KiB stripe whose shards already sit in HBM
(rs_encode_device through the C ABI).  Decode at 1 % and 100 % loss
(loss pattern of the reference's benches/benchmarks.rs:113-138) is timed the
same way and reported beside the headline value.

N > 1 (torchrun, one process per GPU): every rank encodes its own stripes
(independent objects, no data-path collective) -> "scaling": "weak"; value =
bytes of all ranks / max-over-ranks time.

roofline: per-kernel HIP-event timing of the launches of the timed workload
(rs_profile_enable), dominant kernel = largest total time; achieved = its
algorithmic bytes per launch / its average duration; peak = 8 TB/s HBM3E.
cpu_baseline: the reference's AVX2 algorithm restated in C (oracle/avx2_port.c),
single thread, on a bounded sample, rank 0 at N = 1 only.
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

METRIC = "GiB/s (original+recovery) encode & decode, device-resident, 1024:1024×1024B"
HBM_PEAK_GBS = 8000.0

CONFIGS = {
    # name: (original_count, recovery_count, shard_bytes)
    "1024x1024x1k": (1024, 1024, 1024),        # configs[1] (the metric's config)
    "32768x32768x1k": (32768, 32768, 1024),    # configs[2]
    "8192x8192x64k": (8192, 8192, 65536),      # configs[3] (decode)
    "32768x32768x64k": (32768, 32768, 65536),  # configs[4] (column-partitioned over the ranks)
}
SHARDED = "32768x32768x64k"


def reduce_max(x, world, device):
    """Max of a per-rank scalar over all ranks (the timing contract: max over ranks)."""
    if world == 1:
        return x
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--config", default="1024x1024x1k", choices=sorted(CONFIGS))
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-copy", action="store_true", help="skip the 1 GiB device-copy context measurement")
    p.add_argument("--no-decode", action="store_true")
    p.add_argument("--no-host", action="store_true", help="skip the host-memory end-to-end measurement")
    p.add_argument("--profile-steps", type=int, default=50)
    p.add_argument("--batch", type=int, default=64, help="stripes per call of the batched measurement (1 = skip)")
    return p.parse_args()


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    import reed_solomon_simd as rs

    ctx = rs.Context(local)
    N, M, S = CONFIGS[args.config]
    dev = torch.device("cuda", local)
    if args.config == SHARDED:
        sharded_bench(args, rs, ctx, world, rank, dev)
        if world > 1:
            dist.destroy_process_group()
        return
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    d_orig = torch.randint(0, 256, (N, S), dtype=torch.uint8, device=dev, generator=g)
    d_rec = torch.empty((M, S), dtype=torch.uint8, device=dev)
    d_out = torch.empty((N, S), dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(device=dev)

    def barrier():
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        return reduce_max(x, world, dev)

    def timed(fn, steps, warmup):
        with torch.cuda.stream(stream):
            for _ in range(warmup):
                fn()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            ev0.record(stream)
            for _ in range(steps):
                fn()
            ev1.record(stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        barrier()
        return max_over_ranks(wall), max_over_ranks(ev0.elapsed_time(ev1) / 1e3)

    # one C-ABI call per step (rs_encode_device_strided), arguments bound once:
    # the Python keyword wrapper would add ≈3 µs of host time to an 8 µs step
    enc = rs.encode_device_call(N, M, S, d_orig, d_rec, stream=stream, ctx=ctx)

    # ---- headline: encode -------------------------------------------------
    wall, gpu_t = timed(enc, args.steps, args.warmup)
    step_bytes = (N + M) * S
    value = step_bytes * args.steps * world / wall / 2**30

    # ---- per-kernel timing of the same workload ----------------------------
    rs.profile_enable(True, ctx=ctx)
    with torch.cuda.stream(stream):
        for _ in range(args.profile_steps):
            enc()
    torch.cuda.synchronize()
    recs = rs.profile_collect(ctx)
    rs.profile_enable(False, ctx=ctx)
    agg = {}
    for name, ms, by in recs:
        a = agg.setdefault(name, [0.0, 0, 0])
        a[0] += ms
        a[1] += 1
        a[2] += by
    kernels = {k: {"launches_per_step": v[1] / args.profile_steps, "avg_us": round(1e3 * v[0] / v[1], 3),
                   "rows_bytes_per_launch": v[2] // v[1]} for k, v in agg.items()}
    dom = max(agg, key=lambda k: agg[k][0])
    dom_avg_s = agg[dom][0] / agg[dom][1] / 1e3
    # Algorithmic bytes: an encode must read N*S original
    # bytes and write M*S recovery bytes.  When one launch does the whole
    # encode (the headline's column kernel) that is its per-launch figure;
    # otherwise the step's algorithmic bytes are priced against the summed
    # duration of all the step's launches.
    alg_step = (N + M) * S
    kernel_s_per_step = sum(v[0] for v in agg.values()) / 1e3 / args.profile_steps
    if len(agg) == 1 and kernels[dom]["launches_per_step"] == 1:
        # one launch per step: its duration is the step's GPU time measured
        # around the whole timed batch on the launch stream (gpu_t); events
        # bracketing every single launch add their own gaps (kernels[...].avg_us)
        dom_avg_s = gpu_t / args.steps
        scope, achieved = "launch", alg_step / dom_avg_s / 1e9
    else:
        scope, achieved = "step (all launches)", alg_step / kernel_s_per_step / 1e9
    traffic = load_traffic(dom)
    roofline = {"bound": "hbm", "kernel": dom, "scope": scope, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic["hbm_bytes"] if traffic else None,
                "traffic_source": traffic["source"] if traffic else None,
                "algorithmic_bytes": alg_step,
                "avg_us": round(dom_avg_s * 1e6, 3), "kernels": kernels,
                "note": "avg_us: the timed batch's launch-stream event time / steps when one launch is the "
                        "whole step (rocprofv3 kernel-trace average agrees, profiles/); kernels[].avg_us "
                        "brackets every launch with its own events, which adds their overhead"}

    # ---- decode at 1 % and 100 % loss (benchmarks.rs:113-138) --------------
    decode = {}
    if not args.no_decode:
        for pct in (1, 100):
            L = -(-min(N, M) * pct // 100)
            op = rs.present_mask([1] * (N - L) + [0] * L)
            rp = rs.present_mask([1] * L + [0] * (M - L))

            dec = rs.decode_device_call(N, M, S, d_orig, op, d_rec, rp, d_out, stream=stream, ctx=ctx)

            w, gt = timed(dec, args.steps, args.warmup)
            decode[f"{pct}pct"] = round(step_bytes * args.steps * world / w / 2**30, 3)
            decode[f"{pct}pct_us_per_step"] = {"wall": round(w / args.steps * 1e6, 2),
                                               "gpu_events": round(gt / args.steps * 1e6, 2)}

    # ---- a batch of stripes of the same shape per launch (MI355X extension:
    # rs_encode_device_batch / rs_decode_device_batch; one erasure pattern) ----
    batched = None
    if args.batch > 1 and N * S * args.batch <= (1 << 31):
        B = args.batch
        b_orig = torch.randint(0, 256, (B, N, S), dtype=torch.uint8, device=dev, generator=g)
        b_rec = torch.empty((B, M, S), dtype=torch.uint8, device=dev)
        b_out = torch.empty((B, N, S), dtype=torch.uint8, device=dev)
        bsteps = max(5, args.steps // 10)
        w_e, g_e = timed(lambda: rs.encode_device_batch(N, M, S, b_orig, b_rec, stream=stream, ctx=ctx), bsteps,
                         max(2, args.warmup // 5))
        L1 = -(-min(N, M) // 100)
        op1 = rs.present_mask([1] * (N - L1) + [0] * L1)
        rp1 = rs.present_mask([1] * L1 + [0] * (M - L1))
        w_d, _ = timed(lambda: rs.decode_device_batch(N, M, S, b_orig, op1, b_rec, rp1, b_out, stream=stream,
                                                      ctx=ctx), bsteps, max(2, args.warmup // 5))
        bbytes = step_bytes * B * world * bsteps
        batched = {"stripes": B, "encode_GiBps": round(bbytes / w_e / 2**30, 3),
                   "encode_us_per_launch": round(g_e / bsteps * 1e6, 2),
                   "encode_hbm_frac": round(step_bytes * B / (g_e / bsteps) / 1e9 / HBM_PEAK_GBS, 4),
                   "decode_1pct_GiBps": round(bbytes / w_d / 2**30, 3),
                   "note": "B stripes of the workload's shape per call (one column-kernel launch); not the headline"}
        del b_orig, b_rec, b_out

    # ---- host-memory end to end (pinned buffers, PCIe both ways) -------------
    host_e2e = None
    if not args.no_host:
        h_o = d_orig.cpu().pin_memory()
        h_r = torch.empty((M, S), dtype=torch.uint8).pin_memory()
        best = None
        for sl in (1, 2, 4, 8):
            rs.encode_host(N, M, S, h_o, h_r, slices=sl, ctx=ctx)
            it = max(5, args.steps // 10)
            t0 = time.perf_counter()
            for _ in range(it):
                rs.encode_host(N, M, S, h_o, h_r, slices=sl, ctx=ctx)
            dt = (time.perf_counter() - t0) / it
            if best is None or dt < best[1]:
                best = (sl, dt)
        L = -(-min(N, M) // 100)
        op = rs.present_mask([1] * (N - L) + [0] * L)
        rp = rs.present_mask([1] * L + [0] * (M - L))
        h_x = torch.empty((N, S), dtype=torch.uint8).pin_memory()
        h_rc = d_rec.cpu().pin_memory()
        rs.decode_host(N, M, S, h_o, op, h_rc, rp, h_x, slices=best[0], ctx=ctx)
        it = max(5, args.steps // 10)
        t0 = time.perf_counter()
        for _ in range(it):
            rs.decode_host(N, M, S, h_o, op, h_rc, rp, h_x, slices=best[0], ctx=ctx)
        ddt = (time.perf_counter() - t0) / it
        host_e2e = {"encode_GiBps": round(world * step_bytes / best[1] / 2**30, 3),
                    "decode_1pct_GiBps": round(world * step_bytes / ddt / 2**30, 3), "slices": best[0],
                    "note": "pinned host buffers, hipMemcpy2DAsync in + kernels + out, column slices over 3 streams"}

    # ---- device copy for context (STREAM-copy GB/s) ---------
    copy_ref = None
    if not args.no_copy:
        nb = 1 << 30
        c_src = torch.empty(nb, dtype=torch.uint8, device=dev)
        c_dst = torch.empty_like(c_src)
        c_dst.copy_(c_src)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            c_dst.copy_(c_src)
        e1.record()
        torch.cuda.synchronize()
        copy_ref = {"GBps": round(2 * nb * 10 / (e0.elapsed_time(e1) / 1e3) / 1e9, 1),
                    "note": "torch device-to-device copy of 1 GiB (read + write bytes), context for roofline.peak"}
        del c_src, c_dst

    # ---- CPU baseline (rank 0, N = 1 only) ----------------------------------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 5), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u8", "data": "synthetic (uniform random bytes)",
            "config": {"workload": f"encode {N}:{M} x {S} B, device-resident (rs_encode_device)",
                       "original_count": N, "recovery_count": M, "shard_bytes": S,
                       "rate": "high" if rs.use_high_rate(N, M) == 1 else "low",
                       "parallelism": f"replicas x{world} (independent stripes)"},
            "gpu_event_ms_per_step": round(gpu_t / args.steps * 1e3, 5),
            "decode_GiBps": decode,
            "batched": batched,
            "host_e2e": host_e2e,
            "roofline": roofline,
            "device_copy": copy_ref,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line))
    if world > 1:
        dist.destroy_process_group()


def sharded_bench(args, rs, ctx, world, rank, dev):
    """configs[4]: ONE 32768:32768 x 64 KiB stripe column-partitioned over the ranks
    (DESIGN.md "Multi-GPU"): rank r encodes byte columns
    [r*w, (r+1)*w), w = 64 KiB / world, of its resident slice of the originals, and an
    all-gather (RCCL over xGMI) assembles the whole [M x S] recovery matrix on every rank
    (reed_solomon_simd.encode_device_sharded).  Total work is fixed: strong scaling.
    Reported: the whole step (encode + all-gather + re-interleave) and encode alone."""
    import torch
    import torch.distributed as dist

    N, M, S = CONFIGS[args.config]
    w = S // world
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    d_orig = torch.randint(0, 256, (N, w), dtype=torch.uint8, device=dev, generator=g)  # this rank's columns
    d_rec = torch.empty((M, S), dtype=torch.uint8, device=dev)
    part = torch.empty((M, w), dtype=torch.uint8, device=dev) if world > 1 else d_rec
    gathered = torch.empty((world, M, w), dtype=torch.uint8, device=dev) if world > 1 else None
    cur = torch.cuda.current_stream(dev)  # collectives are ordered after this stream's kernels

    def compute():
        rs.encode_device(N, M, w, d_orig, part, stream=cur, ctx=ctx)

    def step():
        compute()
        if world > 1:
            dist.all_gather_into_tensor(gathered, part)
            d_rec.view(M, world, w).copy_(gathered.permute(1, 0, 2))

    def timed(fn):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        t = time.perf_counter() - t0
        if world > 1:
            dist.barrier()
        return reduce_max(t, world, dev) / args.steps

    t_step = timed(step)
    t_comp = timed(compute)
    total = (N + M) * S
    if rank == 0:
        per_gpu = (N + M) * w
        achieved = per_gpu / t_comp / 1e9
        print(json.dumps({
            "metric": "GiB/s (original+recovery) encode, device-resident, 32768:32768x65536B column-partitioned "
                      "+ RCCL all-gather",
            "value": round(total / t_step / 2**30, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(t_step * 1e3, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u8", "data": "synthetic (uniform random bytes)",
            "config": {"workload": "encode 32768:32768 x 64 KiB (configs[4]), column slice of 64 KiB / n per GPU",
                       "original_count": N, "recovery_count": M, "shard_bytes": S, "slice_bytes": w,
                       "parallelism": f"column partition x{world} + all_gather_into_tensor"},
            "encode_only": {"ms_per_step": round(t_comp * 1e3, 4),
                            "GiBps": round(total / t_comp / 2**30, 3)},
            "allgather_and_interleave_ms": round((t_step - t_comp) * 1e3, 4),
            "roofline": {"bound": "hbm", "kernel": "encode passes (all launches of one slice)",
                         "scope": "step (all launches)", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": None,
                         "algorithmic_bytes": per_gpu},
            "cpu_baseline": None,
        }))


def load_traffic(kernel):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/<tag>/traffic.json, written by tools/pmc_traffic.py from
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over this same bench)."""
    pdir = os.path.join(ROOT, "profiles")
    if not os.path.isdir(pdir):
        return None
    for tag in sorted(os.listdir(pdir), reverse=True):
        f = os.path.join(pdir, tag, "traffic.json")
        if os.path.exists(f):
            with open(f) as fh:
                d = json.load(fh)
            if kernel in d["kernels"]:
                return {"hbm_bytes": d["kernels"][kernel]["hbm_bytes"], "source": f"profiles/{tag}/traffic.json"}
    return None


def cpu_baseline(seconds):
    """AVX2 restatement of the reference engine (oracle/avx2_port.c), 1024:1024 x 1 KiB encode:
    `value` on 1 thread (the reference is single-threaded); `all_cores` = independent stripes on
    every host thread this process may use (at most 16, the GPU box's CPU share), an upper bound."""
    import threading

    import numpy as np
    import oracle_lib as O

    if O.lib().orc_select_engine(1) != 0:
        return {"value": None, "unit": "GiB/s", "cores": 1, "kind": "port", "sample": "AVX2 unavailable on host"}
    orig = np.random.default_rng(0).integers(0, 256, (1024, 1024), dtype=np.uint8)
    O.encode("default", orig, 1024)  # tables built once, before any thread starts
    it, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        O.encode("default", orig, 1024)
        it += 1
    dt = time.perf_counter() - t0

    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    counts = [0] * threads
    stop = time.perf_counter() + max(1.0, seconds / 2)

    def worker(i):  # ctypes releases the GIL; the oracle's work buffer is thread-local
        mine = orig.copy()
        while time.perf_counter() < stop:
            O.encode("default", mine, 1024)
            counts[i] += 1

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    t1 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt_all = time.perf_counter() - t1
    O.lib().orc_select_engine(0)
    cpu = f"{platform.processor() or platform.machine()}"
    return {"value": round(2 * 1024 * 1024 * it / dt / 2**30, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{it} encodes of 1024:1024 x 1024 B in {dt:.1f} s (shard copy-in + encode, like "
                      f"benches/benchmarks.rs:101-107), single thread, {cpu}",
            "all_cores": {"value": round(2 * 1024 * 1024 * sum(counts) / dt_all / 2**30, 4), "cores": threads,
                          "sample": f"{sum(counts)} independent encodes on {threads} threads in {dt_all:.1f} s"}}


if __name__ == "__main__":
    main()
