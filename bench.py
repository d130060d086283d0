#!/usr/bin/env python3
"""bench.py -- device-resident Reed-Solomon GF(2^16) encode/decode on MI355X.

Metric (BASELINE.json): GiB/s of (original + recovery) bytes, device-resident,
at 1024:1024 x 1024 B shards (BASELINE.json configs[1]).  A "step" is one
encode of one 1024:1024 x 1 KiB stripe whose shards already sit in HBM
(rs_encode_device through the C ABI).  Decode at 1 % and 100 % loss
(loss pattern of the reference's benches/benchmarks.rs:113-138) is timed the
same way and reported beside the headline value.

--gpus N > 1: the parent process (which never touches the GPU) starts N ranks
with torch.distributed.run, one process per GPU (RCCL = the "nccl" backend).
Every N reports the SAME primary workload: the headline stripe on every rank
(independent stripes, no data-path collective; value = all ranks' bytes / the
max-over-ranks time -> "scaling": "weak"), so the driver's 1/2/4/8 lines form one
curve.  Beside it, the "sharded" sub-object carries north_star's multi-GPU
configuration, configs[4], at the same N: ONE 32768:32768 x 64 KiB stripe
column-partitioned over the ranks (rank r encodes byte columns [r*S/N, (r+1)*S/N)
of every shard), an RCCL all-gather of the recovery slices over xGMI and a
re-interleave -- total work fixed, strong scaling -- with its encode-only time,
the all-gather cost, the per-GPU HBM fraction and a column-partitioned 1 % decode;
its N = 1 point is in the --gpus 1 line.  --config 32768x32768x64k makes that
workload the primary line instead (strong scaling).  The other single-GPU
BASELINE configs ride in the same line: "config3" = configs[2] (32768:32768 x
1 KiB encode, plus its 1 % / 100 % decode) and "config4" = configs[3]
(8192:8192 x 64 KiB decode at 1 % / 100 %), each with the roofline of its
dominant kernel (replicas per rank at N > 1; --no-configs skips them).

Timing: W untimed warmup steps, then exactly K steps bracketed by a barrier +
torch.cuda.synchronize() on both sides, max over ranks.  Nothing else runs in
the timed region (HIP events of the kernels are taken in a separate pass).

roofline: per-launch HIP events on the launch stream (rs_profile_enable) over
the same workload; dominant kernel = largest total time; achieved = the
SURVEY.md 8(d) algorithmic bytes / duration; peak = 8 TB/s HBM3E; traffic =
HBM bytes per launch of that kernel from the committed rocprofv3 PMC passes
(profiles/<tag>/traffic.json); valu_frac = VALU wave-instructions per launch
(SQ_INSTS_VALU, same summary) x 2 cycles / (duration x 1024 SIMDs x 2.4 GHz).
cpu_baseline: the reference's AVX2 algorithm restated in C (oracle/avx2_port.c)
on a bounded sample of the same workload, rank 0.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

METRIC = "GiB/s (original+recovery) encode & decode, device-resident, 1024:1024×1024B"
HBM_PEAK_GBS = 8000.0
SIMDS, CLOCK_HZ, VALU_CYCLES = 1024, 2.4e9, 2  # MI355X: 256 CUs x 4 SIMDs; a wave64 VALU op issues over 2 cycles
# measured issue cost of the GF multiply mixes (gf_muladd2 / gf_muladd4: all VOP3 but a few
# ANDs) at 4 waves per SIMD, in 2.4 GHz clocks per wave64 instruction per SIMD
# (tools/valu_rate.hip, profiles/r05j/valu_rate.txt: VOP3 4.3, VOP2 2.6, the mixes 4.0)
VALU_MIX_CYCLES = 4.0

CONFIGS = {
    # name: (original_count, recovery_count, shard_bytes)
    "1024x1024x1k": (1024, 1024, 1024),        # configs[1] (the metric's config)
    "32768x32768x1k": (32768, 32768, 1024),    # configs[2]
    "8192x8192x64k": (8192, 8192, 65536),      # configs[3] (decode)
    "32768x32768x64k": (32768, 32768, 65536),  # configs[4] (column-partitioned over the ranks)
}
HEADLINE = "1024x1024x1k"
SHARDED = "32768x32768x64k"


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=200)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--config", default=None, choices=sorted(CONFIGS),
                   help=f"default: {HEADLINE} (independent stripes per rank) at every N")
    p.add_argument("--cpu-seconds", type=float, default=10.0)
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-copy", action="store_true", help="skip the 1 GiB device-copy context measurement")
    p.add_argument("--no-decode", action="store_true")
    p.add_argument("--no-host", action="store_true", help="skip the host-memory end-to-end measurement")
    p.add_argument("--no-object", action="store_true", help="skip the object-API (encoder/decoder) measurement")
    p.add_argument("--no-sharded", action="store_true",
                   help="skip the configs[4] strong-scaling sub-object (column partition + all-gather)")
    p.add_argument("--no-configs", action="store_true",
                   help="skip the configs[2] / configs[3] sub-objects of the headline line")
    p.add_argument("--profile-steps", type=int, default=50)
    p.add_argument("--batch", type=int, default=64, help="stripes per call of the batched measurement (1 = skip)")
    p.add_argument("--plumbing", action="store_true",
                   help="CPU/gloo check of the rank launcher and timing reduction (no GPU, no kernels)")
    p.add_argument("--shape-table", action="store_true",
                   help="time the reference README's shape table (README.md:27-45, 1 KiB shards): device "
                        "encode and 1 %% / 100 %% decode, the route each takes, and the AVX2 port on one core")
    return p.parse_args()


# ---------------------------------------------------------------------------
# rank launcher: the parent never initialises the GPU

def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def reduce_max(x, world, device):
    """Max of a per-rank scalar over all ranks (the timing contract: max over ranks)."""
    if world == 1:
        return x
    import torch
    import torch.distributed as dist

    t = torch.tensor([x], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def plumbing(args, world, rank):
    """--plumbing: the multi-rank skeleton of the bench on gloo (CPU tests)."""
    import torch
    import torch.distributed as dist

    for _ in range(args.warmup):
        pass
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        time.sleep(0.001)
    wall = reduce_max(time.perf_counter() - t0, world, "cpu")
    ranks = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
    if world > 1:
        dist.all_gather(ranks, torch.tensor([rank], dtype=torch.int64))
    if rank == 0:
        print(json.dumps({"metric": "plumbing", "value": round(args.steps / wall, 3), "unit": "steps/s",
                          "n_gpus": world if world > 1 else 1, "steps": args.steps, "warmup": args.warmup,
                          "ranks_seen": [int(r.item()) for r in ranks] if world > 1 else [0]}))


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args))
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.plumbing:
        if world > 1:
            dist.init_process_group("gloo")
        plumbing(args, world, rank)
        if world > 1:
            dist.destroy_process_group()
        return
    if os.environ.get("RS_BENCH_REHEARSE") == "1":
        # rehearsal of the N-rank path on a one-GPU box: every rank on cuda:0, collectives on
        # gloo (numbers meaningless; the driver's N-GPU runs use RCCL, one GPU per rank)
        local = 0
    if world > 1:
        if os.environ.get("RS_BENCH_REHEARSE") == "1":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        world = dist.get_world_size()
    torch.cuda.set_device(local)
    import reed_solomon_simd as rs

    ctx = rs.Context(local)
    if args.shape_table:
        shape_table(args, rs, ctx, torch.device("cuda", local))
        return
    config = args.config or HEADLINE
    dev = torch.device("cuda", local)
    if config == SHARDED:
        sharded_bench(args, rs, ctx, world, rank, dev)
    else:
        stripe_bench(args, rs, ctx, config, world, rank, dev)
    if os.environ.get("RS_BENCH_REHEARSE") == "1":
        # the rehearsal's memory record (stderr): this rank's peak of torch allocations, and
        # the device's memory in use (all ranks share the one GPU, the library's own
        # buffers included) as each rank finishes
        free, total = torch.cuda.mem_get_info(dev)
        print(json.dumps({"rank": rank, "world": world,
                          "torch_max_allocated_GiB": round(torch.cuda.max_memory_allocated(dev) / 2**30, 3),
                          "device_used_GiB_all_ranks": round((total - free) / 2**30, 3)}), file=sys.stderr, flush=True)
    if world > 1:
        dist.destroy_process_group()


# ---------------------------------------------------------------------------
# timing helpers

def make_timer(world, dev):
    import torch
    import torch.distributed as dist

    def barrier():
        if world > 1:
            dist.barrier()

    def timed(fn, steps, warmup):
        """Wall time of exactly `steps` calls of fn, bracketed by barrier + synchronize; max over ranks."""
        for _ in range(warmup):
            fn()
        torch.cuda.synchronize()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fn()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        barrier()
        return reduce_max(wall, world, dev)

    def gpu_time(fn, steps, stream):
        """GPU time of `steps` calls from events on the launch stream (separate, untimed pass)."""
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        # one untimed call first: ev0 then completes behind work already on the GPU, not
        # ahead of the host's first launch into an idle queue (that gap read as ≈+1 µs per
        # step at 20 steps and made this launch-scope duration exceed the wall time per step)
        fn()
        ev0.record(stream)
        for _ in range(steps):
            fn()
        ev1.record(stream)
        torch.cuda.synchronize()
        return reduce_max(ev0.elapsed_time(ev1) / 1e3, world, dev)

    return timed, gpu_time


def load_pmc(kernel, config):
    """Per-launch PMC figures of `kernel` in the bench of `config` from the newest committed
    summary that has them (profiles/<tag>/traffic.json, written by tools/pmc_traffic.py from
    rocprofv3 --pmc passes over this bench): HBM bytes (FETCH_SIZE x2 + WRITE_SIZE) and
    SQ_INSTS_VALU."""
    pdir = os.path.join(ROOT, "profiles")
    out = {}
    if not os.path.isdir(pdir):
        return out
    for tag in sorted(os.listdir(pdir), reverse=True):
        f = os.path.join(pdir, tag, "traffic.json")
        if not os.path.exists(f):
            continue
        with open(f) as fh:
            d = json.load(fh)
        k = d["configs"].get(config, {}).get(kernel) if "configs" in d else (
            d["kernels"].get(kernel) if config == HEADLINE else None)
        if not k:
            continue
        if "traffic" not in out and "hbm_bytes" in k:
            out["traffic"] = (k["hbm_bytes"], f"profiles/{tag}/traffic.json")
        if "valu" not in out and "valu_insts" in k:
            out["valu"] = (k["valu_insts"], f"profiles/{tag}/traffic.json")
        if len(out) == 2:
            break
    return out


def roofline_of(rs, ctx, fn, profile_steps, alg_step_bytes, config, launch_scope_s=None):
    """Per-kernel HIP-event timing of `profile_steps` calls of fn (rs_profile_enable) and the
    roofline block of the dominant kernel."""
    import torch

    rs.profile_enable(True, ctx=ctx)
    for _ in range(profile_steps):
        fn()
    torch.cuda.synchronize()
    recs = rs.profile_collect(ctx)
    rs.profile_enable(False, ctx=ctx)
    agg = {}
    for name, ms, by in recs:
        a = agg.setdefault(name, [0.0, 0, 0])
        a[0] += ms
        a[1] += 1
        a[2] += by
    # per-launch event figures: each launch bracketed by its own pair of events, which adds
    # the events' own gaps (≈2.6 µs on the 8 µs headline launch) -- NOT the roofline's avg_us
    kernels = {k: {"launches_per_step": v[1] / profile_steps, "event_bracketed_us": round(1e3 * v[0] / v[1], 3),
                   "alg_bytes_per_launch": v[2] // v[1]} for k, v in agg.items()}
    dom = max(agg, key=lambda k: agg[k][0])
    kernel_s_per_step = sum(v[0] for v in agg.values()) / 1e3 / profile_steps
    if len(agg) == 1 and kernels[dom]["launches_per_step"] == 1 and launch_scope_s:
        # one launch per step: its duration is the step's GPU time measured around a whole
        # batch on the launch stream; events bracketing every single launch add their own gaps
        dom_avg_s = launch_scope_s
        scope, achieved = "launch", alg_step_bytes / dom_avg_s / 1e9
    else:
        dom_avg_s = agg[dom][0] / agg[dom][1] / 1e3
        scope, achieved = "step (all launches)", alg_step_bytes / kernel_s_per_step / 1e9
    pmc = load_pmc(dom, config)
    valu = None
    if "valu" in pmc:
        insts = pmc["valu"][0]
        valu = {"valu_insts_per_launch": insts, "frac": round(insts * VALU_CYCLES / (dom_avg_s * CLOCK_HZ * SIMDS), 4),
                "issue_frac": round(insts * VALU_MIX_CYCLES / (dom_avg_s * CLOCK_HZ * SIMDS), 4),
                "source": pmc["valu"][1],
                "note": "frac: SQ_INSTS_VALU x 2 cycles per wave-instruction / (launch duration x 1024 SIMDs x "
                        "2.4 GHz); issue_frac: x the measured 4.0 cycles of the GF multiply mix instead "
                        "(tools/valu_rate.hip)"}
    return {"bound": "hbm", "kernel": dom, "scope": scope, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
            "traffic": pmc["traffic"][0] if "traffic" in pmc else None,
            "traffic_source": pmc["traffic"][1] if "traffic" in pmc else None,
            "algorithmic_bytes": alg_step_bytes, "avg_us": round(dom_avg_s * 1e6, 3),
            "valu_frac": valu["frac"] if valu else None, "valu": valu, "kernels": kernels,
            "note": "scope 'launch': one launch is the whole step, avg_us = launch-stream event time of a whole "
                    "batch / steps (rocprofv3 kernel-trace average agrees, profiles/); otherwise avg_us = the "
                    "dominant kernel's event-bracketed launch time and achieved = the step's algorithmic bytes / "
                    "the summed durations of the step's launches. kernels[*].event_bracketed_us: every launch "
                    "between its own events (includes the events' gaps)"}


def compact_roofline(rl):
    return {k: rl[k] for k in ("kernel", "achieved", "frac", "avg_us", "traffic", "valu_frac", "algorithmic_bytes")}


def config_block(args, rs, ctx, name, world, dev, encode=True, decode=True):
    """One more single-GPU BASELINE config in the headline line (configs[2], configs[3]): the
    same device-resident calls, timed the same way (W untimed, K timed between barrier +
    synchronize, max over ranks; every rank an independent stripe), with the roofline of the
    dominant kernel of each operation.  Decode: the reference's loss pattern
    (benches/benchmarks.rs:113-138) at 1 % and 100 %; algorithmic bytes = received + restored rows."""
    import torch

    N, M, S = CONFIGS[name]
    timed, gpu_time = make_timer(world, dev)
    steps, warm = (max(3, min(args.steps, 20)), 3) if N * S <= (64 << 20) else (max(3, min(args.steps, 10)), 2)
    g = torch.Generator(device=dev)
    g.manual_seed(99 + N + S)
    d_orig = torch.randint(0, 256, (N, S), dtype=torch.uint8, device=dev, generator=g)
    d_rec = torch.empty((M, S), dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(device=dev)
    enc = rs.encode_device_call(N, M, S, d_orig, d_rec, stream=stream, ctx=ctx)
    step_bytes = (N + M) * S
    out = {"workload": f"{N}:{M} x {S} B", "steps": steps, "parallelism": f"replicas x{world}"}
    if encode:
        w = timed(enc, steps, warm)
        gt = gpu_time(enc, steps, stream)
        out["encode"] = {"GiBps": round(step_bytes * steps * world / w / 2**30, 2),
                         "us_per_step": round(w / steps * 1e6, 1),
                         "roofline": compact_roofline(roofline_of(rs, ctx, enc, 3, step_bytes, name, gt / steps))}
    else:
        enc()
    if decode:
        d_out = torch.empty((N, S), dtype=torch.uint8, device=dev)
        for pct in (1, 100):
            L = -(-min(N, M) * pct // 100)
            op = rs.present_mask([1] * (N - L) + [0] * L)
            rp = rs.present_mask([1] * L + [0] * (M - L))
            dec = rs.decode_device_call(N, M, S, d_orig, op, d_rec, rp, d_out, stream=stream, ctx=ctx)
            w = timed(dec, steps, warm)
            gt = gpu_time(dec, steps, stream)
            out[f"decode_{pct}pct"] = {
                "GiBps": round(step_bytes * steps * world / w / 2**30, 2), "us_per_step": round(w / steps * 1e6, 1),
                "roofline": compact_roofline(roofline_of(rs, ctx, dec, 3, (N + L) * S, name, gt / steps))}
        del d_out
    stream.synchronize()
    del d_orig, d_rec
    torch.cuda.empty_cache()
    return out


# ---------------------------------------------------------------------------
# one stripe per step (configs[1..3]); N > 1: independent stripes per rank

def stripe_bench(args, rs, ctx, config, world, rank, dev):
    import torch

    N, M, S = CONFIGS[config]
    timed, gpu_time = make_timer(world, dev)
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    d_orig = torch.randint(0, 256, (N, S), dtype=torch.uint8, device=dev, generator=g)
    d_rec = torch.empty((M, S), dtype=torch.uint8, device=dev)
    d_out = torch.empty((N, S), dtype=torch.uint8, device=dev)
    stream = torch.cuda.Stream(device=dev)

    # one C-ABI call per step (rs_encode_device_strided), arguments bound once:
    # the Python keyword wrapper would add ≈3 µs of host time to an 8 µs step
    enc = rs.encode_device_call(N, M, S, d_orig, d_rec, stream=stream, ctx=ctx)

    # ---- headline: encode -------------------------------------------------
    wall = timed(enc, args.steps, args.warmup)
    gpu_t = gpu_time(enc, args.steps, stream)
    step_bytes = (N + M) * S
    value = step_bytes * args.steps * world / wall / 2**30
    roofline = roofline_of(rs, ctx, enc, args.profile_steps, step_bytes, config, gpu_t / args.steps)

    # ---- decode at 1 % and 100 % loss (benchmarks.rs:113-138) --------------
    decode = {}
    if not args.no_decode:
        for pct in (1, 100):
            L = -(-min(N, M) * pct // 100)
            op = rs.present_mask([1] * (N - L) + [0] * L)
            rp = rs.present_mask([1] * L + [0] * (M - L))
            dec = rs.decode_device_call(N, M, S, d_orig, op, d_rec, rp, d_out, stream=stream, ctx=ctx)
            w = timed(dec, args.steps, args.warmup)
            gt = gpu_time(dec, args.steps, stream)
            decode[f"{pct}pct"] = round(step_bytes * args.steps * world / w / 2**30, 3)
            decode[f"{pct}pct_us_per_step"] = {"wall": round(w / args.steps * 1e6, 2),
                                               "gpu_events": round(gt / args.steps * 1e6, 2)}
            if pct == 1:
                # roofline of the decode's dominant kernel: algorithmic bytes = received + restored rows
                rl = roofline_of(rs, ctx, dec, args.profile_steps, (N + L) * S, config, gt / args.steps)
                decode["roofline_1pct"] = {k: rl[k] for k in ("kernel", "scope", "achieved", "frac", "avg_us",
                                                              "traffic", "valu_frac", "algorithmic_bytes")}

    # ---- a batch of stripes of the same shape per launch (MI355X extension:
    # rs_encode_device_batch / rs_decode_device_batch; one erasure pattern) ----
    batched = None
    if args.batch > 1 and N * S * args.batch <= (1 << 31):
        B = args.batch
        b_orig = torch.randint(0, 256, (B, N, S), dtype=torch.uint8, device=dev, generator=g)
        b_rec = torch.empty((B, M, S), dtype=torch.uint8, device=dev)
        b_out = torch.empty((B, N, S), dtype=torch.uint8, device=dev)
        bsteps = max(5, args.steps // 10)
        benc = lambda: rs.encode_device_batch(N, M, S, b_orig, b_rec, stream=stream, ctx=ctx)  # noqa: E731
        w_e = timed(benc, bsteps, max(2, args.warmup // 5))
        g_e = gpu_time(benc, bsteps, stream)
        L1 = -(-min(N, M) // 100)
        op1 = rs.present_mask([1] * (N - L1) + [0] * L1)
        rp1 = rs.present_mask([1] * L1 + [0] * (M - L1))
        w_d = timed(lambda: rs.decode_device_batch(N, M, S, b_orig, op1, b_rec, rp1, b_out, stream=stream, ctx=ctx),
                    bsteps, max(2, args.warmup // 5))
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
        # the host link's own floor for this call: one synchronous pinned copy of the
        # originals in and one of the recovery rows out, at these sizes (latency included)
        # plus the kernel, against the measured encode; and the link's bulk rate
        h2d_in, _ = host_link(dev, N * S)
        _, d2h_out = host_link(dev, M * S)
        bulk_h2d, bulk_d2h = host_link(dev, 256 << 20, reps=5)
        floor = h2d_in + d2h_out + gpu_t / args.steps
        host_e2e["link"] = {"h2d_us": round(h2d_in * 1e6, 2), "d2h_us": round(d2h_out * 1e6, 2),
                            "floor_us": round(floor * 1e6, 2), "encode_us": round(best[1] * 1e6, 2),
                            "frac_of_floor": round(floor / best[1], 3),
                            "bulk_h2d_GBps": round((256 << 20) / bulk_h2d / 1e9, 2),
                            "bulk_d2h_GBps": round((256 << 20) / bulk_d2h / 1e9, 2),
                            "note": "floor = one pinned copy in (N*S) + one out (M*S), each synchronous, "
                                    "+ the device encode; bulk = 256 MiB copies"}

    # ---- the drop-in object API (rank 0): ReedSolomonEncoder / Decoder calls as
    # the reference's benchmark makes them, through the C ABI in native code ----
    object_api = None
    if rank == 0 and not args.no_object:
        object_api = object_api_bench(N, M, S, max(20, args.steps // 4), 5)

    copy_ref = None if args.no_copy else device_copy(dev)

    # ---- the other single-GPU BASELINE configs, in the same line ----------------
    cfg3 = cfg4 = None
    if config == HEADLINE and not args.no_configs:
        cfg3 = config_block(args, rs, ctx, "32768x32768x1k", world, dev)                 # configs[2]
        cfg4 = config_block(args, rs, ctx, "8192x8192x64k", world, dev, encode=False)    # configs[3]

    # ---- configs[4] at the same N: strong scaling, column partition + RCCL all-gather ----
    sharded = None
    if config == HEADLINE and not args.no_sharded:
        sharded = sharded_block(args, rs, ctx, world, rank, dev)

    # ---- CPU baseline (rank 0, N = 1 only) ----------------------------------
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args.cpu_seconds, N, M, S)

    if rank == 0:
        line = {
            "metric": METRIC, "value": round(value, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(wall / args.steps * 1e3, 6),
            "us_per_step": round(wall / args.steps * 1e6, 2), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "u8", "data": "synthetic (uniform random bytes)",
            "config": {"workload": f"encode {N}:{M} x {S} B, device-resident (rs_encode_device)",
                       "original_count": N, "recovery_count": M, "shard_bytes": S,
                       "rate": "high" if rs.use_high_rate(N, M) == 1 else "low",
                       "parallelism": f"replicas x{world} (independent stripes)"},
            "gpu_event_ms_per_step": round(gpu_t / args.steps * 1e3, 5),
            "decode_GiBps": decode,
            "batched": batched,
            "host_e2e": host_e2e,
            "object_api": object_api,
            "roofline": roofline,
            "cpu_baseline": cpu,
            "device_copy": copy_ref,
            # last, so that a reader of the line's tail sees configs[2..4]
            "sharded": sharded,
            "config3": cfg3,
            "config4": cfg4,
        }
        print(json.dumps(line))


def object_api_bench(N, M, S, iters, warmup):
    """The object API in the reference benchmark's scope (benches/benchmarks.rs:97-139):
    N x rs_encoder_add_original_shard + rs_encoder_encode, and the decoder at 1 % / 100 %
    loss, host shards in and out, timed by tools/object_bench.cpp (built by build()) in a
    child process -- what a Rust caller of the INTEGRATION.md shim pays per call."""
    exe = os.path.join(ROOT, "reed-solomon-simd_amd", "lib", "rs_object_bench")
    if not os.path.exists(exe):
        return {"error": "rs_object_bench not built (run __graft_entry__.build())"}
    try:
        out = subprocess.run([exe, str(N), str(M), str(S), str(iters), str(warmup)], capture_output=True,
                             text=True, timeout=300)
    except subprocess.TimeoutExpired:
        return {"error": "timeout"}
    if out.returncode != 0:
        return {"error": (out.stderr or out.stdout).strip()[-300:]}
    r = json.loads(out.stdout.strip().splitlines()[-1])
    r["note"] = ("C ABI from native code: add shards (host, pinned staging) + encode/decode; one stream, "
                 "received rows in, recovery/restored rows out (PCIe included)")
    return r


def host_link(dev, nbytes, reps=50):
    """Seconds per synchronous pinned host->device and device->host copy of nbytes."""
    import torch

    h = torch.empty(nbytes, dtype=torch.uint8).pin_memory()
    d = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    out = []
    for fwd in (True, False):
        for i in range(reps + 2):
            if i == 2:
                t0 = time.perf_counter()
            if fwd:
                d.copy_(h, non_blocking=True)
            else:
                h.copy_(d, non_blocking=True)
            torch.cuda.synchronize()
        out.append((time.perf_counter() - t0) / reps)
    return out[0], out[1]


def device_copy(dev):
    """A 1 GiB device-to-device copy timed with events: the achievable-bandwidth context
    for roofline.peak (STREAM-copy GB/s)."""
    import torch

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
    return {"GBps": round(2 * nb * 10 / (e0.elapsed_time(e1) / 1e3) / 1e9, 1),
            "note": "torch device-to-device copy of 1 GiB (read + write bytes), context for roofline.peak"}


# ---------------------------------------------------------------------------
# configs[4]: one 32768:32768 x 64 KiB stripe column-partitioned over the ranks

def sharded_block(args, rs, ctx, world, rank, dev):
    """The "sharded" sub-object of every headline line: configs[4] at this N (strong scaling).
    Rank r holds byte columns [r*w, (r+1)*w), w = 64 KiB / N, of the originals; `step` = its
    encode in pieces + the RCCL all-gather of the recovery slices + the re-interleave
    (ShardedEncoder), `encode_only` = the slice encode alone, both max over ranks; the
    per-GPU roofline is the slice encode's.  `decode_1pct`: the reference's 1 % loss pattern
    (benches/benchmarks.rs:113-138) decoded column-partitioned (ShardedDecoder: eval_poly on
    every rank, slice decode, all-gather of the restored rows).  At N = 1 the step is the
    single-device encode / decode (nothing to gather)."""
    import torch

    N, M, S = CONFIGS[SHARDED]
    steps, warm = max(3, min(args.steps, 10)), 4  # (2 warmups read 4.1-5.1 ms per encode step on one box, profiles/r06ae)
    timed, _ = make_timer(world, dev)
    stream = torch.cuda.current_stream(dev)  # collectives are ordered after this stream's kernels
    w = S // world
    g = torch.Generator(device=dev)
    g.manual_seed(4321 + rank)
    d_orig = torch.randint(0, 256, (N, w), dtype=torch.uint8, device=dev, generator=g)  # this rank's columns
    d_rec = torch.empty((M, S), dtype=torch.uint8, device=dev)
    enc = rs.ShardedEncoder(N, M, S, device=dev, stream=stream, ctx=ctx) if world > 1 else None
    part = enc.part if world > 1 else d_rec
    compute = rs.encode_device_call(N, M, w, d_orig, part, stream=stream, ctx=ctx)
    t_comp = timed(compute, steps, warm) / steps
    t_step = timed(lambda: enc(d_orig, d_rec), steps, warm) / steps if world > 1 else t_comp
    per_gpu = (N + M) * w
    rl = roofline_of(rs, ctx, compute, 3, per_gpu, SHARDED)
    total = (N + M) * S
    out = {"config": f"{N}:{M} x {S} B (configs[4]), column slice of {w} B per GPU",
           "n_gpus": world, "scaling": "strong", "steps": steps,
           "step_ms": round(t_step * 1e3, 4), "GiBps": round(total / t_step / 2**30, 3),
           "encode_only": {"ms_per_step": round(t_comp * 1e3, 4), "GiBps": round(total / t_comp / 2**30, 3)},
           "allgather_and_interleave_ms": round((t_step - t_comp) * 1e3, 4),
           "pipeline_pieces": enc.chunks if world > 1 else 1,
           "per_gpu_roofline": {k: rl[k] for k in ("kernel", "achieved", "frac", "traffic", "valu_frac")},
           "parallelism": f"column partition x{world}" + (
               "" if world == 1 else " + all_gather (gloo rehearsal on one GPU)"
               if os.environ.get("RS_BENCH_REHEARSE") == "1" else " + all_gather_into_tensor (RCCL)")}
    if world > 1:  # the committed PMC figures are the whole matrix's (N = 1), not a slice's
        out["per_gpu_roofline"].update(traffic=None, valu_frac=None)
    del enc
    # column-partitioned decode at 1 % loss: every rank restores the lost originals' full rows
    L = -(-min(N, M) // 100)
    op = rs.present_mask([1] * (N - L) + [0] * L)
    rp = rs.present_mask([1] * L + [0] * (M - L))
    rec_cols = part if world > 1 else d_rec  # this rank's recovery columns (its own encode above)
    d_x = torch.empty((N, S), dtype=torch.uint8, device=dev)
    if world > 1:
        dec = rs.ShardedDecoder(N, M, S, device=dev, stream=stream, ctx=ctx)
        x_cols = torch.empty((N, w), dtype=torch.uint8, device=dev)
        dcomp = rs.decode_device_call(N, M, w, d_orig, op, rec_cols, rp, x_cols, stream=stream, ctx=ctx)
        td_comp = timed(dcomp, steps, warm) / steps
        td_step = timed(lambda: dec(d_orig, op, rec_cols, rp, d_x), steps, warm) / steps
        del dec, x_cols
    else:
        dcomp = rs.decode_device_call(N, M, w, d_orig, op, rec_cols, rp, d_x, stream=stream, ctx=ctx)
        td_comp = td_step = timed(dcomp, steps, warm) / steps
    out["decode_1pct"] = {"step_ms": round(td_step * 1e3, 4), "GiBps": round(total / td_step / 2**30, 3),
                          "decode_only_ms": round(td_comp * 1e3, 4),
                          "decode_only_GiBps": round(total / td_comp / 2**30, 3),
                          "restored_rows": L}
    del d_orig, d_rec, d_x
    torch.cuda.empty_cache()
    return out


def sharded_bench(args, rs, ctx, world, rank, dev):
    """SURVEY.md 8(e), DESIGN.md "Multi-GPU": rank r encodes byte columns [r*w, (r+1)*w),
    w = 64 KiB / world, of its resident column slice of the originals, and an all-gather (RCCL
    over xGMI) assembles the whole [M x S] recovery matrix on every rank
    (reed_solomon_simd.ShardedEncoder; at N > 1 in pieces whose all-gathers overlap the next
    piece's encode and the previous one's interleave).  Total work is fixed: strong scaling.  Reported: the
    whole step (encode + all-gather + re-interleave) and encode alone."""
    import torch

    N, M, S = CONFIGS[SHARDED]
    timed, gpu_time = make_timer(world, dev)
    stream = torch.cuda.current_stream(dev)  # collectives are ordered after this stream's kernels
    if world > 1:
        shard = rs.ShardedEncoder(N, M, S, device=dev, stream=stream, ctx=ctx)
    w = S // world
    g = torch.Generator(device=dev)
    g.manual_seed(1234 + rank)
    d_orig = torch.randint(0, 256, (N, w), dtype=torch.uint8, device=dev, generator=g)  # this rank's columns
    d_rec = torch.empty((M, S), dtype=torch.uint8, device=dev)
    part = shard.part if world > 1 else d_rec
    compute = rs.encode_device_call(N, M, w, d_orig, part, stream=stream, ctx=ctx)

    def step():
        if world > 1:
            shard(d_orig, d_rec)  # pieces of the slice: encode, all-gather and interleave pipelined
        else:
            compute()

    t_step = timed(step, args.steps, args.warmup) / args.steps
    t_comp = timed(compute, args.steps, args.warmup) / args.steps
    per_gpu = (N + M) * w
    roofline = roofline_of(rs, ctx, compute, max(3, args.profile_steps // 10), per_gpu, SHARDED)
    total = (N + M) * S
    cpu = None
    if rank == 0 and not args.no_cpu:
        cpu = cpu_baseline(min(args.cpu_seconds, 10.0), N, M, S)
    if rank == 0:
        print(json.dumps({
            "metric": "GiB/s (original+recovery) encode, device-resident, 32768:32768x65536B column-partitioned "
                      "+ RCCL all-gather",
            "value": round(total / t_step / 2**30, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(t_step * 1e3, 4), "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "u8", "data": "synthetic (uniform random bytes)",
            "config": {"workload": "encode 32768:32768 x 64 KiB (configs[4]), column slice of 64 KiB / n per GPU",
                       "original_count": N, "recovery_count": M, "shard_bytes": S, "slice_bytes": w,
                       "parallelism": f"column partition x{world} + all_gather_into_tensor (RCCL)"},
            "encode_only": {"ms_per_step": round(t_comp * 1e3, 4), "GiBps": round(total / t_comp / 2**30, 3)},
            "allgather_and_interleave_ms": round((t_step - t_comp) * 1e3, 4),
            "pipeline_pieces": shard.chunks if world > 1 else 1,
            "roofline": roofline,
            "cpu_baseline": cpu,
        }))


# ---------------------------------------------------------------------------
# --shape-table: the reference's published shape table (README.md:27-45)

README_SHAPES = [(32, 32), (64, 64), (128, 128), (256, 256), (512, 512), (1024, 1024), (2048, 2048),
                 (4096, 4096), (8192, 8192), (16384, 16384), (32768, 32768), (128, 1024), (1000, 100),
                 (1000, 10000), (8192, 57344), (10000, 1000), (57344, 8192)]


def _route(rs, ctx, fn):
    """The kernels one call launches (rs_profile_enable records), e.g. 'k_mono<10, ...>' or the passes."""
    import torch

    rs.profile_enable(True, ctx=ctx)
    fn()
    torch.cuda.synchronize()
    recs = rs.profile_collect(ctx)
    rs.profile_enable(False, ctx=ctx)
    return " + ".join(name for name, _, _ in recs)


def _cpu_rate(fn, unit_bytes, seconds):
    fn()
    it, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        fn()
        it += 1
    return unit_bytes * it / (time.perf_counter() - t0) / 2**30


def shape_table(args, rs, ctx, dev):
    """Every shape of the reference's benchmark table (README.md:27-45) at 1 KiB shards: device-
    resident encode and decode (1 % and 100 % original loss, the reference's pattern
    benches/benchmarks.rs:113-138), wall time of `--steps` calls (at most 50) on one stream; the
    route (kernels of one call); the AVX2 port (oracle/avx2_port.c) on one core, ≈0.2 s per
    measurement.  GiB/s are of original + recovery bytes, as in the reference's table."""
    import numpy as np
    import torch
    import oracle_lib as O

    S = 1024
    timed, _ = make_timer(1, dev)
    stream = torch.cuda.Stream(device=dev)
    steps = max(5, min(args.steps, 50))
    cpu_ok = not args.no_cpu and O.lib().orc_select_engine(1) == 0
    rows = []
    for N, M in README_SHAPES:
        g = torch.Generator(device=dev)
        g.manual_seed(N * 7 + M)
        d_orig = torch.randint(0, 256, (N, S), dtype=torch.uint8, device=dev, generator=g)
        d_rec = torch.empty((M, S), dtype=torch.uint8, device=dev)
        d_out = torch.empty((N, S), dtype=torch.uint8, device=dev)
        enc = rs.encode_device_call(N, M, S, d_orig, d_rec, stream=stream, ctx=ctx)
        step_bytes = (N + M) * S
        row = {"shape": f"{N}:{M}", "rate": "high" if rs.use_high_rate(N, M) == 1 else "low"}
        w = timed(enc, steps, 3)
        row["encode_GiBps"] = round(step_bytes * steps / w / 2**30, 2)
        row["encode_us"] = round(w / steps * 1e6, 2)
        row["encode_route"] = _route(rs, ctx, enc)
        enc()
        torch.cuda.synchronize()
        h_orig, h_rec = d_orig.cpu().numpy(), d_rec.cpu().numpy()
        for pct in (1, 100):
            L = -(-min(N, M) * pct // 100)
            opf, rpf = [1] * (N - L) + [0] * L, [1] * L + [0] * (M - L)
            dec = rs.decode_device_call(N, M, S, d_orig, rs.present_mask(opf), d_rec, rs.present_mask(rpf), d_out,
                                        stream=stream, ctx=ctx)
            w = timed(dec, steps, 3)
            row[f"decode_{pct}pct_GiBps"] = round(step_bytes * steps / w / 2**30, 2)
            row[f"decode_{pct}pct_us"] = round(w / steps * 1e6, 2)
            if pct == 1:
                row["decode_route"] = _route(rs, ctx, dec)
            if cpu_ok:
                row[f"cpu_decode_{pct}pct_GiBps"] = round(_cpu_rate(
                    lambda: O.decode("default", h_orig, np.array(opf, np.uint8), h_rec, np.array(rpf, np.uint8)),
                    step_bytes, 0.2), 3)
        if cpu_ok:
            row["cpu_encode_GiBps"] = round(_cpu_rate(lambda: O.encode("default", h_orig, M), step_bytes, 0.2), 3)
        rows.append(row)
        del d_orig, d_rec, d_out
    if cpu_ok:
        O.lib().orc_select_engine(0)
    print(json.dumps({"metric": "shape table (README.md:27-45), 1 KiB shards, GiB/s of original + recovery",
                      "steps": steps, "cpu": (f"AVX2 port, 1 thread, {_cpu_model()}" if cpu_ok else None),
                      "rows": rows}))


# ---------------------------------------------------------------------------
# CPU baseline: the reference's AVX2 engine restated in C (oracle/avx2_port.c)

def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform
    return platform.processor() or platform.machine()


def cpu_baseline(seconds, N, M, S):
    """The AVX2 restatement of the reference engine (oracle/avx2_port.c) on a bounded sample of
    the workload (shard copy-in + encode, like benches/benchmarks.rs:101-107): `value` on 1 thread
    (the reference is single-threaded); `all_cores` = independent encodes on every host thread
    this process may use (at most 16, the GPU box's CPU share), an upper bound.  Large shards
    are sampled by 64-byte column blocks: every engine op is column-wise, so a 64-B-shard encode
    is the same work per byte."""
    import threading

    import numpy as np
    import oracle_lib as O

    cols = S if N * S <= (64 << 20) else 64
    if O.lib().orc_select_engine(1) != 0:
        return {"value": None, "unit": "GiB/s", "cores": 1, "kind": "port", "sample": "AVX2 unavailable on host"}
    orig = np.random.default_rng(0).integers(0, 256, (N, cols), dtype=np.uint8)
    O.encode("default", orig, M)  # tables built once, before any thread starts
    it, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        O.encode("default", orig, M)
        it += 1
    dt = time.perf_counter() - t0

    threads = max(1, min(16, len(os.sched_getaffinity(0))))
    counts = [0] * threads
    stop = time.perf_counter() + max(1.0, seconds / 2)

    def worker(i):  # ctypes releases the GIL; the oracle's work buffer is thread-local
        mine = orig.copy()
        while time.perf_counter() < stop:
            O.encode("default", mine, M)
            counts[i] += 1

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(threads)]
    t1 = time.perf_counter()
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    dt_all = time.perf_counter() - t1
    O.lib().orc_select_engine(0)
    unit_bytes = (N + M) * cols
    shape = f"{N}:{M} x {cols} B" + ("" if cols == S else f" (one 64-byte column block of the {S} B shards)")
    return {"value": round(unit_bytes * it / dt / 2**30, 4), "unit": "GiB/s", "cores": 1, "kind": "port",
            "sample": f"{it} encodes of {shape} in {dt:.1f} s (shard copy-in + encode, like "
                      f"benches/benchmarks.rs:101-107), single thread, {_cpu_model()}",
            "all_cores": {"value": round(unit_bytes * sum(counts) / dt_all / 2**30, 4), "cores": threads,
                          "sample": f"{sum(counts)} independent encodes on {threads} threads in {dt_all:.1f} s"}}


if __name__ == "__main__":
    main()
