"""Multi-rank plumbing on CPU (gloo, 127.0.0.1).

- Column-partitioned encode: the product's
  `encode_device_sharded` / `ShardedEncoder` (partition into whole 64-byte
  blocks, per-rank slice encode, all-gather, re-interleave), world sizes 2 and
  4.  Only the per-slice device call (`encode_device` = rs_encode_device_strided
  on the GPU) is replaced by a CPU stand-in (the oracle); everything around it
  is the product code.
- bench.py's max-over-ranks timing reduction, and its `--gpus N` launcher:
  the parent process starts N ranks (torch.distributed.run) and rank 0 reports
  n_gpus = the process group's world size.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _worker_sharded(rank, world, port, N, M, S, rate, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    import reed_solomon_simd as rs
    _init(rank, world, port)
    calls = []

    def slice_standin(n, m, w, cols, out, stream=None, rate_=0, ctx=None):
        # CPU stand-in for rs_encode_device_strided on this rank's column slice
        assert (n, m, w) == (N, M, S // world) and cols.shape == (N, w) and out.shape == (M, w)
        calls.append(w)
        out.copy_(torch.from_numpy(O.encode(rate, np.ascontiguousarray(cols.numpy()), m)))

    rs.encode_device = slice_standin
    try:
        orig = O.generate_original(N, S, 21)
        d_orig = torch.from_numpy(orig)
        want = O.encode(rate, orig, M)
        ok = True
        for _ in range(2):  # second call reuses the cached ShardedEncoder's buffers
            d_rec = torch.zeros((M, S), dtype=torch.uint8)
            rs.encode_device_sharded(N, M, S, d_orig, d_rec, rate_={"high": 1, "low": 2}[rate])
            ok = ok and bool(np.array_equal(d_rec.numpy(), want))
        q.put((rank, (ok, len(calls), len(rs._sharded_cache))))
    finally:
        dist.destroy_process_group()


def _worker_pipelined(rank, world, port, N, M, S, chunks, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    import reed_solomon_simd as rs
    _init(rank, world, port)
    widths = []

    def piece_standin(cols, out):
        # CPU stand-in for the per-piece device encode (rs_encode_device_strided on a column piece)
        widths.append(cols.shape[1])
        out.copy_(torch.from_numpy(O.encode("high", np.ascontiguousarray(cols.numpy()), M)))

    try:
        orig = O.generate_original(N, S, 5 + chunks)
        want = O.encode("high", orig, M)
        enc = rs.ShardedEncoder(N, M, S, group=None, rate_=1, encode_slice=piece_standin, chunks=chunks)
        ok = True
        for _ in range(2):
            d_rec = torch.zeros((M, S), dtype=torch.uint8)
            enc(enc.columns(torch.from_numpy(orig)), d_rec)
            ok = ok and bool(np.array_equal(d_rec.numpy(), want))
        # the unpipelined path (one slice encode, then gather) gives the same matrix
        enc.encode_local(enc.columns(torch.from_numpy(orig)))
        d2 = torch.zeros((M, S), dtype=torch.uint8)
        enc.gather(d2)
        ok = ok and bool(np.array_equal(d2.numpy(), want))
        q.put((rank, (ok, widths)))
    finally:
        dist.destroy_process_group()


def _worker_reduce(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    import bench
    _init(rank, world, port)
    try:
        q.put((rank, bench.reduce_max(1.5 + rank, world, "cpu")))
    finally:
        dist.destroy_process_group()


def _spawn(fn, world, *args):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port) + args + (q,)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


@pytest.mark.parametrize("world,N,M,S,rate", [(2, 64, 64, 256, "high"), (2, 100, 300, 512, "low"),
                                              (2, 1000, 1000, 128, "high"), (4, 300, 200, 1024, "high")])
def test_column_partitioned_encode(world, N, M, S, rate):
    out = _spawn(_worker_sharded, world, N, M, S, rate)
    assert out == {r: (True, 2, 1) for r in range(world)}


@pytest.mark.parametrize("world,N,M,S,chunks", [(2, 64, 64, 512, 2), (2, 300, 200, 1024, 4), (4, 100, 100, 1024, 4),
                                                (2, 64, 64, 256, 1)])
def test_pipelined_column_partitioned_encode(world, N, M, S, chunks):
    """ShardedEncoder in pieces: piece c's all-gather (async) overlaps piece c+1's encode and
    piece c-1's interleave; every rank ends with the single-device recovery matrix."""
    out = _spawn(_worker_pipelined, world, N, M, S, chunks)
    w = S // world
    assert out == {r: (True, [w // chunks] * (2 * chunks) + [w]) for r in range(world)}


def test_bench_max_over_ranks_world2():
    out = _spawn(_worker_reduce, 2)
    assert out == {0: 2.5, 1: 2.5}


def test_bench_gpus_flag_launches_ranks():
    """`python bench.py --gpus 2` from a plain parent starts 2 ranks; --plumbing runs the rank
    set-up, barriers and max-over-ranks timing on gloo without touching a GPU."""
    import json
    import subprocess
    import sys

    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--plumbing", "--steps", "3",
                        "--warmup", "1"], capture_output=True, text=True, timeout=240, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks_seen"] == [0, 1] and lines[0]["steps"] == 3


def _worker_sharded_decode(rank, world, port, N, M, S, chunks, q):
    """ShardedDecoder / decode_device_sharded with the per-piece device decode replaced by the
    oracle: every rank must end with the missing originals' full rows, present rows untouched."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    import reed_solomon_simd as rs
    _init(rank, world, port)
    widths = []

    def piece_standin(orig_cols, op, rec_cols, rp, out):
        # CPU stand-in for rs_decode_device_strided on a column piece: only missing rows written
        widths.append(out.shape[1])
        opa, rpa = np.frombuffer(op, np.uint8), np.frombuffer(rp, np.uint8)
        got = O.decode("high", np.ascontiguousarray(orig_cols.numpy()), opa, np.ascontiguousarray(rec_cols.numpy()),
                       rpa)
        miss = np.flatnonzero(opa == 0)
        out[torch.from_numpy(miss)] = torch.from_numpy(got[miss])

    try:
        rng = np.random.default_rng(9)
        orig = O.generate_original(N, S, 31)
        rec = O.encode("high", orig, M)
        L1 = -(-min(N, M) // 100)
        patterns = [
            ([1] * (N - L1) + [0] * L1, [1] * L1 + [0] * (M - L1)),              # benchmarks.rs:113-138, 1 %
            ([1] * (N - min(N, M)) + [0] * min(N, M), [1] * min(N, M) + [0] * (M - min(N, M))),  # 100 %
        ]
        lost = rng.choice(N, size=min(N, M) // 3, replace=False)
        opr = np.ones(N, np.uint8)
        opr[lost] = 0
        patterns.append((list(opr), [1] * M))                                 # scattered
        patterns.append(([1] * N, [0] * M))                                   # nothing to restore
        dec = rs.ShardedDecoder(N, M, S, rate_=1, decode_slice=piece_standin, chunks=chunks)
        ok = True
        for op, rp in patterns:
            for _ in range(2):  # the second call reuses the pattern's gather buffers
                out = torch.full((N, S), 0xAB, dtype=torch.uint8)
                dec(dec.columns(torch.from_numpy(orig)), op, dec.columns(torch.from_numpy(rec)), rp, out)
                o = out.numpy()
                miss = np.flatnonzero(np.asarray(op) == 0)
                keep = np.flatnonzero(np.asarray(op) != 0)
                ok = ok and bool(np.array_equal(o[miss], orig[miss])) and bool((o[keep] == 0xAB).all())
        # the cached module-level entry point with the device call replaced
        rs.decode_device = lambda n, m, w, oc, op, rc, rp, out, stream=None, rate_=0, ctx=None: piece_standin(
            oc, op, rc, rp, out)
        out = torch.zeros((N, S), dtype=torch.uint8)
        op, rp = patterns[0]
        rs.decode_device_sharded(N, M, S, torch.from_numpy(orig), rs.present_mask(op), torch.from_numpy(rec),
                                 rs.present_mask(rp), out, rate_=1)
        miss = np.flatnonzero(np.asarray(op) == 0)
        ok = ok and bool(np.array_equal(out.numpy()[miss], orig[miss]))
        q.put((rank, (ok, sorted(set(widths)))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N,M,S,chunks", [(2, 64, 64, 512, 2), (2, 300, 200, 1024, 4), (4, 100, 100, 1024, 4),
                                                (4, 1000, 1000, 256, 1)])
def test_column_partitioned_decode(world, N, M, S, chunks):
    """eval_poly replicated per rank, each rank decodes its column slice, the
    restored rows are all-gathered and re-interleaved (ShardedDecoder); 1 %, 100 %,
    scattered and no loss, at world sizes 2 and 4."""
    out = _spawn(_worker_sharded_decode, world, N, M, S, chunks)
    # pieces of the explicit decoder, then the whole slice (decode_device_sharded's default for slices < 4 KiB)
    assert out == {r: (True, sorted({S // world // chunks, S // world})) for r in range(world)}, out


def _worker_forced(rank, world, port, q):
    """world 1 with force_collective: pieces -> all-gather of one rank -> interleave."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    import reed_solomon_simd as rs
    _init(rank, world, port)
    try:
        N, M, S = 200, 100, 512
        orig = O.generate_original(N, S, 3)
        want = O.encode("high", orig, M)
        calls = []

        def enc_standin(cols, out):
            calls.append(cols.shape[1])
            out.copy_(torch.from_numpy(O.encode("high", np.ascontiguousarray(cols.numpy()), M)))

        enc = rs.ShardedEncoder(N, M, S, rate_=1, encode_slice=enc_standin, chunks=4, force_collective=True)
        d_rec = torch.zeros((M, S), dtype=torch.uint8)
        enc(enc.columns(torch.from_numpy(orig)), d_rec)
        q.put((rank, (bool(np.array_equal(d_rec.numpy(), want)), enc.collective, calls)))
    finally:
        dist.destroy_process_group()


def test_forced_collective_world1():
    out = _spawn(_worker_forced, 1)
    assert out == {0: (True, True, [128] * 4)}


def _worker_config5_geometry(rank, world, port, N, M, S, q):
    """configs[4]'s split at world 8: S = 64 KiB over 8 ranks is an 8 KiB slice
    per rank, coded in 4 pieces of 2 KiB -- the smallest piece the default chunking allows.
    Encode through ShardedEncoder and the cached encode_device_sharded, decode at 1 % / 100 % /
    scattered loss through ShardedDecoder, with only the per-piece device call replaced by the
    oracle (/root/reference/src/engine/utils.rs:35-43: every op is column-wise)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib as O
    import reed_solomon_simd as rs
    _init(rank, world, port)
    enc_w, dec_w = [], []

    def enc_piece(cols, out):
        enc_w.append(cols.shape[1])
        out.copy_(torch.from_numpy(O.encode("high", np.ascontiguousarray(cols.numpy()), M)))

    def dec_piece(orig_cols, op, rec_cols, rp, out):
        dec_w.append(out.shape[1])
        opa, rpa = np.frombuffer(op, np.uint8), np.frombuffer(rp, np.uint8)
        got = O.decode("high", np.ascontiguousarray(orig_cols.numpy()), opa, np.ascontiguousarray(rec_cols.numpy()),
                       rpa)
        miss = np.flatnonzero(opa == 0)
        out[torch.from_numpy(miss)] = torch.from_numpy(got[miss])

    try:
        orig = O.generate_original(N, S, 77)
        want = O.encode("high", orig, M)
        enc = rs.ShardedEncoder(N, M, S, rate_=1, encode_slice=enc_piece)
        ok = {"encode": True, "decode": True}
        d_rec = torch.zeros((M, S), dtype=torch.uint8)
        enc(enc.columns(torch.from_numpy(orig)), d_rec)
        ok["encode"] = bool(np.array_equal(d_rec.numpy(), want))
        # the module-level entry point (cached ShardedEncoder) with the device call replaced
        rs.encode_device = lambda n, m, w, cols, out, stream=None, rate_=0, ctx=None: enc_piece(cols, out)
        d2 = torch.zeros((M, S), dtype=torch.uint8)
        rs.encode_device_sharded(N, M, S, torch.from_numpy(orig), d2, rate_=1)
        ok["encode"] = ok["encode"] and bool(np.array_equal(d2.numpy(), want))
        rng = np.random.default_rng(123)
        L1 = -(-min(N, M) // 100)
        scat = np.ones(N, np.uint8)
        scat[rng.choice(N, size=min(N, M) // 2, replace=False)] = 0
        patterns = [([1] * (N - L1) + [0] * L1, [1] * L1 + [0] * (M - L1)),  # benchmarks.rs:113-138, 1 %
                    ([0] * min(N, M) + [1] * (N - min(N, M)), [1] * M),       # 100 % (of min(N, M))
                    (list(scat), [1] * M)]                                    # scattered
        dec = rs.ShardedDecoder(N, M, S, rate_=1, decode_slice=dec_piece)
        for op, rp in patterns + patterns[:1]:  # a repeat reuses the pattern's views
            out = torch.full((N, S), 0xAB, dtype=torch.uint8)
            dec(dec.columns(torch.from_numpy(orig)), op, dec.columns(torch.from_numpy(want)), rp, out)
            o = out.numpy()
            miss = np.flatnonzero(np.asarray(op) == 0)
            keep = np.flatnonzero(np.asarray(op) != 0)
            ok["decode"] = ok["decode"] and bool(np.array_equal(o[miss], orig[miss])) and bool((o[keep] == 0xAB).all())
        q.put((rank, (ok, enc.w, enc.chunks, sorted(set(enc_w)), sorted(set(dec_w)))))
    finally:
        dist.destroy_process_group()


def test_world8_config5_geometry():
    """World 8 at configs[4]'s column geometry (64 KiB shards: 8 KiB per rank, 4 pieces of
    2 KiB), with few rows so the oracle finishes in seconds."""
    N, M, S = 200, 100, 65536
    out = _spawn(_worker_config5_geometry, 8, N, M, S)
    assert out == {r: ({"encode": True, "decode": True}, 8192, 4, [2048], [2048]) for r in range(8)}, out


def _worker_mask_mismatch(rank, world, port, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))
    import reed_solomon_simd as rs
    _init(rank, world, port)
    try:
        os.environ["RS_MI355X_DEBUG_MASKS"] = "1"
        dec = rs.ShardedDecoder(64, 64, 256, rate_=1, decode_slice=lambda *a: None)
        op = [1] * 64
        op[rank] = 0  # a different lost shard on every rank
        try:
            dec(torch.zeros((64, 128), dtype=torch.uint8), op, torch.zeros((64, 128), dtype=torch.uint8), [1] * 64,
                torch.zeros((64, 256), dtype=torch.uint8))
            q.put((rank, "no error"))
        except ValueError as e:
            q.put((rank, "different" in str(e)))
    finally:
        dist.destroy_process_group()


def test_sharded_decoder_rejects_different_masks_in_debug_mode():
    """the gathers are sized by the loss count, so ranks with different erasure
    patterns would hang; RS_MI355X_DEBUG_MASKS=1 all-reduces a hash of the mask first."""
    assert _spawn(_worker_mask_mismatch, 2) == {0: True, 1: True}
