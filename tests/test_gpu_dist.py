"""Multi-rank column-partitioned encode / decode with the real HIP kernels (GPU box, one GPU).

- Two gloo ranks share cuda:0: each codes its column slice in pieces through the device
  API (rs_encode_device_strided / rs_decode_device_strided on strided column views) and the
  pieces' all-gathers (gloo on CUDA tensors) and interleaves run pipelined
  (ShardedEncoder / ShardedDecoder).  The assembled matrices must equal the oracle on every rank.
- RCCL: one rank on the "nccl" backend (init with device_id=, as bench.py does) runs the
  same pipeline with force_collective=True, so all_gather_into_tensor, the collective's own
  stream and work.wait() ordering run on the GPU against the oracle (RCCL needs one GPU per
  rank, so one rank is what a one-GPU box can run).
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, N, M, S, chunks, side, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    import oracle_lib as O
    import reed_solomon_simd as rs

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        # side: the encoder runs on a caller-supplied stream that is not the current
        # one; the inputs of every round are written on the current stream just before
        # the call, and the pieces are reused round after round
        stream = torch.cuda.Stream() if side else None
        enc = rs.ShardedEncoder(N, M, S, device="cuda:0", chunks=chunks, stream=stream)
        origs = [O.generate_original(N, S, 77 + it) for it in range(3)]
        d_cols = [torch.from_numpy(o[:, rank * enc.w:(rank + 1) * enc.w].copy()).cuda() for o in origs]
        cols = torch.empty_like(d_cols[0])
        d_rec = torch.zeros((M, S), dtype=torch.uint8, device="cuda:0")
        torch.cuda.synchronize()
        ok = True
        for it, orig in enumerate(origs):
            d_rec.zero_()
            cols.copy_(d_cols[it])  # on the current stream
            enc(cols, d_rec)
            torch.cuda.synchronize()
            got = d_rec.cpu().numpy()
            if rank == 0:
                want = O.encode("default", orig, M)
                ok = ok and bool(np.array_equal(got, want))
            else:  # every rank holds the same matrix
                ok = ok and bool(np.array_equal(got[:, :64], O.encode("default", np.ascontiguousarray(orig[:, :64]), M)))
        rs.check_device()
        q.put((rank, ok))
    except Exception as e:  # report, do not hang the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("N,M,S,chunks,side", [(1024, 1024, 8192, 4, False), (700, 300, 2048, 2, False),
                                               (1024, 1024, 8192, 4, True)])
def test_sharded_pipelined_encode_two_ranks_one_gpu(N, M, S, chunks, side):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, N, M, S, chunks, side, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=110) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    assert out == {0: True, 1: True}, out


def _decode_worker(rank, world, port, N, M, S, chunks, side, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    import oracle_lib as O
    import reed_solomon_simd as rs

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.cuda.set_device(0)
        stream = torch.cuda.Stream() if side else None
        dec = rs.ShardedDecoder(N, M, S, device="cuda:0", chunks=chunks, stream=stream)
        orig = O.generate_original(N, S, 41)
        rec = O.encode("default", orig, M)
        d_o = torch.from_numpy(orig[:, rank * dec.w:(rank + 1) * dec.w].copy()).cuda()
        d_r = torch.from_numpy(rec[:, rank * dec.w:(rank + 1) * dec.w].copy()).cuda()
        ok = True
        for op, rp in _patterns(N, M):
            out = torch.full((N, S), 0xAB, dtype=torch.uint8, device="cuda:0")
            dec(d_o, op, d_r, rp, out)
            torch.cuda.synchronize()
            ok = ok and _restored_ok(out.cpu().numpy(), orig, op)
        rs.check_device()
        q.put((rank, ok))
    except Exception as e:
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _patterns(N, M):
    """1 % (benches/benchmarks.rs:113-138), scattered and 100 % loss."""
    L1 = -(-min(N, M) // 100)
    rng = np.random.default_rng(N + M)
    sc = np.ones(N, np.uint8)
    sc[rng.choice(N, size=min(N, M) // 4, replace=False)] = 0
    L = min(N, M)
    return [([1] * (N - L1) + [0] * L1, [1] * L1 + [0] * (M - L1)), (list(sc), [1] * M),
            ([1] * (N - L) + [0] * L, [1] * L + [0] * (M - L))]


def _restored_ok(got, orig, op):
    op = np.asarray(op)
    miss, keep = np.flatnonzero(op == 0), np.flatnonzero(op != 0)
    return bool(np.array_equal(got[miss], orig[miss])) and bool((got[keep] == 0xAB).all())


@pytest.mark.parametrize("N,M,S,chunks,side", [(1024, 1024, 8192, 4, True), (700, 300, 2048, 2, False)])
def test_sharded_pipelined_decode_two_ranks_one_gpu(N, M, S, chunks, side):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_decode_worker, args=(r, 2, port, N, M, S, chunks, side, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=110) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    assert out == {0: True, 1: True}, out


def _nccl_worker(port, N, M, S, chunks, q):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "reed-solomon-simd_amd"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist
    import oracle_lib as O
    import reed_solomon_simd as rs

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        res = {"backend": dist.get_backend()}
        stream = torch.cuda.Stream()  # a caller stream that is not the current one
        enc = rs.ShardedEncoder(N, M, S, device="cuda:0", chunks=chunks, stream=stream, force_collective=True)
        dec = rs.ShardedDecoder(N, M, S, device="cuda:0", chunks=chunks, stream=stream, force_collective=True)
        res["collective"] = (enc.collective, dec.collective, enc.nccl, enc.chunks)
        ok = True
        d_rec = torch.zeros((M, S), dtype=torch.uint8, device="cuda:0")
        cols = torch.empty((N, S), dtype=torch.uint8, device="cuda:0")
        for it in range(2):  # pieces and gather buffers reused across calls
            orig = O.generate_original(N, S, 50 + it)
            cols.copy_(torch.from_numpy(orig))  # written on the current stream just before the call
            d_rec.zero_()
            enc(enc.columns(cols), d_rec)
            torch.cuda.synchronize()
            rec = d_rec.cpu().numpy()
            ok = ok and bool(np.array_equal(rec, O.encode("default", orig, M)))
            for op, rp in _patterns(N, M):
                out = torch.full((N, S), 0xAB, dtype=torch.uint8, device="cuda:0")
                dec(dec.columns(cols), op, dec.columns(d_rec), rp, out)
                torch.cuda.synchronize()
                ok = ok and _restored_ok(out.cpu().numpy(), orig, op)
        rs.check_device()
        res["ok"] = ok
        q.put(res)
    except Exception as e:
        q.put({"error": repr(e)})
    finally:
        dist.destroy_process_group()


def test_rccl_forced_collective_one_rank():
    """the RCCL path (all_gather_into_tensor on the nccl backend, its own
    stream, work.wait()) on hardware, config-5-shaped pieces (4096:4096 x 8 KiB, 4 pieces,
    caller stream), encode and decode against the oracle."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), 4096, 4096, 8192, 4, q))
    p.start()
    out = q.get(timeout=110)
    p.join(timeout=30)
    assert out == {"backend": "nccl", "collective": (True, True, True, 4), "ok": True}, out
