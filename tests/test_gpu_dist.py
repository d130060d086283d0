"""Multi-rank column-partitioned encode with the real HIP kernels (GPU box, one GPU).

Two gloo ranks share cuda:0: each encodes its column slice in pieces through the device
API (rs_encode_device_strided on strided column views) and the pieces' all-gathers (gloo
on CUDA tensors; RCCL in the bench) and interleaves run pipelined (ShardedEncoder).  The
assembled recovery matrix must equal the oracle on every rank.  RCCL itself needs one GPU
per rank, so the collective here is gloo; everything else is the product path.
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
