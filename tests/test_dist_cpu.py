"""Multi-rank plumbing on CPU (gloo, world_size 2, 127.0.0.1).

- Column-partitioned encode: the product's
  `_sharded_encode` (partition into whole 64-byte blocks, all-gather,
  re-interleave) with the CPU oracle injected as the per-rank slice encoder
  -- on the GPU the slice encoder is rs_encode_device_strided.
- bench.py's max-over-ranks timing reduction.
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
    try:
        orig = O.generate_original(N, S, 21)
        d_orig = torch.from_numpy(orig)
        d_rec = torch.zeros((M, S), dtype=torch.uint8)

        def enc_slice(cols, out):
            out.copy_(torch.from_numpy(O.encode(rate, np.ascontiguousarray(cols.numpy()), M)))

        rs._sharded_encode(N, M, S, d_orig, d_rec, enc_slice)
        want = O.encode(rate, orig, M)
        q.put((rank, bool(np.array_equal(d_rec.numpy(), want))))
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


@pytest.mark.parametrize("N,M,S,rate", [(64, 64, 256, "high"), (100, 300, 512, "low"), (1000, 1000, 128, "high")])
def test_column_partitioned_encode_world2(N, M, S, rate):
    out = _spawn(_worker_sharded, 2, N, M, S, rate)
    assert out == {0: True, 1: True}


def test_bench_max_over_ranks_world2():
    out = _spawn(_worker_reduce, 2)
    assert out == {0: 2.5, 1: 2.5}
