"""GPU parity of the streaming pass kernel (rs_kernels.hip k_stream).

Large encodes run their transform passes as persistent 1024-thread workgroups
that load the next block's rows by LDS-DMA while the current block computes
(rs_stream_enable).  Here it is forced onto oracle-sized shapes (mode 2, column
kernel off) and compared with the CPU oracle bit-exactly -- every K from 3 to
8, slices wider than the rows (lanes outside the matrix read the zero line and
store to the junk line), row ranges of sources and destinations that are not
powers of two, and runs of blocks that cross sets -- and at full size (mode 1,
its default threshold) against the one-block-per-workgroup pass kernels.
"""
import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

RATE = {"default": 0, "high": 1, "low": 2}


@pytest.fixture(scope="module")
def torch():
    import torch as t
    if not t.cuda.is_available():
        pytest.skip("no GPU")
    return t


@pytest.fixture(scope="module")
def rs(torch):
    import reed_solomon_simd
    return reed_solomon_simd


def _encode(torch, rs, rate, orig, M):
    N, S = orig.shape
    d_orig = torch.from_numpy(np.ascontiguousarray(orig)).cuda()
    d_rec = torch.full((M, S), 0xEE, dtype=torch.uint8, device="cuda")
    rs.encode_device(N, M, S, d_orig, d_rec, rate_=RATE[rate])
    torch.cuda.synchronize()
    return d_rec.cpu().numpy()


# (rate, N, M, S): the passes each case runs (levels of <= 8 bits; SP = 2^(13 - K) packs)
STREAM_CASES = [
    ("high", 16, 16, 128),        # L = 4: one fused pass, K = 4 (no column kernel below 2^7)
    ("high", 200, 256, 192),      # L = 8: one fused K = 8 pass, which stays on k_pass (two table sets)
    ("high", 1024, 1024, 1024),   # L = 10: K = 5 + 5, 128 packs in 256-pack slices
    ("high", 3000, 3000, 2048),   # L = 12: K = 6 + 6, source / destination row ranges of 3000
    ("low", 700, 3000, 320),      # LowRate, n = 1024: K = 5 IFFT from the originals, FFT per chunk
    ("high", 4096, 4096, 512),    # L = 12, 64 packs
    ("default", 8192, 8192, 128), # L = 13: K = 7 + 6
    ("high", 32768, 32768, 64),   # L = 15: K = 8 + 7, 8 packs in 32-pack slices
    ("high", 20000, 30000, 64),   # L = 15 with partial row ranges
    ("high", 12000, 4000, 256),   # n = 4096, 3 chunks: multi-chunk IFFT passes stay on k_pass
]


@pytest.mark.parametrize("rate,N,M,S", STREAM_CASES)
def test_stream_pass_matches_oracle(torch, rs, rate, N, M, S):
    rs.mono_enable(0)
    rs.stream_enable(2)
    try:
        orig = O.generate_original(N, S, (N * 13 + M + S) & 0xFF)
        want = O.encode(rate, orig, M)
        got = _encode(torch, rs, rate, orig, M)
        assert np.array_equal(got, want)
        rs.check_device()
    finally:
        rs.stream_enable(1)
        rs.mono_enable(1)


def test_stream_pass_routes_where_expected(torch, rs):
    """Mode 2 runs k_stream for these passes (the profile's kernel names), mode 0 none."""
    N = M = 4096
    S = 512
    d_orig = torch.randint(0, 256, (N, S), dtype=torch.uint8, device="cuda")
    d_rec = torch.empty((M, S), dtype=torch.uint8, device="cuda")
    rs.mono_enable(0)
    try:
        names = {}
        for mode in (0, 2):
            rs.stream_enable(mode)
            rs.profile_enable(True)
            rs.encode_device(N, M, S, d_orig, d_rec, rate_=1)
            recs = rs.profile_collect()
            rs.profile_enable(False)
            names[mode] = [r[0] for r in recs]
        assert names[2] and all(n.startswith("k_stream") for n in names[2]), names[2]
        assert not any(n.startswith("k_stream") for n in names[0]), names[0]
    finally:
        rs.stream_enable(1)
        rs.mono_enable(1)


@pytest.mark.parametrize("N,M,S", [(8192, 8192, 65536), (32768, 32768, 16384)])
def test_stream_default_matches_pass_kernels_full_size(torch, rs, N, M, S):
    """BASELINE config 4's encode (k_stream at its default threshold: K = 7 and 6, 8192 blocks each)
    and a 32768:32768 stripe, bit-exact against the one-block-per-workgroup pass kernels; then the
    encode -> erase -> decode round trip of 1 % of the originals."""
    g = torch.Generator(device="cuda")
    g.manual_seed(N + S)
    d_orig = torch.randint(0, 256, (N, S), dtype=torch.uint8, device="cuda", generator=g)
    out = {}
    for mode in (0, 1):
        rs.stream_enable(mode)
        d_rec = torch.empty((M, S), dtype=torch.uint8, device="cuda")
        rs.encode_device(N, M, S, d_orig, d_rec, rate_=1)
        torch.cuda.synchronize()
        out[mode] = d_rec
    rs.stream_enable(1)
    assert torch.equal(out[0], out[1])
    del out[0]
    rng = np.random.default_rng(N)
    L = max(1, N // 100)
    op = np.ones(N, np.uint8)
    op[rng.choice(N, L, replace=False)] = 0
    rp = np.zeros(M, np.uint8)
    rp[:L] = 1
    miss = torch.from_numpy(op == 0).cuda()
    d_in = d_orig.clone()
    d_in[miss] = 0
    d_out = torch.zeros_like(d_orig)
    rs.decode_device(N, M, S, d_in, op, out[1], rp, d_out, rate_=1)
    torch.cuda.synchronize()
    assert torch.equal(d_out[miss], d_orig[miss])
    rs.check_device()
