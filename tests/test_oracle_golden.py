"""Pin the CPU oracle to the reference's own golden vectors (CPU only).

Every case of tests/golden/golden_cases.json (SHA-256 of the concatenated
recovery shards from /root/reference/src/test_util.rs:575-850, loss patterns
from the cited reference tests) is encoded by the oracle and hashed, then
decoded with the reference test's loss pattern and compared with the originals.
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as O

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden_cases.json")))
BIG = 20000


def _cases(big):
    out = []
    for c in GOLD["single"]:
        is_big = max(c["original_count"], c["recovery_count"]) > BIG
        if is_big == big:
            out.append(pytest.param(c, id=c["name"]))
    return out


def run_case(c):
    n, m, s = c["original_count"], c["recovery_count"], c["shard_bytes"]
    orig = O.generate_original(n, s, c["seed"])
    rec = O.encode(c["rate"], orig, m)
    assert hashlib.sha256(rec.tobytes()).hexdigest() == c["recovery_sha256"], c["source"]
    op = O.ranges_mask(c["decoder_original"], n)
    rp = O.ranges_mask(c["decoder_recovery"], m)
    if op.sum() + rp.sum() < n:
        return
    garbage = np.where(op[:, None] == 1, orig, 0xA5).astype(np.uint8)
    restored = O.decode(c["rate"], garbage, op, np.where(rp[:, None] == 1, rec, 0x5A).astype(np.uint8), rp)
    missing = op == 0
    assert np.array_equal(restored[missing], orig[missing]), c["source"]


@pytest.mark.parametrize("case", _cases(False))
def test_golden_small(case):
    run_case(case)


@pytest.mark.slow
@pytest.mark.parametrize("case", _cases(True))
def test_golden_large(case):
    run_case(case)


@pytest.mark.parametrize("seq", [pytest.param(s, id=s["name"]) for s in GOLD["two_rounds"]])
def test_two_round_hashes(seq):
    for r in seq["rounds"]:
        orig = O.generate_original(r["original_count"], r["shard_bytes"], r["seed"])
        rec = O.encode(seq["rate"], orig, r["recovery_count"])
        assert hashlib.sha256(rec.tobytes()).hexdigest() == r["recovery_sha256"]


def test_tables_invariants():
    exp = O.table("exp", 65536)
    log = O.table("log", 65536)
    assert log[0] == 65535
    nz = np.arange(1, 65536)
    assert np.array_equal(exp[log[nz]], nz)
    assert exp[65535] == exp[0] == 1


def test_zero_twiddles_are_the_skew_offset_0_top_layers():
    """The premise of the kernels' multiply-free top layers (RS_MONO_ZERO_TOP,
    rs_mono.hip run_seq zero_top): the skew table (tables.rs:285-324) holds
    GF_MODULUS (a zero twiddle) exactly at skew[2^b - 1], the single twiddle of
    layer b of a transform at skew offset 0; so an image-0 transform of 2^L rows
    has a zero-twiddle top layer and every offset n*t > 0 none."""
    skew = O.table("skew", 65535)
    zeros = np.flatnonzero(skew == 65535)
    assert zeros.tolist() == [(1 << b) - 1 for b in range(16)]
    for L in range(1, 16):
        n = 1 << L
        top = [(n >> 1) - 1 + t * n for t in range(65536 // n)]
        assert skew[top[0]] == 65535
        assert all(skew[i] != 65535 for i in top[1:])


def test_formal_derivative_closed_form():
    """utils.rs:99-104 equals out[q] = in[q] ^ XOR_{b: q_b=0, 2^b<n} in[q|2^b]."""
    rng = np.random.default_rng(1)
    for n in (1, 2, 4, 8, 64, 512):
        x = rng.integers(0, 256, (n, 64), dtype=np.uint8)
        y = x.copy()
        O.lib().orc_formal_derivative(O.ptr(y), 1, n)
        z = x.copy()
        for q in range(n):
            b = 1
            while b < n:
                if not q & b:
                    z[q] ^= x[q | b]
                b <<= 1
        assert np.array_equal(y, z)


def test_fft_inverts_ifft():
    rng = np.random.default_rng(2)
    for n, delta in ((16, 0), (256, 256), (1024, 7 * 1024)):
        x = rng.integers(0, 256, (n, 128), dtype=np.uint8)
        y = x.copy()
        O.lib().orc_ifft(O.ptr(y), 2, 0, n, n, delta)
        O.lib().orc_fft(O.ptr(y), 2, 0, n, n, delta)
        assert np.array_equal(x, y)


def test_use_high_rate():
    # rate_default.rs:437-462
    M = 2**64 - 1
    for n, m, want in ((0, 1, -1), (1, 0, -1), (3, 3, 1), (3, 4, 1), (3, 5, 0), (4, 3, 0), (5, 3, 1),
                       (4096, 61440, 0), (4096, 61441, -1), (4097, 61440, -1), (61440, 4096, 1),
                       (61440, 4097, -1), (61441, 4096, -1), (M, M, -1)):
        assert O.lib().orc_use_high_rate(n, m) == want, (n, m)


@pytest.fixture
def avx2_engine():
    if O.lib().orc_select_engine(1) != 0:
        pytest.skip("host CPU lacks AVX2")
    yield
    O.lib().orc_select_engine(0)


@pytest.mark.parametrize("case", _cases(False)[::3] + _cases(True))
def test_avx2_port_golden(case, avx2_engine):
    """The AVX2-restatement CPU baseline reproduces the reference hashes too."""
    run_case(case)


def test_oracle_under_address_and_ub_sanitizers():
    """oracle/Makefile `asan`: the oracle (both engines) built with -fsanitize=address,undefined
    runs encode -> erase -> decode round trips (every rate, tail sizes, multi-chunk shapes)
    without a sanitizer report and restores every lost shard."""
    import subprocess
    odir = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "oracle")
    subprocess.run(["make", "-s", "-C", odir, "asan"], check=True)
    r = subprocess.run([os.path.join(odir, "_build", "asan_check")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout
