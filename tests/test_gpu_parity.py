"""GPU parity: the HIP path (through the C ABI) against the CPU oracle.

Bit-exact comparisons at oracle-sized configurations, the reference's golden
SHA-256 vectors through the drop-in API, the reference's error semantics, and
size-independent properties at BASELINE.json's full sizes (encode -> erase ->
decode round trips, and column-sampled comparisons: every engine op is
column-wise, so encoding 64-byte column blocks of a large shard matrix on the
CPU must reproduce the same columns of the GPU result).
"""
import hashlib
import json
import os

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

GOLD = json.load(open(os.path.join(os.path.dirname(__file__), "golden", "golden_cases.json")))
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


def _dev(torch, a):
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def assert_rows_equal(got, want, what="rows"):
    """Byte-exact comparison that names the first differing (row, byte), the number of
    differing bytes and rows, and the first differing rows' indices -- enough to tell a
    whole-table race (many rows of one column) from a single corrupted row."""
    got = np.asarray(got)
    want = np.asarray(want)
    assert got.shape == want.shape, f"{what}: shape {got.shape} != {want.shape}"
    diff = got != want
    if not diff.any():
        return
    rows = np.flatnonzero(diff.reshape(diff.shape[0], -1).any(axis=1))
    r0 = int(rows[0])
    b0 = int(np.flatnonzero(diff[r0].reshape(-1))[0])
    cols = np.flatnonzero(diff.reshape(diff.shape[0], -1).any(axis=0))
    raise AssertionError(
        f"{what}: {int(diff.sum())} of {diff.size} bytes differ in {rows.size} of {diff.shape[0]} rows; "
        f"first at (row {r0}, byte {b0}): got {int(got.reshape(got.shape[0], -1)[r0, b0])} want "
        f"{int(want.reshape(want.shape[0], -1)[r0, b0])}; rows {rows[:16].tolist()}; byte columns {cols[:16].tolist()}"
        f"{' ...' if cols.size > 16 else ''}")


def gpu_encode(torch, rs, rate, orig, M):
    N, S = orig.shape
    d_orig = _dev(torch, orig)
    d_rec = torch.full((M, S), 0xEE, dtype=torch.uint8, device="cuda")
    rs.encode_device(N, M, S, d_orig, d_rec, rate_=RATE[rate])
    torch.cuda.synchronize()
    return d_rec.cpu().numpy()


def gpu_decode(torch, rs, rate, orig, op, rec, rp):
    N, S = orig.shape
    M = rec.shape[0]
    d_o = _dev(torch, np.where(op[:, None] == 1, orig, 0xA5).astype(np.uint8))
    d_r = _dev(torch, np.where(rp[:, None] == 1, rec, 0x5A).astype(np.uint8))
    d_out = torch.full((N, S), 0x33, dtype=torch.uint8, device="cuda")
    rs.decode_device(N, M, S, d_o, op, d_r, rp, d_out, rate_=RATE[rate])
    torch.cuda.synchronize()
    return d_out.cpu().numpy()


# ---------------------------------------------------------------------------
# device-resident path vs oracle, bit-exact

ENC_CASES = [
    # (rate, N, M, S) -- single-pass (n <= 256), multi-pass (n > 256), multi-chunk
    ("default", 1, 1, 64), ("default", 3, 5, 64), ("high", 5, 3, 128), ("low", 3, 5, 128),
    ("default", 64, 64, 1024), ("default", 100, 37, 192), ("default", 37, 100, 320),
    ("high", 1000, 100, 128), ("low", 100, 1000, 128), ("default", 1024, 1024, 1024),
    ("default", 1000, 1000, 576), ("high", 3000, 700, 64), ("low", 700, 3000, 64),
    ("default", 5000, 300, 256), ("default", 300, 5000, 256), ("default", 4096, 4096, 512),
    ("default", 10000, 1000, 128), ("high", 32768, 32768, 64), ("low", 32768, 32768, 64),
    ("high", 61440, 4096, 64), ("low", 4096, 61440, 64),
]


@pytest.mark.parametrize("rate,N,M,S", ENC_CASES)
def test_encode_device_matches_oracle(torch, rs, rate, N, M, S):
    orig = O.generate_original(N, S, (N * 31 + M) & 0xFF)
    want = O.encode(rate, orig, M)
    got = gpu_encode(torch, rs, rate, orig, M)
    assert_rows_equal(got, want)


# Single-level multi-chunk encodes in both forms (rs_codec.cpp chunk_parallel): chunks one
# after another in one workgroup (RS_MI355X_CHUNK_PARALLEL=0) and chunks over the grid
# (=1: HighRate per-chunk IFFT passes + an XOR-fold FFT pass; LowRate one IFFT + FFT per
# output chunk); the environment is read when a context is created.
CHUNK_CASES = [("high", 1000, 100, 128), ("low", 100, 1000, 128), ("high", 5000, 300, 256),
               ("low", 300, 5000, 256), ("high", 129, 1, 64), ("low", 1, 129, 64), ("high", 1000, 64, 8192),
               ("low", 64, 1000, 8192), ("high", 3000, 200, 130), ("low", 200, 3000, 130)]


@pytest.mark.parametrize("forced", ["0", "1"])
def test_chunk_forms_match_oracle(torch, rs, forced, monkeypatch):
    monkeypatch.setenv("RS_MI355X_CHUNK_PARALLEL", forced)
    ctx = rs.Context(0)
    try:
        for rate, N, M, S in CHUNK_CASES:
            orig = O.generate_original(N, S, (N * 13 + M + S) & 0xFF)
            want = O.encode(rate, orig, M)
            d_orig = _dev(torch, orig)
            d_rec = torch.full((M, S), 0xEE, dtype=torch.uint8, device="cuda")
            rs.encode_device(N, M, S, d_orig, d_rec, rate_=RATE[rate], ctx=ctx)
            torch.cuda.synchronize()
            assert_rows_equal(d_rec.cpu().numpy(), want, str((forced, rate, N, M, S)))
    finally:
        ctx.close()


DEC_CASES = [
    ("default", 3, 5, 64, 0.5), ("high", 5, 3, 128, 0.5), ("low", 3, 5, 128, 1.0), ("default", 64, 64, 1024, 0.3),
    ("default", 100, 37, 192, 0.2), ("default", 37, 100, 320, 1.0), ("default", 1024, 1024, 1024, 0.01),
    ("default", 1024, 1024, 1024, 1.0), ("high", 1000, 100, 128, 0.1), ("low", 100, 1000, 128, 0.9),
    ("default", 3000, 700, 64, 0.2), ("low", 700, 3000, 64, 0.5), ("default", 4096, 4096, 512, 0.5),
    ("high", 32768, 32768, 64, 1.0), ("low", 32768, 32768, 64, 0.3), ("high", 61440, 4096, 64, 0.05),
]


@pytest.mark.parametrize("rate,N,M,S,loss", DEC_CASES)
def test_decode_device_matches_oracle(torch, rs, rate, N, M, S, loss):
    rng = np.random.default_rng(N + 3 * M)
    orig = O.generate_original(N, S, 5)
    rec = O.encode(rate, orig, M)
    L = max(1, int(round(min(N, M) * loss)))
    op = np.ones(N, np.uint8)
    op[rng.choice(N, L, replace=False)] = 0
    rp = np.zeros(M, np.uint8)
    rp[rng.choice(M, L, replace=False)] = 1
    want = O.decode(rate, orig, op, rec, rp)
    got = gpu_decode(torch, rs, rate, orig, op, rec, rp)
    miss = op == 0
    assert_rows_equal(got[miss], orig[miss])
    assert_rows_equal(got[miss], want[miss])
    assert np.all(got[~miss] == 0x33), "present rows of the output must not be written"


# eval_poly forms by work rows 2^u (rs_eval.hip): one workgroup (k_eval_fast, value-major LDS
# rounds) at u = 11..13 on the pass-kernel route, three launches (k_walsh_part) at u >= 14;
# both rates, LowRate with end < 2^u.  (rate, N, M): u
# (2^11 rows take the pass kernels only past the column kernel's 256 packs: 4 KiB shards)
EVAL_DEC = [("high", 1500, 20, 11, 4096), ("low", 20, 3000, 12, 64), ("high", 2048, 2048, 12, 64),
            ("low", 2000, 6000, 13, 64), ("high", 4096, 4096, 13, 64), ("high", 6000, 1500, 13, 64),
            ("high", 5000, 3000, 14, 64), ("low", 3000, 9000, 14, 64)]


@pytest.mark.parametrize("rate,N,M,u,S", EVAL_DEC)
def test_eval_poly_forms_match_oracle(torch, rs, rate, N, M, u, S):
    chunk = 1 << ((M if rate == "high" else N) - 1).bit_length()
    end = chunk + (N if rate == "high" else M)
    assert (1 << (end - 1).bit_length()) == 1 << u
    rng = np.random.default_rng(u * 1000 + N)
    orig = O.generate_original(N, S, u)
    rec = O.encode(rate, orig, M)
    L = max(1, min(N, M) // 3)
    op = np.ones(N, np.uint8)
    op[rng.choice(N, L, replace=False)] = 0
    rp = np.zeros(M, np.uint8)
    rp[rng.choice(M, L, replace=False)] = 1
    want = O.decode(rate, orig, op, rec, rp)
    got = gpu_decode(torch, rs, rate, orig, op, rec, rp)
    miss = op == 0
    assert np.array_equal(got[miss], orig[miss]) and np.array_equal(got[miss], want[miss])


# decodes of at most 64 work rows, one launch: 16..64 rows of shards up to 2 KiB on the
# column kernel's 2^7-row transform (padded work rows), the others one pass that
# evaluates eval_poly itself (rs_kernels.hip pass_eval_poly); (rate, N, M): work rows
# 2..64, both rates, the LowRate end < n and the HighRate recovery padding
SMALL_DEC = [("high", 1, 1), ("low", 1, 1), ("high", 3, 5), ("low", 5, 3), ("high", 2, 30), ("low", 30, 2),
             ("high", 32, 32), ("low", 32, 32), ("high", 31, 17), ("low", 17, 31), ("high", 40, 16),
             ("low", 16, 40), ("high", 1, 32), ("low", 32, 1)]


def _work_rows(rate, N, M):
    chunk = 1 << max(0, ((M if rate == "high" else N) - 1).bit_length())
    end = chunk + (N if rate == "high" else M)
    return 1 << (end - 1).bit_length()


@pytest.mark.parametrize("rate,N,M", SMALL_DEC)
@pytest.mark.parametrize("S", [64, 1024, 130, 4096])
def test_small_decode_is_one_fused_launch(torch, rs, rate, N, M, S):
    assert _work_rows(rate, N, M) <= 64
    rng = np.random.default_rng(N * 97 + M + S)
    orig = O.generate_original(N, S, (N + M + S) & 0xFF)
    rec = O.encode(rate, orig, M)
    for trial in range(3):
        L = int(rng.integers(1, min(N, M) + 1))
        op = np.ones(N, np.uint8)
        op[rng.choice(N, L, replace=False)] = 0
        rp = np.zeros(M, np.uint8)
        rp[rng.choice(M, L, replace=False)] = 1
        want = O.decode(rate, orig, op, rec, rp)
        rs.profile_enable(True)
        try:
            got = gpu_decode(torch, rs, rate, orig, op, rec, rp)
            names = [r[0] for r in rs.profile_collect()]
        finally:
            rs.profile_enable(False)
        miss = op == 0
        assert np.array_equal(got[miss], orig[miss]) and np.array_equal(got[miss], want[miss]), (trial, L)
        assert len(names) == 1, names
        if _work_rows(rate, N, M) >= 16 and S <= 2048:
            assert names[0].startswith("k_mono<7, "), names
        else:
            assert names[0].startswith("k_pass<") and names[0].endswith(", 435>"), names


# ---------------------------------------------------------------------------
# the reference's golden vectors through the drop-in object API

def _run_golden(rs, c):
    n, m, s = c["original_count"], c["recovery_count"], c["shard_bytes"]
    orig = O.generate_original(n, s, c["seed"])
    cls = {"default": rs.rate.DefaultRateEncoder, "high": rs.rate.HighRateEncoder,
           "low": rs.rate.LowRateEncoder}[c["rate"]]
    dcls = {"default": rs.rate.DefaultRateDecoder, "high": rs.rate.HighRateDecoder,
            "low": rs.rate.LowRateDecoder}[c["rate"]]
    enc = cls(n, m, s)
    for row in orig:
        enc.add_original_shard(row.tobytes())
    res = enc.encode()
    rec = list(res.recovery_iter())
    assert hashlib.sha256(b"".join(rec)).hexdigest() == c["recovery_sha256"], c["source"]
    dec = dcls(n, m, s)
    got = np.zeros(n, bool)
    for a, b in c["decoder_original"]:
        for i in range(a, b):
            dec.add_original_shard(i, orig[i].tobytes())
            got[i] = True
    for a, b in c["decoder_recovery"]:
        for i in range(a, b):
            dec.add_recovery_shard(i, rec[i])
    r = dec.decode()
    restored = dict(r.restored_original_iter())
    for i in np.where(~got)[0]:
        assert restored[int(i)] == orig[i].tobytes(), (c["source"], int(i))


@pytest.mark.parametrize("case", [pytest.param(c, id=c["name"]) for c in GOLD["single"]])
def test_golden_vectors_object_api(rs, case):
    _run_golden(rs, case)


@pytest.mark.parametrize("seq", [pytest.param(s, id=s["name"]) for s in GOLD["two_rounds"]])
def test_two_rounds(rs, seq):
    """roundtrip_two_rounds! (test_util.rs:211-364): work re-use with implicit or explicit reset."""
    enc_cls = {"default": rs.rate.DefaultRateEncoder, "high": rs.rate.HighRateEncoder,
               "low": rs.rate.LowRateEncoder}[seq["rate"]]
    dec_cls = {"default": rs.rate.DefaultRateDecoder, "high": rs.rate.HighRateDecoder,
               "low": rs.rate.LowRateDecoder}[seq["rate"]]
    r0 = seq["rounds"][0]
    enc = enc_cls(r0["original_count"], r0["recovery_count"], r0["shard_bytes"])
    dec = dec_cls(r0["original_count"], r0["recovery_count"], r0["shard_bytes"])
    for k, r in enumerate(seq["rounds"]):
        if k and seq["explicit_reset"]:
            enc.reset(r["original_count"], r["recovery_count"], r["shard_bytes"])
            dec.reset(r["original_count"], r["recovery_count"], r["shard_bytes"])
        orig = O.generate_original(r["original_count"], r["shard_bytes"], r["seed"])
        for row in orig:
            enc.add_original_shard(row.tobytes())
        res = enc.encode()
        rec = list(res.recovery_iter())
        res.drop()
        assert hashlib.sha256(b"".join(rec)).hexdigest() == r["recovery_sha256"]
        have = set()
        for a, b in r["decoder_original"]:
            for i in range(a, b):
                dec.add_original_shard(i, orig[i].tobytes())
                have.add(i)
        for a, b in r["decoder_recovery"]:
            for i in range(a, b):
                dec.add_recovery_shard(i, rec[i])
        out = dec.decode()
        for i in range(r["original_count"]):
            if i not in have:
                assert out.restored_original(i) == orig[i].tobytes()
        out.drop()


def test_readme_example(rs):
    """README.md:87-115: 3 original x 64 B, 5 recovery; restore #0 and #2."""
    original = [b"Lorem ipsum dolor sit amet, consectetur adipiscing elit, sed do ",
                b"eiusmod tempor incididunt ut labore et dolore magna aliqua. Ut e",
                b"nim ad minim veniam, quis nostrud exercitation ullamco laboris n"]
    recovery = rs.encode(3, 5, original)
    want = O.encode("default", np.frombuffer(b"".join(original), np.uint8).reshape(3, 64), 5)
    assert b"".join(recovery) == want.tobytes()
    restored = rs.decode(3, 5, [(1, original[1])], [(1, recovery[1]), (4, recovery[4])])
    assert restored == {0: original[0], 2: original[2]}


@pytest.mark.parametrize("S", [2, 4, 6, 30, 32, 34, 62, 64, 66, 126, 128, 130])
def test_shard_size_not_divisible_by_64(rs, S):
    """decoder_result.rs:166-171 sizes; tail re-pack (shards.rs:38-74) vs the oracle."""
    orig = O.generate_original(3, S, 0)
    want = O.encode("default", orig, 2)
    enc = rs.ReedSolomonEncoder(3, 2, S)
    for row in orig:
        enc.add_original_shard(row.tobytes())
    res = enc.encode()
    rec = list(res.recovery_iter())
    assert b"".join(rec) == want.tobytes()
    dec = rs.ReedSolomonDecoder(3, 2, S)
    dec.add_original_shard(1, orig[1].tobytes())
    dec.add_recovery_shard(0, rec[0])
    dec.add_recovery_shard(1, rec[1])
    out = dec.decode()
    assert out.restored_original(0) == orig[0].tobytes()
    assert out.restored_original(1) is None
    assert out.restored_original(2) == orig[2].tobytes()
    assert out.restored_original(3) is None
    assert list(out.restored_original_iter()) == [(0, orig[0].tobytes()), (2, orig[2].tobytes())]


# ---------------------------------------------------------------------------
# error semantics (test_util.rs:369-573, lib.rs:420-617)

@pytest.mark.parametrize("which", ["default", "high", "low"])
def test_encoder_errors(rs, which):
    E = {"default": rs.rate.DefaultRateEncoder, "high": rs.rate.HighRateEncoder, "low": rs.rate.LowRateEncoder}[which]
    enc = E(1, 1, 64)
    with pytest.raises(rs.DifferentShardSize) as e:
        enc.add_original_shard(bytes(128))
    assert e.value == rs.DifferentShardSize(shard_bytes=64, got=128)
    with pytest.raises(rs.InvalidShardSize) as e:
        E(1, 1, 123)
    assert e.value == rs.InvalidShardSize(shard_bytes=123)
    with pytest.raises(rs.InvalidShardSize):
        E(1, 1, 64).reset(1, 1, 123)
    with pytest.raises(rs.TooFewOriginalShards) as e:
        E(1, 1, 64).encode()
    assert e.value == rs.TooFewOriginalShards(original_count=1, original_received_count=0)
    enc = E(1, 1, 64)
    enc.add_original_shard(bytes(64))
    with pytest.raises(rs.TooManyOriginalShards) as e:
        enc.add_original_shard(bytes(64))
    assert e.value == rs.TooManyOriginalShards(original_count=1)
    with pytest.raises(rs.UnsupportedShardCount) as e:
        E(0, 1, 64)
    assert e.value == rs.UnsupportedShardCount(original_count=0, recovery_count=1)
    with pytest.raises(rs.UnsupportedShardCount):
        E(1, 1, 64).reset(0, 1, 64)


@pytest.mark.parametrize("which", ["default", "high", "low"])
def test_decoder_errors(rs, which):
    D = {"default": rs.rate.DefaultRateDecoder, "high": rs.rate.HighRateDecoder, "low": rs.rate.LowRateDecoder}[which]
    with pytest.raises(rs.DifferentShardSize) as e:
        D(1, 1, 64).add_original_shard(0, bytes(128))
    assert e.value == rs.DifferentShardSize(shard_bytes=64, got=128)
    with pytest.raises(rs.DifferentShardSize):
        D(1, 1, 64).add_recovery_shard(0, bytes(128))
    d = D(1, 1, 64)
    d.add_original_shard(0, bytes(64))
    with pytest.raises(rs.DuplicateOriginalShardIndex) as e:
        d.add_original_shard(0, bytes(64))
    assert e.value == rs.DuplicateOriginalShardIndex(index=0)
    d = D(1, 1, 64)
    d.add_recovery_shard(0, bytes(64))
    with pytest.raises(rs.DuplicateRecoveryShardIndex) as e:
        d.add_recovery_shard(0, bytes(64))
    assert e.value == rs.DuplicateRecoveryShardIndex(index=0)
    with pytest.raises(rs.InvalidOriginalShardIndex) as e:
        D(1, 1, 64).add_original_shard(1, bytes(64))
    assert e.value == rs.InvalidOriginalShardIndex(original_count=1, index=1)
    with pytest.raises(rs.InvalidRecoveryShardIndex) as e:
        D(1, 1, 64).add_recovery_shard(1, bytes(64))
    assert e.value == rs.InvalidRecoveryShardIndex(recovery_count=1, index=1)
    with pytest.raises(rs.InvalidShardSize):
        D(1, 1, 123)
    with pytest.raises(rs.InvalidShardSize):
        D(1, 1, 64).reset(1, 1, 123)
    with pytest.raises(rs.NotEnoughShards) as e:
        D(1, 1, 64).decode()
    assert e.value == rs.NotEnoughShards(original_count=1, original_received_count=0, recovery_received_count=0)
    with pytest.raises(rs.UnsupportedShardCount):
        D(0, 1, 64)
    with pytest.raises(rs.UnsupportedShardCount):
        D(1, 1, 64).reset(0, 1, 64)


def test_oneshot_errors(rs):
    with pytest.raises(rs.DifferentShardSize) as e:
        rs.encode(2, 1, [bytes(64), bytes(128)])
    assert e.value == rs.DifferentShardSize(shard_bytes=64, got=128)
    with pytest.raises(rs.InvalidShardSize):
        rs.encode(1, 1, [b""])
    with pytest.raises(rs.TooFewOriginalShards) as e:
        rs.encode(1, 1, [])
    assert e.value == rs.TooFewOriginalShards(original_count=1, original_received_count=0)
    with pytest.raises(rs.TooManyOriginalShards):
        rs.encode(1, 1, [bytes(64), bytes(64)])
    with pytest.raises(rs.UnsupportedShardCount):
        rs.encode(0, 1, [])
    with pytest.raises(rs.UnsupportedShardCount):
        rs.encode(1, 0, [bytes(64)])
    assert rs.decode(1, 1, [(0, bytes(64))], []) == {}
    with pytest.raises(rs.DifferentShardSize):
        rs.decode(2, 1, [(0, bytes(64)), (1, bytes(128))], [(0, bytes(64))])
    with pytest.raises(rs.DifferentShardSize):
        rs.decode(1, 2, [(0, bytes(64))], [(0, bytes(64)), (1, bytes(128))])
    with pytest.raises(rs.DifferentShardSize) as e:
        rs.decode(1, 1, [(0, b"")], [(0, bytes(64))])
    assert e.value == rs.DifferentShardSize(shard_bytes=64, got=0)
    with pytest.raises(rs.DuplicateOriginalShardIndex):
        rs.decode(2, 1, [(0, bytes(64)), (0, bytes(64))], [(0, bytes(64))])
    with pytest.raises(rs.DuplicateRecoveryShardIndex):
        rs.decode(1, 2, [(0, bytes(64))], [(0, bytes(64)), (0, bytes(64))])
    with pytest.raises(rs.InvalidOriginalShardIndex):
        rs.decode(1, 1, [(1, bytes(64))], [(0, bytes(64))])
    with pytest.raises(rs.InvalidRecoveryShardIndex):
        rs.decode(1, 1, [(0, bytes(64))], [(1, bytes(64))])
    with pytest.raises(rs.InvalidShardSize):
        rs.decode(1, 1, [(0, bytes(64))], [(0, b"")])
    with pytest.raises(rs.NotEnoughShards):
        rs.decode(1, 1, [], [])
    with pytest.raises(rs.UnsupportedShardCount):
        rs.decode(0, 1, [], [])
    with pytest.raises(rs.UnsupportedShardCount):
        rs.decode(1, 0, [], [])


def test_encoder_result_and_size(rs):
    """encoder_result.rs:122-172"""
    orig = O.generate_original(2, 1024, 123)
    enc = rs.ReedSolomonEncoder(2, 3, 1024)
    for row in orig:
        enc.add_original_shard(row.tobytes())
    res = enc.encode()
    allr = [res.recovery(0), res.recovery(1), res.recovery(2)]
    assert res.recovery(3) is None
    assert hashlib.sha256(b"".join(allr)).hexdigest() == [c for c in GOLD["single"] if c["name"] == "lib_roundtrip"][0][
        "recovery_sha256"]


def test_decoder_no_missing(rs):
    """decoder_result.rs:209-238: all originals given -> empty result."""
    orig = O.generate_original(3, 64, 0)
    dec = rs.ReedSolomonDecoder(3, 2, 64)
    for i in range(3):
        dec.add_original_shard(i, orig[i].tobytes())
    out = dec.decode()
    assert len(out) == 0 and list(out.restored_original_iter()) == []


# ---------------------------------------------------------------------------
# Engine trait over device rows (src/engine.rs:234-291) vs the oracle

@pytest.mark.parametrize("size,pos,delta,trunc,blocks", [(1, 0, 0, 1, 1), (2, 0, 5, 2, 2), (16, 3, 0, 16, 1),
                                                         (256, 0, 256, 200, 3), (1024, 2, 1024, 1024, 2),
                                                         (4096, 0, 4096, 4096, 1), (32768, 0, 0, 32768, 1),
                                                         (64, 1, 0, 37, 1), (2048, 0, 2048, 1000, 2),
                                                         (8, 0, 8, 0, 1)])
@pytest.mark.parametrize("which", ["fft", "ifft"])
def test_engine_transforms(torch, rs, size, pos, delta, trunc, blocks, which):
    """Every row equals engine_naive.rs:43-105 -- including the rows at and past truncated_size,
    where only the groups that start below it were transformed, with arbitrary (non-zero) data
    there."""
    rng = np.random.default_rng(size + pos + trunc)
    rows = pos + size + 1
    x = rng.integers(0, 256, (rows, blocks * 64), dtype=np.uint8)
    want = x.copy()
    getattr(O.lib(), f"orc_{which}")(O.ptr(want), blocks, pos, size, trunc, delta)
    d = _dev(torch, x)
    getattr(rs.engine, which)(d, rows, blocks, pos, size, trunc, delta)
    torch.cuda.synchronize()
    got = d.cpu().numpy()
    assert_rows_equal(got, want)


def test_engine_mul_and_formal_derivative(torch, rs):
    rng = np.random.default_rng(11)
    x = rng.integers(0, 256, (5, 128), dtype=np.uint8)
    for lm in (0, 1, 777, 65534, 65535):
        want = x.copy()
        O.lib().orc_mul(O.ptr(want), 10, lm)
        d = _dev(torch, x)
        rs.engine.mul(d, 10, lm)
        torch.cuda.synchronize()
        assert_rows_equal(d.cpu().numpy(), want)
    # utils.rs:99-104 is defined for power-of-two row counts only (it slices past
    # the end otherwise); the device API rejects other counts
    for n in (1, 2, 64, 1024):
        x = rng.integers(0, 256, (n, 64), dtype=np.uint8)
        want = x.copy()
        O.lib().orc_formal_derivative(O.ptr(want), 1, n)
        d = _dev(torch, x)
        rs.engine.formal_derivative(d, n, 1)
        torch.cuda.synchronize()
        assert_rows_equal(d.cpu().numpy(), want)
    with pytest.raises(ValueError):
        rs.engine.formal_derivative(_dev(torch, np.zeros((3, 64), np.uint8)), 3, 1)


@pytest.mark.parametrize("which", ["fft", "ifft"])
def test_engine_host_slices_match_oracle(torch, rs, which):
    """rs_engine_{fft,ifft,mul}_host: the Engine trait on a host ShardsRefMut-style array (what the
    Rust `impl Engine` of INTEGRATION.md binds) -- rows outside [pos, pos + size) untouched."""
    rng = np.random.default_rng(77)
    for size, pos, trunc, delta, blocks in ((1024, 3, 1024, 1024, 2), (256, 0, 100, 0, 1), (4, 1, 4, 60000, 3)):
        rows = pos + size + 2
        x = rng.integers(0, 256, (rows, blocks * 64), dtype=np.uint8)
        want = x.copy()
        getattr(O.lib(), f"orc_{which}")(O.ptr(want), blocks, pos, size, trunc, delta)
        got = x.copy()
        getattr(rs.engine, f"{which}_host")(got, rows, blocks, pos, size, trunc, delta)
        assert_rows_equal(got, want, str((size, pos, trunc, delta)))
    x = rng.integers(0, 256, (7, 64), dtype=np.uint8)
    for lm in (0, 12345, 65535):
        want = x.copy()
        O.lib().orc_mul(O.ptr(want), 7, lm)
        got = x.copy()
        rs.engine.mul_host(got, 7, lm)
        assert_rows_equal(got, want)


# ---------------------------------------------------------------------------
# per-stream device scratch (rs_mi355x.h "Thread-safety"): capped per context

def test_stream_scratch_is_capped_and_released(torch, rs):
    """Pass-kernel encodes (which need work buffers) on more streams than the context
    keeps scratch for (RS_MAX_STREAM_WORKSPACES = 16): every result equals the oracle,
    the least recently used stream's scratch is evicted behind a device synchronize, and
    release_stream_scratch frees one stream's scratch on demand."""
    N, M, S = 4096, 4096, 256
    origs = [O.generate_original(N, S, 90 + k) for k in range(2)]
    wants = [O.encode("high", o, M) for o in origs]
    d_o = [_dev(torch, o) for o in origs]
    streams = [torch.cuda.Stream() for _ in range(20)]
    outs = [torch.empty((M, S), dtype=torch.uint8, device="cuda") for _ in streams]
    torch.cuda.synchronize()
    for rep in range(2):
        for k, st in enumerate(streams):
            st.wait_stream(torch.cuda.current_stream())
            rs.encode_device(N, M, S, d_o[(k + rep) & 1], outs[k], rate_=rs.RATE_HIGH, stream=st)
        torch.cuda.synchronize()
        for k, o in enumerate(outs):
            assert_rows_equal(o.cpu().numpy(), wants[(k + rep) & 1], str((rep, k)))
    for st in streams:
        rs.release_stream_scratch(st)
    rs.release_stream_scratch(streams[0])  # already released: no-op
    rs.check_device()


def test_work_moves_between_contexts(torch, rs):
    """EncoderWork / DecoderWork handed to a second context: the work records
    its context's device; on the same device its buffers are reused, and the results of
    both contexts equal the oracle."""
    ctx2 = rs.Context(0)
    try:
        orig = O.generate_original(300, 1024, 5)
        want = O.encode("high", orig, 200)
        enc = rs.rate.HighRateEncoder(300, 200, 1024)
        for row in orig:
            enc.add_original_shard(row.tobytes())
        assert b"".join(enc.encode().recovery_iter()) == want.tobytes()
        _, work = enc.into_parts()
        enc2 = rs.rate.HighRateEncoder(300, 200, 1024, ctx=ctx2, work=work)
        for row in orig:
            enc2.add_original_shard(row.tobytes())
        assert b"".join(enc2.encode().recovery_iter()) == want.tobytes()
        dec = rs.rate.HighRateDecoder(300, 200, 1024, ctx=ctx2)
        for i in range(100, 300):
            dec.add_original_shard(i, orig[i].tobytes())
        for i in range(100):
            dec.add_recovery_shard(i, want[i].tobytes())
        assert all(v == orig[i].tobytes() for i, v in dec.decode().restored_original_iter())
        _, dwork = dec.into_parts()
        dec2 = rs.rate.HighRateDecoder(300, 200, 1024, work=dwork)
        for i in range(100, 300):
            dec2.add_original_shard(i, orig[i].tobytes())
        for i in range(100):
            dec2.add_recovery_shard(i, want[i].tobytes())
        got = dict(dec2.decode().restored_original_iter())
        assert sorted(got) == list(range(100)) and all(got[i] == orig[i].tobytes() for i in got)
        del enc2, dec2
    finally:
        ctx2.close()


def test_two_streams_share_one_context(torch, rs):
    """Device scratch is per (context, stream): encodes and decodes that need scratch (pass
    kernels, 4096-row transforms) alternate between two streams of one context without a
    synchronisation in between; both streams' results equal the oracle."""
    N, M, S = 4096, 4096, 512
    rate = "high"
    origs = [O.generate_original(N, S, 60 + k) for k in range(2)]
    wants = [O.encode(rate, o, M) for o in origs]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    d_o = [_dev(torch, o) for o in origs]
    d_r = [torch.zeros((M, S), dtype=torch.uint8, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    for _ in range(6):
        for k in range(2):
            rs.encode_device(N, M, S, d_o[k], d_r[k], stream=streams[k], rate_=RATE[rate])
    torch.cuda.synchronize()
    for k in range(2):
        assert_rows_equal(d_r[k].cpu().numpy(), wants[k], f"stream {k}")
    rng = np.random.default_rng(5)
    L = 1500
    op = np.ones(N, np.uint8)
    op[rng.choice(N, L, replace=False)] = 0
    rp = np.zeros(M, np.uint8)
    rp[rng.choice(M, L, replace=False)] = 1
    outs = [torch.full((N, S), 0x33, dtype=torch.uint8, device="cuda") for _ in range(2)]
    ins = [_dev(torch, np.where(op[:, None] == 1, o, 0).astype(np.uint8)) for o in origs]
    for _ in range(4):
        for k in range(2):
            rs.decode_device(N, M, S, ins[k], op, d_r[k], rp, outs[k], stream=streams[k], rate_=RATE[rate])
    torch.cuda.synchronize()
    miss = op == 0
    for k in range(2):
        assert_rows_equal(outs[k].cpu().numpy()[miss], origs[k][miss], f"stream {k}")


def test_device_arguments_are_checked(torch, rs):
    """Undersized / wrong-dtype / host tensors and wrong-length masks are rejected before any
    kernel runs (the reference rejects wrong sizes with DifferentShardSize)."""
    d = torch.zeros((64, 128), dtype=torch.uint8, device="cuda")
    with pytest.raises(ValueError):
        rs.encode_device(64, 64, 256, d, d)  # rows of 128 bytes, shard_bytes 256
    with pytest.raises(ValueError):
        rs.encode_device(65, 64, 128, d, d)  # 64 rows for 65 originals
    with pytest.raises(ValueError):
        rs.encode_device(64, 64, 128, d.to(torch.int16), d)
    with pytest.raises(ValueError):
        rs.encode_device(64, 64, 128, d.cpu(), d)
    with pytest.raises(ValueError):
        rs.decode_device(64, 64, 128, d, [1] * 63, d, [0] * 64, d)  # mask too short
    with pytest.raises(ValueError):
        rs.encode_device_call(64, 64, 128, d, d[:10])


# ---------------------------------------------------------------------------
# BASELINE.json configurations at full size: properties + column samples

def _column_sample_check(orig, got, M, rate, blocks=(0, 7, -1)):
    S = orig.shape[1]
    nb = S // 64
    for b in blocks:
        b %= nb
        cols = slice(64 * b, 64 * b + 64)
        want = O.encode(rate, np.ascontiguousarray(orig[:, cols]), M)
        assert_rows_equal(got[:, cols], want, f"column block {b}")


@pytest.mark.parametrize("N,M,S", [(1024, 1024, 1024), (32768, 32768, 1024)])
def test_baseline_encode_configs(torch, rs, N, M, S):
    orig = O.generate_original(N, S, 0)
    got = gpu_encode(torch, rs, "default", orig, M)
    _column_sample_check(orig, got, M, "default")
    if N * S <= (64 << 20):
        O.lib().orc_select_engine(1)
        try:
            assert_rows_equal(got, O.encode("default", orig, M))
        finally:
            O.lib().orc_select_engine(0)


def _sampled_blocks_match(torch, d_orig, d_rec, M, blocks):
    """The 64-byte column blocks `blocks` of a device encode equal the oracle's encode of
    the same blocks (every engine op is column-wise: a 64-B-shard encode of one block is
    that block of the full encode).  One oracle call (AVX2 restatement) for all blocks."""
    cols = np.concatenate([np.arange(64 * b, 64 * b + 64) for b in blocks])
    idx = torch.from_numpy(cols).cuda()
    o = d_orig.index_select(1, idx).cpu().numpy()
    got = d_rec.index_select(1, idx).cpu().numpy()
    O.lib().orc_select_engine(1)
    try:
        want = O.encode("default", o, M)
    finally:
        O.lib().orc_select_engine(0)
    for k, b in enumerate(blocks):
        assert_rows_equal(got[:, 64 * k:64 * k + 64], want[:, 64 * k:64 * k + 64], f"column block {b}")


def test_config5_full_size_encode(torch, rs):
    """configs[4]: 32768:32768 x 64 KiB (2 GiB in, 2 GiB out) on one GPU, compared with the
    oracle on column blocks: first, middle, last, and two blocks inside every one of the 8
    rank slices (8 KiB each) of the column-partitioned multi-GPU encode.
    The reference pins 32768:32768 at 64 B (EITHER_32768_32768_11, rate_high.rs:376-389),
    which tests/test_oracle_golden.py checks against the oracle."""
    N = M = 32768
    S = 65536
    g = torch.Generator(device="cuda")
    g.manual_seed(55)
    d_orig = torch.randint(0, 256, (N, S), dtype=torch.uint8, device="cuda", generator=g)
    d_rec = torch.full((M, S), 0xEE, dtype=torch.uint8, device="cuda")
    rs.encode_device(N, M, S, d_orig, d_rec)
    torch.cuda.synchronize()
    rs.check_device()
    nb = S // 64
    blocks = sorted({0, nb // 2, nb - 1} | {r * (nb // 8) + k for r in range(8) for k in (0, 77)})
    _sampled_blocks_match(torch, d_orig, d_rec, M, blocks)
    # the 8 column slices of encode_device_sharded's partition, one after another through
    # rs_encode_device_strided, reassemble the single-call result exactly
    w = S // 8
    d_rec8 = torch.full((M, S), 0x11, dtype=torch.uint8, device="cuda")
    for r in range(8):
        rs.encode_device(N, M, w, d_orig[:, r * w:(r + 1) * w], d_rec8[:, r * w:(r + 1) * w])
    torch.cuda.synchronize()
    assert torch.equal(d_rec8, d_rec)


def test_config4_encode_sampled_blocks(torch, rs):
    """configs[3] shape 8192:8192 x 64 KiB: the encode on 16 column blocks spread over the
    whole shard (first .. last) equals the oracle."""
    N = M = 8192
    S = 65536
    g = torch.Generator(device="cuda")
    g.manual_seed(4)
    d_orig = torch.randint(0, 256, (N, S), dtype=torch.uint8, device="cuda", generator=g)
    d_rec = torch.empty((M, S), dtype=torch.uint8, device="cuda")
    rs.encode_device(N, M, S, d_orig, d_rec)
    torch.cuda.synchronize()
    nb = S // 64
    _sampled_blocks_match(torch, d_orig, d_rec, M, sorted({int(x) for x in np.linspace(0, nb - 1, 16)} | {333}))


@pytest.mark.parametrize("loss", [0.01, 1.0])
def test_baseline_decode_8192_64k(torch, rs, loss):
    """config 4: 8192:8192 x 64 KiB, decode at 1% and 100% loss (benchmarks.rs:113-138 pattern)."""
    N = M = 8192
    S = 65536
    orig = np.random.default_rng(1).integers(0, 256, (N, S), dtype=np.uint8)
    d_orig = _dev(torch, orig)
    d_rec = torch.empty((M, S), dtype=torch.uint8, device="cuda")
    rs.encode_device(N, M, S, d_orig, d_rec)
    torch.cuda.synchronize()
    _sampled_blocks_match(torch, d_orig, d_rec, M, [0, 1, 255, 512, 1023])
    L = -(-min(N, M) * int(loss * 100) // 100)
    op = np.ones(N, np.uint8)
    op[N - L:] = 0
    rp = np.zeros(M, np.uint8)
    rp[:L] = 1
    d_out = torch.zeros_like(d_orig)
    d_in = d_orig.clone()
    d_in[N - L:] = 0
    rs.decode_device(N, M, S, d_in, op, d_rec, rp, d_out)
    torch.cuda.synchronize()
    assert torch.equal(d_out[N - L:], d_orig[N - L:])


@pytest.mark.parametrize("rate,N,M,S,loss", [("low", 2048, 6144, 65536, 0.5), ("high", 6000, 2000, 65536, 0.3),
                                               ("default", 4096, 4096, 32768, 1.0)])
def test_large_matrix_passes_match_oracle(torch, rs, rate, N, M, S, loss):
    """Matrices of many times the resident workgroups (more row sets x column slices
    than the chip holds at once, so each pass's workgroups run in several rounds) on the
    multi-level pass kernels: encode on sampled column blocks vs the oracle, decode
    restores exactly."""
    g = torch.Generator(device="cuda")
    g.manual_seed(N + M)
    d_orig = torch.randint(0, 256, (N, S), dtype=torch.uint8, device="cuda", generator=g)
    d_rec = torch.empty((M, S), dtype=torch.uint8, device="cuda")
    rs.encode_device(N, M, S, d_orig, d_rec, rate_=RATE[rate])
    torch.cuda.synchronize()
    nb = S // 64
    cols = sorted({0, 1, nb // 3, nb // 2 + 5, nb - 1})
    idx = torch.from_numpy(np.concatenate([np.arange(64 * b, 64 * b + 64) for b in cols])).cuda()
    o = d_orig.index_select(1, idx).cpu().numpy()
    got = d_rec.index_select(1, idx).cpu().numpy()
    O.lib().orc_select_engine(1)
    try:
        want = O.encode(rate, o, M)
    finally:
        O.lib().orc_select_engine(0)
    assert_rows_equal(got, want)
    rng = np.random.default_rng(N)
    L = max(1, int(min(N, M) * loss))
    op = np.ones(N, np.uint8)
    op[rng.choice(N, L, replace=False)] = 0
    rp = np.zeros(M, np.uint8)
    rp[rng.choice(M, L, replace=False)] = 1
    miss = torch.from_numpy(op == 0).cuda()
    d_in = d_orig.clone()
    d_in[miss] = 0
    d_out = torch.zeros_like(d_orig)
    rs.decode_device(N, M, S, d_in, op, d_rec, rp, d_out, rate_=RATE[rate])
    torch.cuda.synchronize()
    assert torch.equal(d_out[miss], d_orig[miss])


# ---------------------------------------------------------------------------
# pass kernels on 2-level transforms (2^7 .. 2^12 rows), column kernel off

PASS_CASES = [
    ("high", 128, 128, 64), ("high", 1024, 1024, 1024), ("high", 4000, 128, 192), ("low", 128, 4000, 192),
    ("high", 4096, 4096, 64), ("low", 1000, 1500, 1088), ("high", 2048, 2048, 4096), ("default", 600, 200, 8192),
    ("high", 1024, 1024, 2048),
]


@pytest.mark.parametrize("rate,N,M,S", PASS_CASES)
def test_pass_path_matches_oracle(torch, rs, rate, N, M, S):
    rs.mono_enable(0)
    try:
        orig = O.generate_original(N, S, (N + M + S) & 0xFF)
        want = O.encode(rate, orig, M)
        got = gpu_encode(torch, rs, rate, orig, M)
        assert_rows_equal(got, want)
        rng = np.random.default_rng(N * 7 + M)
        L = min(N, M)
        op = np.ones(N, np.uint8)
        op[rng.choice(N, L, replace=False)] = 0
        rp = np.zeros(M, np.uint8)
        rp[rng.choice(M, L, replace=False)] = 1
        dw = O.decode(rate, orig, op, want, rp)
        dg = gpu_decode(torch, rs, rate, orig, op, want, rp)
        miss = op == 0
        assert np.array_equal(dg[miss], orig[miss]) and np.array_equal(dg[miss], dw[miss])
        rs.check_device()
    finally:
        rs.mono_enable(1)


def test_repeated_launches_stay_exact(torch, rs):
    """Back-to-back device encodes of the headline shape reuse one context's scratch."""
    N = M = 1024
    S = 1024
    orig = O.generate_original(N, S, 9)
    want = O.encode("high", orig, M)
    d_orig = _dev(torch, orig)
    d_rec = torch.empty((M, S), dtype=torch.uint8, device="cuda")
    for _ in range(200):
        rs.encode_device(N, M, S, d_orig, d_rec, rate_=1)
    rs.check_device()
    assert_rows_equal(d_rec.cpu().numpy(), want)


# ---------------------------------------------------------------------------
# column-slice (strided) device API: the multi-GPU column partition's building block

@pytest.mark.parametrize("rate,N,M,S,cols", [("high", 1024, 1024, 4096, (1024, 2048)), ("low", 200, 900, 1024, (0, 512)),
                                             ("high", 5000, 300, 640, (576, 640))])
def test_strided_column_slice_encode_decode(torch, rs, rate, N, M, S, cols):
    a, b = cols
    orig = O.generate_original(N, S, 3)
    want = O.encode(rate, orig, M)
    d_orig = _dev(torch, orig)
    d_rec = torch.full((M, S), 0x77, dtype=torch.uint8, device="cuda")
    rs.encode_device(N, M, b - a, d_orig[:, a:b], d_rec[:, a:b], rate_=RATE[rate])
    torch.cuda.synchronize()
    got = d_rec.cpu().numpy()
    assert_rows_equal(got[:, a:b], want[:, a:b])
    assert np.all(got[:, :a] == 0x77) and np.all(got[:, b:] == 0x77), "columns outside the slice untouched"
    rng = np.random.default_rng(1)
    L = min(N, M) // 2
    op = np.ones(N, np.uint8)
    op[rng.choice(N, L, replace=False)] = 0
    rp = np.zeros(M, np.uint8)
    rp[rng.choice(M, L, replace=False)] = 1
    d_o = _dev(torch, np.where(op[:, None] == 1, orig, 0).astype(np.uint8))
    d_r = _dev(torch, want)
    d_out = torch.full((N, S), 0x33, dtype=torch.uint8, device="cuda")
    rs.decode_device(N, M, b - a, d_o[:, a:b], op, d_r[:, a:b], rp, d_out[:, a:b], rate_=RATE[rate])
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    miss = op == 0
    assert_rows_equal(out[miss][:, a:b], orig[miss][:, a:b])
    assert np.all(out[:, :a] == 0x33) and np.all(out[:, b:] == 0x33)


# ---------------------------------------------------------------------------
# column kernel (one workgroup per pack, 2^7 .. 2^12 rows) vs pass kernels

MONO_CASES = [
    # encode transform sizes L = 7 .. 12, partial and multi-chunk inputs / outputs
    ("high", 128, 128, 64), ("high", 200, 256, 64), ("low", 256, 200, 128), ("high", 512, 300, 576),
    ("default", 1024, 1024, 1024), ("high", 3000, 1024, 64), ("low", 1000, 2500, 128), ("high", 2048, 2048, 64),
    ("low", 2048, 4000, 64), ("high", 4096, 4096, 64), ("low", 3000, 5000, 64), ("high", 40, 100, 192),
    ("high", 64, 64, 2048), ("low", 100, 37, 192),
]


@pytest.mark.parametrize("mono", [1, 1 | 8, 1 | 16, 2, 0])
@pytest.mark.parametrize("rate,N,M,S", MONO_CASES)
def test_column_kernel_and_pass_paths_match_oracle(torch, rs, rate, N, M, S, mono):
    """mono 1: default routing (2-element packs for small single-chunk launches), + 8: 4-element
    packs only, + 16: 2-element packs for every single-chunk launch, 2: column kernel for
    multi-chunk / 2^11-2^12 rows too, 0: pass kernels."""
    rs.mono_enable(mono)
    try:
        orig = O.generate_original(N, S, (N * 3 + M + S) & 0xFF)
        want = O.encode(rate, orig, M)
        got = gpu_encode(torch, rs, rate, orig, M)
        assert_rows_equal(got, want)
        rng = np.random.default_rng(N * 5 + M)
        for L in sorted({1, min(N, M) // 3 + 1, min(N, M)}):
            op = np.ones(N, np.uint8)
            op[rng.choice(N, L, replace=False)] = 0
            rp = np.zeros(M, np.uint8)
            rp[rng.choice(M, L, replace=False)] = 1
            dw = O.decode(rate, orig, op, want, rp)
            dg = gpu_decode(torch, rs, rate, orig, op, want, rp)
            miss = op == 0
            assert np.array_equal(dg[miss], orig[miss]) and np.array_equal(dg[miss], dw[miss])
            assert np.all(dg[~miss] == 0x33), "present rows of the output must not be written"
    finally:
        rs.mono_enable(1)


# ---------------------------------------------------------------------------
# one-row-per-lane column kernel (rs_lane.hip): single-chunk 2-element encodes of
# 2^8 .. 2^10 rows, HighRate and LowRate, tails, strided rows, batches

LANE_CASES = [
    ("default", 1024, 1024, 1024), ("high", 1000, 1024, 1024), ("high", 700, 513, 512), ("high", 200, 256, 256),
    ("low", 256, 200, 128), ("low", 400, 500, 64), ("high", 1024, 1024, 130), ("high", 900, 600, 1000),
    ("low", 129, 256, 6), ("high", 1, 1000, 64), ("high", 512, 512, 2),
]


def _route_of(torch, rs, fn):
    rs.profile_enable(True)
    fn()
    torch.cuda.synchronize()
    recs = rs.profile_collect()
    rs.profile_enable(False)
    return [name for name, _, _ in recs]


@pytest.mark.parametrize("rate,N,M,S", LANE_CASES)
def test_lane_kernel_encode_matches_oracle(torch, rs, rate, N, M, S):
    rs.mono_enable(1 | 32)
    try:
        orig = O.generate_original(N, S, (N + 2 * M + S) & 0xFF)
        want = O.encode(rate, orig, M)
        d_o = _dev(torch, orig)
        d_r = torch.full((M, S), 0xEE, dtype=torch.uint8, device="cuda")
        route = _route_of(torch, rs, lambda: rs.encode_device(N, M, S, d_o, d_r, rate_=RATE[rate]))
        assert len(route) == 1 and route[0].startswith("k_lane<"), route
        assert_rows_equal(d_r.cpu().numpy(), want)
        # strided rows: column slices of wider matrices (the rows' base and stride differ)
        wo = torch.full((N, S + 64), 0x11, dtype=torch.uint8, device="cuda")
        wr = torch.full((M, S + 64), 0x22, dtype=torch.uint8, device="cuda")
        wo[:, 32:32 + S] = d_o
        rs.encode_device(N, M, S, wo[:, 32:32 + S], wr[:, 32:32 + S], rate_=RATE[rate])
        torch.cuda.synchronize()
        got = wr.cpu().numpy()
        assert_rows_equal(got[:, 32:32 + S], want)
        assert np.all(got[:, :32] == 0x22) and np.all(got[:, 32 + S:] == 0x22)
        # a batch of 3 stripes in one launch
        origs = [orig] + [O.generate_original(N, S, 90 + b) for b in range(2)]
        b_o = _dev(torch, np.stack(origs))
        b_r = torch.empty((3, M, S), dtype=torch.uint8, device="cuda")
        rs.encode_device_batch(N, M, S, b_o, b_r, rate_=RATE[rate])
        torch.cuda.synchronize()
        for b in range(3):
            assert_rows_equal(b_r[b].cpu().numpy(), O.encode(rate, origs[b], M), f"stripe {b}")
    finally:
        rs.mono_enable(1)


# ---------------------------------------------------------------------------
# quad encode (rs_mono.hip kMonoQuadEnc, rs_codec.cpp try_quad): single-chunk 2-element
# encodes of 2^10 rows as the 4-element kernel of 2^9 pair rows (pack = 2 elements x rows
# 2q, 2q + 1), layer 0 inside the packs before the IFFT and after the FFT

QUAD_CASES = [
    # (rate, N, M, S): 2^10-row transforms, one chunk; tails, odd row counts, both rates
    ("high", 1024, 1024, 1024), ("high", 1000, 1000, 576), ("high", 1, 513, 64), ("high", 600, 1000, 130),
    ("high", 1023, 1021, 6), ("high", 1024, 600, 2), ("low", 1024, 1024, 256), ("low", 1000, 600, 192),
    ("low", 513, 7, 66), ("default", 700, 999, 1000),
]


@pytest.mark.parametrize("rate,N,M,S", QUAD_CASES)
def test_quad_encode_matches_oracle(torch, rs, rate, N, M, S):
    rs.mono_enable(1 | 2048)
    try:
        orig = O.generate_original(N, S, (N + 3 * M + S) & 0xFF)
        want = O.encode(rate, orig, M)
        d_o = _dev(torch, orig)
        d_r = torch.full((M, S), 0xEE, dtype=torch.uint8, device="cuda")
        route = _route_of(torch, rs, lambda: rs.encode_device(N, M, S, d_o, d_r, rate_=RATE[rate]))
        assert len(route) == 1 and route[0].startswith("k_mono<9, 1, 7,"), route
        assert_rows_equal(d_r.cpu().numpy(), want, "quad encode")
        # strided rows: column slices of wider matrices (the rows' base and stride differ)
        wo = torch.full((N, S + 64), 0x11, dtype=torch.uint8, device="cuda")
        wr = torch.full((M, S + 64), 0x22, dtype=torch.uint8, device="cuda")
        wo[:, 32:32 + S] = d_o
        rs.encode_device(N, M, S, wo[:, 32:32 + S], wr[:, 32:32 + S], rate_=RATE[rate])
        torch.cuda.synchronize()
        got = wr.cpu().numpy()
        assert_rows_equal(got[:, 32:32 + S], want, "quad encode, strided")
        assert np.all(got[:, :32] == 0x22) and np.all(got[:, 32 + S:] == 0x22)
        # a batch of 3 stripes in one launch (2-element packs while packs x stripes fit)
        if S <= 1024:
            origs = [orig] + [O.generate_original(N, S, 70 + b) for b in range(2)]
            b_o = _dev(torch, np.stack(origs))
            b_r = torch.empty((3, M, S), dtype=torch.uint8, device="cuda")
            rs.encode_device_batch(N, M, S, b_o, b_r, rate_=RATE[rate])
            torch.cuda.synchronize()
            for b in range(3):
                assert_rows_equal(b_r[b].cpu().numpy(), O.encode(rate, origs[b], M), f"quad batch stripe {b}")
        # quad off: the 2-element column kernel, the same bytes
        rs.mono_enable(1 | 4096)
        d_r2 = torch.full((M, S), 0x77, dtype=torch.uint8, device="cuda")
        route = _route_of(torch, rs, lambda: rs.encode_device(N, M, S, d_o, d_r2, rate_=RATE[rate]))
        assert not any(r.startswith("k_mono<9, 1, 7,") for r in route), route
        assert torch.equal(d_r, d_r2)
    finally:
        rs.mono_enable(1)


# ---------------------------------------------------------------------------
# multi-chunk encodes of 2^2..2^7-row transforms in one launch (rs_chunks.hip k_chunks): the
# waves of a pack's workgroup take HighRate input chunks / LowRate output chunks in parallel
# (routed by default where it measured faster, rs_codec.cpp use_chunks; rs_mono_enable + 512
# forces every shape; 2-element packs stage 8-word basis tables, CTabsBasis)

CHUNKS_CASES = [
    # (rate, N, M, S): HighRate N > pow2(M) (chunks = ceil(N / pow2(M))), LowRate M > pow2(N)
    ("high", 1000, 100, 1024), ("high", 1000, 128, 256), ("high", 2000, 100, 192), ("high", 500, 64, 130),
    ("high", 300, 30, 64), ("high", 100, 10, 6), ("high", 50, 5, 64), ("high", 20, 3, 2), ("high", 9000, 100, 2),
    ("low", 128, 1024, 1024), ("low", 100, 1000, 256), ("low", 64, 640, 130), ("low", 10, 100, 64),
    ("low", 3, 20, 6), ("low", 100, 9000, 2), ("default", 4000, 120, 64), ("default", 5, 41, 320),
    # two packs per wave past 256 4-element packs (HighRate), odd pack counts, tails
    ("high", 1000, 100, 4096), ("high", 600, 100, 3000), ("high", 300, 60, 2050),
]


@pytest.mark.parametrize("mono", [1 | 512, 1 | 8 | 512, 1 | 16 | 512])
@pytest.mark.parametrize("rate,N,M,S", CHUNKS_CASES)
def test_chunks_kernel_encode_matches_oracle(torch, rs, rate, N, M, S, mono):
    rs.mono_enable(mono)
    try:
        orig = O.generate_original(N, S, (3 * N + M + S) & 0xFF)
        want = O.encode(rate, orig, M)
        d_o = _dev(torch, orig)
        d_r = torch.full((M, S), 0xEE, dtype=torch.uint8, device="cuda")
        route = _route_of(torch, rs, lambda: rs.encode_device(N, M, S, d_o, d_r, rate_=RATE[rate]))
        assert len(route) == 1 and route[0].startswith("k_chunks<"), route
        assert_rows_equal(d_r.cpu().numpy(), want)
        # strided rows: column slices of wider matrices
        wo = torch.full((N, S + 64), 0x11, dtype=torch.uint8, device="cuda")
        wr = torch.full((M, S + 64), 0x22, dtype=torch.uint8, device="cuda")
        wo[:, 32:32 + S] = d_o
        rs.encode_device(N, M, S, wo[:, 32:32 + S], wr[:, 32:32 + S], rate_=RATE[rate])
        torch.cuda.synchronize()
        got = wr.cpu().numpy()
        assert_rows_equal(got[:, 32:32 + S], want)
        assert np.all(got[:, :32] == 0x22) and np.all(got[:, 32 + S:] == 0x22)
    finally:
        rs.mono_enable(1)


def test_chunks_kernel_off_matches_on(torch, rs):
    """rs_mono_enable + 1024 (k_chunks off: the chunk-parallel passes) gives the same bytes as the
    default route (k_chunks for this HighRate 8-chunk shape)."""
    N, M, S = 1000, 100, 1024
    g = torch.Generator(device="cuda")
    g.manual_seed(5)
    d_o = torch.randint(0, 256, (N, S), dtype=torch.uint8, device="cuda", generator=g)
    outs = []
    for mode in (1 | 1024, 1):
        rs.mono_enable(mode)
        try:
            d_r = torch.empty((M, S), dtype=torch.uint8, device="cuda")
            rs.encode_device(N, M, S, d_o, d_r)
            torch.cuda.synchronize()
            outs.append(d_r)
        finally:
            rs.mono_enable(1)
    assert torch.equal(outs[0], outs[1])


# ---------------------------------------------------------------------------
# half-split 2^12-row transforms (rs_codec.cpp half_split, rs_mono_enable + 128; off by
# default, slower than the passes): two launches of the 2^11-row column kernel -- the IFFT
# below the top layer per half with input rows, then the top layer (+ the decode's formal
# derivative) and the FFT per half with output rows

HALF_ENC = [
    # (rate, N, M, S): single-chunk encodes of 2^12 rows; inputs / outputs in one or both halves
    ("high", 4096, 4096, 1024), ("high", 2000, 3000, 256), ("high", 4000, 2500, 130), ("high", 1, 2049, 64),
    ("low", 4096, 4096, 64), ("low", 3000, 1000, 64), ("low", 2500, 4000, 6), ("low", 4096, 1, 2),
]
HALF_DEC = [
    # (rate, N, M, S, pattern): 4096 work rows; "lost_all": every original lost, so the
    # received rows lie in one half (the other half's IFFT is not launched)
    ("high", 2048, 2048, 1024, "random"), ("high", 2048, 2048, 64, "lost_all"), ("high", 3000, 1000, 128, "random"),
    ("low", 2000, 2000, 64, "random"), ("low", 1024, 3000, 130, "random"), ("low", 2000, 2000, 6, "lost_all"),
    ("high", 2048, 2048, 1024, "one"),
]


def _half_modes(route, dec):
    """kMonoHalf* modes (rs_device.hpp MonoMode) in launch order"""
    return [int(n.split(",")[2]) for n in route if n.startswith("k_mono<11,")]


@pytest.mark.parametrize("mono", [1 | 128, 1 | 8 | 128, 1 | 16 | 128])
@pytest.mark.parametrize("rate,N,M,S", HALF_ENC)
def test_half_split_encode_matches_oracle(torch, rs, rate, N, M, S, mono):
    rs.mono_enable(mono)
    try:
        orig = O.generate_original(N, S, (N + 5 * M + S) & 0xFF)
        want = O.encode(rate, orig, M)
        d_o = _dev(torch, orig)
        d_r = torch.full((M, S), 0xEE, dtype=torch.uint8, device="cuda")
        route = _route_of(torch, rs, lambda: rs.encode_device(N, M, S, d_o, d_r, rate_=RATE[rate]))
        assert _half_modes(route, False) == [3, 5] and len(route) == 2, route
        assert_rows_equal(d_r.cpu().numpy(), want, "half-split encode")
        # strided rows: column slices of wider matrices
        wo = torch.full((N, S + 64), 0x11, dtype=torch.uint8, device="cuda")
        wr = torch.full((M, S + 64), 0x22, dtype=torch.uint8, device="cuda")
        wo[:, 32:32 + S] = d_o
        rs.encode_device(N, M, S, wo[:, 32:32 + S], wr[:, 32:32 + S], rate_=RATE[rate])
        torch.cuda.synchronize()
        got = wr.cpu().numpy()
        assert_rows_equal(got[:, 32:32 + S], want, "half-split encode, strided")
        assert np.all(got[:, :32] == 0x22) and np.all(got[:, 32 + S:] == 0x22)
    finally:
        rs.mono_enable(1)


@pytest.mark.parametrize("mono", [1 | 128, 1 | 8 | 128, 1 | 16 | 128])
@pytest.mark.parametrize("rate,N,M,S,kind", HALF_DEC)
def test_half_split_decode_matches_oracle(torch, rs, rate, N, M, S, kind, mono):
    rs.mono_enable(mono)
    try:
        rng = np.random.default_rng(N + 7 * M + S)
        orig = O.generate_original(N, S, (N + M + S) & 0xFF)
        rec = O.encode(rate, orig, M)
        op = np.ones(N, np.uint8)
        if kind == "lost_all":
            op[:] = 0
        elif kind == "one":
            op[N // 3] = 0
        else:
            op[rng.choice(N, max(1, min(N, M) // 3), replace=False)] = 0
        lost = int((op == 0).sum())
        rp = np.zeros(M, np.uint8)
        rp[rng.choice(M, lost, replace=False)] = 1
        want = O.decode(rate, orig, op, rec, rp)
        d_o = _dev(torch, np.where(op[:, None] == 1, orig, 0xA5).astype(np.uint8))
        d_r = _dev(torch, np.where(rp[:, None] == 1, rec, 0x5A).astype(np.uint8))
        d_out = torch.full((N, S), 0x33, dtype=torch.uint8, device="cuda")
        route = _route_of(torch, rs, lambda: rs.decode_device(N, M, S, d_o, op, d_r, rp, d_out, rate_=RATE[rate]))
        assert _half_modes(route, True) == [4, 6] and len(route) == 3, route  # + k_eval_poly
        got = d_out.cpu().numpy()
        miss = op == 0
        assert_rows_equal(got[miss], orig[miss], "half-split decode vs originals")
        assert_rows_equal(got[miss], want[miss], "half-split decode vs oracle")
        assert np.all(got[~miss] == 0x33), "present rows of the output must not be written"
        rs.check_device()
    finally:
        rs.mono_enable(1)


def test_half_split_off_matches_on(torch, rs):
    """rs_mono_enable + 256 (half-split off: the pass kernels) and + 128 give the same bytes."""
    N, M, S = 4096, 4096, 512
    g = torch.Generator(device="cuda")
    g.manual_seed(11)
    d_o = torch.randint(0, 256, (N, S), dtype=torch.uint8, device="cuda", generator=g)
    outs = []
    for mode in (1 | 256, 1 | 128):
        rs.mono_enable(mode)
        try:
            d_r = torch.empty((M, S), dtype=torch.uint8, device="cuda")
            rs.encode_device(N, M, S, d_o, d_r)
            torch.cuda.synchronize()
            outs.append(d_r)
        finally:
            rs.mono_enable(1)
    assert torch.equal(outs[0], outs[1])


# ---------------------------------------------------------------------------
# host-memory pipeline (column slices over several streams, pinned or pageable buffers)

@pytest.mark.parametrize("rate,N,M,S,slices,pinned", [
    ("default", 1024, 1024, 1024, 4, True), ("default", 1024, 1024, 1024, 1, False), ("high", 3000, 700, 640, 3, True),
    ("low", 100, 1000, 192, 8, False), ("default", 5000, 300, 4096, 5, True),
    # shards with a tail block: the last slice carries it (34 bytes alone for 130 / 2)
    ("default", 1000, 1000, 130, 2, True), ("high", 300, 50, 1000, 3, False), ("low", 50, 300, 6, 4, True)])
def test_host_pipeline_matches_oracle(torch, rs, rate, N, M, S, slices, pinned):
    orig = O.generate_original(N, S, 21)
    want = O.encode(rate, orig, M)
    if pinned:
        h_o = torch.from_numpy(orig).pin_memory()
        h_r = torch.full((M, S), 0xEE, dtype=torch.uint8).pin_memory()
    else:
        h_o, h_r = orig.copy(), np.full((M, S), 0xEE, np.uint8)
    rs.encode_host(N, M, S, h_o, h_r, slices=slices, rate_=RATE[rate])
    got = h_r.numpy() if pinned else h_r
    assert_rows_equal(got, want)
    rng = np.random.default_rng(N + M + S)
    L = max(1, min(N, M) // 3)
    op = np.ones(N, np.uint8)
    op[rng.choice(N, L, replace=False)] = 0
    rp = np.zeros(M, np.uint8)
    rp[rng.choice(M, L, replace=False)] = 1
    h_out = np.full((N, S), 0x33, np.uint8)
    rs.decode_host(N, M, S, np.where(op[:, None] == 1, orig, 0xA5).astype(np.uint8), op,
                   np.where(rp[:, None] == 1, want, 0x5A).astype(np.uint8), rp, h_out, slices=slices,
                   rate_=RATE[rate])
    miss = op == 0
    assert_rows_equal(h_out[miss], orig[miss])
    assert np.all(h_out[~miss] == 0x33), "present rows of the output must not be written"


# ---------------------------------------------------------------------------
# batches of stripes (rs_encode_device_batch / rs_decode_device_batch): every
# stripe equals the oracle's single-stripe result.  Column-kernel shapes run
# the batch as one launch; the others loop over the stripes.

BATCH_CASES = [
    # (rate, N, M, S, stripes)
    ("default", 1024, 1024, 1024, 3), ("default", 1000, 1000, 576, 2), ("low", 100, 1000, 128, 3),
    ("default", 200, 56, 2048, 4), ("default", 5000, 300, 256, 2), ("default", 64, 64, 1024, 5),
]


@pytest.mark.parametrize("rate,N,M,S,B", BATCH_CASES)
def test_batch_encode_decode_match_oracle(torch, rs, rate, N, M, S, B):
    origs = [O.generate_original(N, S, 40 + b) for b in range(B)]
    d_o = _dev(torch, np.stack(origs))
    # recovery rows padded to a wider stripe pitch: the stripe stride is not M rows
    d_r_full = torch.full((B, M + 3, S), 0xEE, dtype=torch.uint8, device="cuda")
    d_r = d_r_full[:, :M, :]
    rs.encode_device_batch(N, M, S, d_o, d_r, rate_=RATE[rate])
    torch.cuda.synchronize()
    got = d_r.cpu().numpy()
    recs = [O.encode(rate, origs[b], M) for b in range(B)]
    for b in range(B):
        assert_rows_equal(got[b], recs[b], f"stripe {b}")
    assert np.all(d_r_full[:, M:, :].cpu().numpy() == 0xEE), "padding rows must not be written"
    # one erasure pattern for every stripe
    rng = np.random.default_rng(N + M + B)
    L = max(1, min(N, M) // 10)
    op = np.ones(N, np.uint8)
    op[rng.choice(N, L, replace=False)] = 0
    rp = np.zeros(M, np.uint8)
    rp[rng.choice(M, L, replace=False)] = 1
    d_oo = _dev(torch, np.stack([np.where(op[:, None] == 1, o, 0xA5).astype(np.uint8) for o in origs]))
    d_rr = _dev(torch, np.stack([np.where(rp[:, None] == 1, r, 0x5A).astype(np.uint8) for r in recs]))
    d_out = torch.full((B, N, S), 0x33, dtype=torch.uint8, device="cuda")
    rs.decode_device_batch(N, M, S, d_oo, op, d_rr, rp, d_out, rate_=RATE[rate])
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    miss = op == 0
    for b in range(B):
        assert_rows_equal(out[b][miss], origs[b][miss], f"stripe {b}")
        assert np.all(out[b][~miss] == 0x33)


def test_batch_matches_single_stripe_calls_at_headline(torch, rs):
    """64 stripes of the headline shape in one launch == 64 single-stripe encodes."""
    B, N, M, S = 64, 1024, 1024, 1024
    g = torch.Generator(device="cuda")
    g.manual_seed(7)
    d_o = torch.randint(0, 256, (B, N, S), dtype=torch.uint8, device="cuda", generator=g)
    d_r = torch.empty((B, M, S), dtype=torch.uint8, device="cuda")
    rs.encode_device_batch(N, M, S, d_o, d_r)
    one = torch.empty((M, S), dtype=torch.uint8, device="cuda")
    for b in (0, 17, 63):
        rs.encode_device(N, M, S, d_o[b], one)
        torch.cuda.synchronize()
        assert torch.equal(one, d_r[b]), f"stripe {b}"


# ---------------------------------------------------------------------------
# pruned FFT passes (rs_codec.cpp fft_pass_pruned): below the top level, only
# the row sets whose superblock holds erased originals are launched (at most 4
# runs per pass); 16384:16384 and 20000:30000 (low) decode over 3 levels

def _loss_pattern(kind, N, rng):
    op = np.ones(N, np.uint8)
    if kind == "tail":
        op[N - max(1, N // 100):] = 0
    elif kind == "head":
        op[:max(1, N // 100)] = 0
    elif kind == "middle":
        op[N // 2 - 40:N // 2 + 41] = 0
    elif kind == "one":
        op[N // 3] = 0
    elif kind == "spread":  # many runs: gaps bridged down to 4 launches
        op[::max(1, N // 9)] = 0
    elif kind == "random":
        op[rng.choice(N, max(1, N // 50), replace=False)] = 0
    elif kind == "all":
        op[:] = 0
    return op


@pytest.mark.parametrize("kind", ["tail", "head", "middle", "one", "spread", "random", "all"])
@pytest.mark.parametrize("rate,N,M,S", [("high", 4096, 4096, 128), ("low", 3000, 5000, 64),
                                        ("high", 8192, 8192, 64), ("high", 1024, 1024, 1024),
                                        ("high", 16384, 16384, 64), ("low", 20000, 30000, 64),
                                        # rows >= 8 KiB: per-row U-store masks (keep_out) with
                                        # zero_in blocks and bridged runs
                                        ("high", 4096, 4096, 8192)])
@pytest.mark.parametrize("mono", [1, 0])
def test_decode_loss_patterns_pruned_reveal(torch, rs, kind, rate, N, M, S, mono):
    rs.mono_enable(mono)
    try:
        orig = O.generate_original(N, S, 9)
        O.lib().orc_select_engine(1)
        try:
            rec = O.encode(rate, orig, M)
        finally:
            O.lib().orc_select_engine(0)
        op = _loss_pattern(kind, N, np.random.default_rng(N + S))
        L = int((op == 0).sum())
        if L > M:
            pytest.skip("more losses than recovery shards")
        rp = np.zeros(M, np.uint8)
        rp[np.random.default_rng(M).choice(M, L, replace=False)] = 1
        got = gpu_decode(torch, rs, rate, orig, op, rec, rp)
        miss = op == 0
        assert_rows_equal(got[miss], orig[miss])
        assert np.all(got[~miss] == 0x33), "present rows of the output must not be written"
        rs.check_device()
    finally:
        rs.mono_enable(1)


SPLIT_CASES = [
    # (rate, N, M, S): 2^9 .. 2^11 work rows, restored rows in the upper (high) / lower (low) half
    ("high", 1024, 1024, 1024), ("low", 1024, 1000, 512), ("high", 512, 512, 640), ("low", 512, 300, 192),
    ("high", 256, 256, 128), ("low", 256, 200, 64), ("high", 700, 1000, 256), ("high", 1500, 500, 192),
]


@pytest.mark.parametrize("kind", ["tail", "head", "one", "random", "all", "straddle"])
@pytest.mark.parametrize("rate,N,M,S", SPLIT_CASES)
def test_split_decode_matches_oracle(torch, rs, rate, N, M, S, kind):
    """Column-kernel decodes under the split plan (restored rows in one half of the work rows:
    only that half runs the FFT below the top layer) and, for losses in both halves of
    1500:500 (work rows 512..2011 hold originals), the unsplit plan; split on and off give
    the same bytes."""
    orig = O.generate_original(N, S, 17)
    rec = O.encode(rate, orig, M)
    rng = np.random.default_rng(N + M + S)
    if kind == "straddle":
        op = np.ones(N, np.uint8)
        op[[0, N // 2, N - 1]] = 0
    else:
        op = _loss_pattern(kind, N, rng)
    L = int((op == 0).sum())
    if L > M:
        pytest.skip("more losses than recovery shards")
    rp = np.zeros(M, np.uint8)
    rp[rng.choice(M, L, replace=False)] = 1
    outs = []
    for flag in (1, 1 | 4, 1 | 8, 1 | 4 | 8):
        rs.mono_enable(flag)
        try:
            outs.append(gpu_decode(torch, rs, rate, orig, op, rec, rp))
        finally:
            rs.mono_enable(1)
    miss = op == 0
    for got in outs:
        assert_rows_equal(got[miss], orig[miss])
        assert np.all(got[~miss] == 0x33), "present rows of the output must not be written"
    rs.check_device()


def test_bound_device_calls_match_oracle(torch, rs):
    """encode_device_call / decode_device_call (the bench's timed calls) = the oracle."""
    N, M, S = 1024, 1024, 1024
    orig = O.generate_original(N, S, 3)
    want = O.encode("default", orig, M)
    d_orig = _dev(torch, orig)
    d_rec = torch.zeros((M, S), dtype=torch.uint8, device="cuda")
    enc = rs.encode_device_call(N, M, S, d_orig, d_rec)
    for _ in range(3):
        enc()
    torch.cuda.synchronize()
    assert_rows_equal(d_rec.cpu().numpy(), want)
    L = 11
    op = np.ones(N, np.uint8)
    op[N - L:] = 0
    rp = np.zeros(M, np.uint8)
    rp[:L] = 1
    d_out = torch.full((N, S), 0x33, dtype=torch.uint8, device="cuda")
    dec = rs.decode_device_call(N, M, S, d_orig, op, d_rec, rp, d_out)
    dec()
    torch.cuda.synchronize()
    got = d_out.cpu().numpy()
    assert np.array_equal(got[N - L:], orig[N - L:]) and np.all(got[:N - L] == 0x33)
    with pytest.raises(rs.Error):
        rs.encode_device_call(3, 70000, 64, d_orig, d_rec)()


# ---------------------------------------------------------------------------
# device path on shards of any even length (rs_device.hpp ShardFormat): the tail
# block keeps the reference's layout (shards.rs:38-74), so the device result must
# equal the oracle's (which re-packs like the reference) byte for byte, and the
# reference's golden vectors must hash equal through the device path too.

def _device_golden(torch, rs, c):
    n, m, s = c["original_count"], c["recovery_count"], c["shard_bytes"]
    orig = O.generate_original(n, s, c["seed"])
    d_o = _dev(torch, orig)
    d_r = torch.full((m, s), 0xEE, dtype=torch.uint8, device="cuda")
    rs.encode_device(n, m, s, d_o, d_r, rate_=RATE[c["rate"]])
    torch.cuda.synchronize()
    rec = d_r.cpu().numpy()
    assert hashlib.sha256(rec.tobytes()).hexdigest() == c["recovery_sha256"], c["source"]
    op = np.zeros(n, np.uint8)
    rp = np.zeros(m, np.uint8)
    for a, b in c["decoder_original"]:
        op[a:b] = 1
    for a, b in c["decoder_recovery"]:
        rp[a:b] = 1
    if op.all():
        return
    d_oo = _dev(torch, np.where(op[:, None] == 1, orig, 0xA5).astype(np.uint8))
    d_rr = _dev(torch, np.where(rp[:, None] == 1, rec, 0x5A).astype(np.uint8))
    d_out = torch.full((n, s), 0x33, dtype=torch.uint8, device="cuda")
    rs.decode_device(n, m, s, d_oo, op, d_rr, rp, d_out, rate_=RATE[c["rate"]])
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    miss = op == 0
    assert_rows_equal(out[miss], orig[miss], str(c["source"]))
    assert np.all(out[~miss] == 0x33)


@pytest.mark.parametrize("case", [pytest.param(c, id=c["name"]) for c in GOLD["single"]
                                  if not c["name"].startswith(("DEFAULT_TINY", "LOW_TINY"))])
def test_golden_vectors_device_path(torch, rs, case):
    """Every golden case (HIGH_34000_2000_s8 / LOW_2000_34000_s8: 8-byte shards, all tail) via the device API."""
    _device_golden(torch, rs, case)


TAIL_SIZES = [2, 4, 6, 30, 32, 34, 62, 64, 66, 126, 128, 130]


@pytest.mark.parametrize("S", TAIL_SIZES)
@pytest.mark.parametrize("rate,N,M", [("default", 3, 2), ("high", 1000, 100), ("low", 100, 1000),
                                      ("default", 4096, 4096), ("high", 20000, 3000)])
def test_device_path_any_even_shard_size(torch, rs, rate, N, M, S):
    """decoder_result.rs:166-171 sizes through rs_encode_device / rs_decode_device (column kernel and passes)."""
    orig = O.generate_original(N, S, S)
    want = O.encode(rate, orig, M)
    got = gpu_encode(torch, rs, rate, orig, M)
    assert_rows_equal(got, want)
    rng = np.random.default_rng(S + N)
    L = max(1, min(N, M) // 4)
    op = np.ones(N, np.uint8)
    op[rng.choice(N, L, replace=False)] = 0
    rp = np.zeros(M, np.uint8)
    rp[rng.choice(M, L, replace=False)] = 1
    out = gpu_decode(torch, rs, rate, orig, op, want, rp)
    miss = op == 0
    assert_rows_equal(out[miss], orig[miss])
    assert np.all(out[~miss] == 0x33)


@pytest.mark.parametrize("S,off,pad", [(64, 1, 3), (130, 2, 0), (34, 1, 1), (1024, 3, 5), (6, 0, 1)])
@pytest.mark.parametrize("rate,N,M", [("default", 1000, 1000), ("high", 3000, 300), ("low", 64, 64)])
def test_device_path_unaligned_matrices(torch, rs, rate, N, M, S, off, pad):
    """Row strides / base addresses that are not multiples of 4 go byte by byte; same bytes as the oracle."""
    orig = O.generate_original(N, S, 9)
    want = O.encode(rate, orig, M)
    W = S + off + pad
    d_ob = torch.full((N, W), 0x11, dtype=torch.uint8, device="cuda")
    d_ob[:, off:off + S] = _dev(torch, orig)
    d_rb = torch.full((M, W), 0xEE, dtype=torch.uint8, device="cuda")
    rs.encode_device(N, M, S, d_ob[:, off:off + S], d_rb[:, off:off + S], rate_=RATE[rate])
    torch.cuda.synchronize()
    rb = d_rb.cpu().numpy()
    assert_rows_equal(rb[:, off:off + S], want)
    assert np.all(rb[:, :off] == 0xEE) and np.all(rb[:, off + S:] == 0xEE), "bytes around the slice must not change"
    rng = np.random.default_rng(N + S)
    L = max(1, min(N, M) // 3)
    op = np.ones(N, np.uint8)
    op[rng.choice(N, L, replace=False)] = 0
    rp = np.zeros(M, np.uint8)
    rp[rng.choice(M, L, replace=False)] = 1
    d_xb = torch.full((N, W), 0x33, dtype=torch.uint8, device="cuda")
    rs.decode_device(N, M, S, d_ob[:, off:off + S], op, d_rb[:, off:off + S], rp, d_xb[:, off:off + S],
                     rate_=RATE[rate])
    torch.cuda.synchronize()
    xb = d_xb.cpu().numpy()
    miss = op == 0
    assert_rows_equal(xb[miss, off:off + S], orig[miss])
    assert np.all(xb[~miss] == 0x33)
    assert np.all(xb[:, :off] == 0x33) and np.all(xb[:, off + S:] == 0x33)


@pytest.mark.parametrize("rate,N,M,S,B", [("default", 1024, 1024, 130, 3), ("low", 100, 1000, 34, 2),
                                          ("default", 64, 64, 1000, 4)])
def test_batch_with_tail_shards(torch, rs, rate, N, M, S, B):
    origs = [O.generate_original(N, S, 60 + b) for b in range(B)]
    d_o = _dev(torch, np.stack(origs))
    d_r = torch.full((B, M, S), 0xEE, dtype=torch.uint8, device="cuda")
    rs.encode_device_batch(N, M, S, d_o, d_r, rate_=RATE[rate])
    torch.cuda.synchronize()
    got = d_r.cpu().numpy()
    for b in range(B):
        assert_rows_equal(got[b], O.encode(rate, origs[b], M), f"stripe {b}")


def test_work_handoff_between_encoders_and_decoders(rs):
    """RateEncoder/RateDecoder::into_parts -> new(.., Some(work)) (src/rate.rs:129-139, 206-218; the
    DefaultRate reset path, rate_default.rs:170-195): a consumed encoder's buffers serve a new
    encoder of another rate and shape, the same for decoders; a failing `new` consumes the work."""
    def encode_with(cls, n, m, s, seed, work=None):
        orig = O.generate_original(n, s, seed)
        enc = cls(n, m, s, work=work)
        for row in orig:
            enc.add_original_shard(row.tobytes())
        rec = b"".join(enc.encode().recovery_iter())
        assert rec == O.encode({rs.rate.HighRateEncoder: "high", rs.rate.LowRateEncoder: "low",
                                rs.ReedSolomonEncoder: "default"}[cls], orig, m).tobytes()
        return enc, orig, rec

    enc, _, _ = encode_with(rs.rate.HighRateEncoder, 100, 37, 128, 1)
    ctx, work = enc.into_parts()
    assert ctx is not None
    enc2, _, _ = encode_with(rs.rate.LowRateEncoder, 37, 100, 64, 2, work=work)
    _, work2 = enc2.into_parts()
    with pytest.raises(rs.InvalidShardSize):
        rs.ReedSolomonEncoder(3, 2, 7, work=work2)  # consumed although new fails
    with pytest.raises(ValueError):
        rs.ReedSolomonEncoder(3, 2, 64, work=work2)
    enc3, orig3, rec3 = encode_with(rs.ReedSolomonEncoder, 3, 5, 130, 3)

    dec = rs.rate.LowRateDecoder(3, 5, 130)
    dec.add_original_shard(1, orig3[1].tobytes())
    for i in range(2):
        dec.add_recovery_shard(i, rec3[130 * i:130 * (i + 1)])
    out = dec.decode()
    assert out.restored_original(0) == orig3[0].tobytes() and out.restored_original(2) == orig3[2].tobytes()
    _, dwork = dec.into_parts()
    orig = O.generate_original(1000, 256, 9)
    rec = O.encode("high", orig, 100)
    dec2 = rs.rate.HighRateDecoder(1000, 100, 256, work=dwork)
    for i in range(100, 1000):
        dec2.add_original_shard(i, orig[i].tobytes())
    for i in range(100):
        dec2.add_recovery_shard(i, rec[i].tobytes())
    restored = dict(dec2.decode().restored_original_iter())
    assert all(restored[i] == orig[i].tobytes() for i in range(100))


# ---------------------------------------------------------------------------
# copy_rows' span mode (rs_codec.cpp): with more than 4 runs of received rows, the host
# pipeline and the decoder object copy whole spans, absent rows included, and the object's
# D2H copy writes present rows of its output staging.  So every decode route must never
# read an absent row of its inputs, and nothing may read present rows of the staging
# (ADVICE r05).  Absent rows here hold another stripe's bytes (the object's staging left by
# the previous decode) or 0xEE (the host pipeline's inputs), under scattered losses.

SPAN_CASES = [
    # (rate, N, M, S): the decode routes -- column kernel 2^11 (split / not), 2^7 padded,
    # eval_poly + passes (2^12, 2^13 rows), one fused single pass, LowRate
    ("high", 1024, 1024, 1024), ("high", 700, 300, 512), ("high", 40, 20, 320), ("high", 12, 4, 4096),
    ("high", 2048, 2048, 256), ("high", 3000, 1000, 128), ("low", 100, 1000, 192), ("low", 300, 2500, 64),
]


@pytest.mark.parametrize("rate,N,M,S", SPAN_CASES)
def test_decode_ignores_absent_rows_and_stale_staging(torch, rs, rate, N, M, S):
    cls_d = {"high": rs.rate.HighRateDecoder, "low": rs.rate.LowRateDecoder}[rate]
    rng = np.random.default_rng(N * 3 + M + S)
    a = O.generate_original(N, S, 5)
    b = O.generate_original(N, S, 6)
    rec_a, rec_b = O.encode(rate, a, M), O.encode(rate, b, M)
    L = max(1, min(N, M) // 2)
    dec = cls_d(N, M, S)
    # stripe a: lose a contiguous head, so the staging's rows of b's scattered losses hold a's bytes
    op_a = np.ones(N, np.uint8)
    op_a[:L] = 0
    for i in np.flatnonzero(op_a):
        dec.add_original_shard(int(i), a[i].tobytes())
    for i in range(L):
        dec.add_recovery_shard(i, rec_a[i].tobytes())
    got = dict(dec.decode().restored_original_iter())
    assert all(got[i] == a[i].tobytes() for i in range(L))
    # stripe b: scattered losses (> 4 runs of received rows whenever L allows)
    dec.reset(N, M, S)
    op_b = np.ones(N, np.uint8)
    op_b[rng.choice(N, L, replace=False)] = 0
    rp_b = np.zeros(M, np.uint8)
    rp_b[rng.choice(M, L, replace=False)] = 1
    for i in np.flatnonzero(op_b):
        dec.add_original_shard(int(i), b[i].tobytes())
    for i in np.flatnonzero(rp_b):
        dec.add_recovery_shard(int(i), rec_b[i].tobytes())
    got = dict(dec.decode().restored_original_iter())
    assert sorted(got) == [int(i) for i in np.flatnonzero(op_b == 0)]
    bad = [i for i in got if got[i] != b[i].tobytes()]
    assert not bad, f"object API decode: restored rows {bad[:8]} differ (stale staging read?)"
    # the host pipeline with 0xEE in every absent input row
    h_out = np.full((N, S), 0x33, np.uint8)
    rs.decode_host(N, M, S, np.where(op_b[:, None] == 1, b, 0xEE).astype(np.uint8), op_b,
                   np.where(rp_b[:, None] == 1, rec_b, 0xEE).astype(np.uint8), rp_b, h_out, slices=2,
                   rate_=RATE[rate])
    miss = op_b == 0
    assert_rows_equal(h_out[miss], b[miss], "host pipeline decode")
    assert np.all(h_out[~miss] == 0x33), "present rows of the output must not be written"


# ---------------------------------------------------------------------------
# the C ABI's one-shot rs_encode / rs_decode (lib.rs:251-353): shards copied into the
# staging and results copied out on the context's helper threads (rs_codec.cpp CopyPool)

def _c_oneshot(rs):
    import ctypes
    lib = rs._lib
    u64, vp = ctypes.c_uint64, ctypes.c_void_p
    lib.rs_encode.restype = ctypes.c_int
    lib.rs_encode.argtypes = [vp, u64, u64, u64, vp, u64, vp, vp]
    lib.rs_decode.restype = ctypes.c_int
    lib.rs_decode.argtypes = [vp, u64, u64, u64, vp, vp, u64, vp, vp, u64, vp, vp, vp]
    return lib


def _ptrs(rows):
    import ctypes
    return (ctypes.c_void_p * max(1, len(rows)))(*[r.ctypes.data for r in rows])


@pytest.mark.parametrize("N,M,S", [(1024, 1024, 1024), (3, 5, 64), (300, 200, 130), (100, 1000, 256), (5000, 300, 64),
                                   (1000, 2000, 130)])
def test_c_oneshot_matches_oracle(torch, rs, N, M, S):
    import ctypes
    lib = _c_oneshot(rs)
    ctx = rs.default_context().handle
    orig = O.generate_original(N, S, (N + M) & 0xFF)
    want = O.encode("default", orig, M)
    rows = [np.ascontiguousarray(orig[i]) for i in range(N)]
    out = np.full((M, S), 0xEE, np.uint8)
    err = rs._RsError()
    for _ in range(2):  # the second call reuses the pooled working space
        assert lib.rs_encode(ctx, N, M, S, _ptrs(rows), N, out.ctypes.data, ctypes.byref(err)) == 0
        assert_rows_equal(out, want, "rs_encode")
    rng = np.random.default_rng(N + 3 * M)
    L = max(1, min(N, M) // 3)
    lost = np.sort(rng.choice(N, L, replace=False))
    have = np.setdiff1d(np.arange(N), lost)
    ridx = np.sort(rng.choice(M, L, replace=False)).astype(np.uint64)
    oidx = have.astype(np.uint64)
    rrows = [np.ascontiguousarray(want[i]) for i in ridx]
    orows = [rows[i] for i in have]
    rest = np.full((N, S), 0x33, np.uint8)
    mask = np.zeros(N, np.uint8)
    assert lib.rs_decode(ctx, N, M, S, oidx.ctypes.data, _ptrs(orows), len(orows), ridx.ctypes.data, _ptrs(rrows),
                         len(rrows), rest.ctypes.data, mask.ctypes.data, ctypes.byref(err)) == 0
    assert np.array_equal(np.flatnonzero(mask), lost)
    assert_rows_equal(rest[lost], orig[lost], "rs_decode")
    assert np.all(rest[have] == 0x33)
    # the reference's error order survives the checks-first / copies-after split
    dup = np.array([oidx[0], oidx[min(1, len(oidx) - 1)], oidx[0]], np.uint64)  # (a duplicate by the 3rd at the latest)
    dup_rows = [orows[0], orows[min(1, len(orows) - 1)], orows[0]]
    assert lib.rs_decode(ctx, N, M, S, dup.ctypes.data, _ptrs(dup_rows), 3, ridx.ctypes.data, _ptrs(rrows),
                         len(rrows), rest.ctypes.data, mask.ctypes.data, ctypes.byref(err)) == 2  # duplicate original
    bad = np.array([N], np.uint64)
    assert lib.rs_decode(ctx, N, M, S, bad.ctypes.data, _ptrs(orows[:1]), 1, ridx.ctypes.data, _ptrs(rrows),
                         len(rrows), rest.ctypes.data, mask.ctypes.data, ctypes.byref(err)) == 4  # invalid index
    assert err.index == N
    extra = rows + rows[:1]
    assert lib.rs_encode(ctx, N, M, S, _ptrs(extra), N + 1, out.ctypes.data, ctypes.byref(err)) == 9  # too many
    assert lib.rs_encode(ctx, N, M, S, _ptrs(rows), N - 1 if N > 1 else 0, out.ctypes.data,
                         ctypes.byref(err)) == 8  # too few
    nul = _ptrs(rows)
    nul[N // 2] = None  # a null shard pointer: the checked path's invalid-argument code
    assert lib.rs_encode(ctx, N, M, S, nul, N, out.ctypes.data, ctypes.byref(err)) == 101
    onul = _ptrs(orows)
    onul[0] = None
    assert lib.rs_decode(ctx, N, M, S, oidx.ctypes.data, onul, len(orows), ridx.ctypes.data, _ptrs(rrows),
                         len(rrows), rest.ctypes.data, mask.ctypes.data, ctypes.byref(err)) == 101
    # and the context still encodes afterwards
    assert lib.rs_encode(ctx, N, M, S, _ptrs(rows), N, out.ctypes.data, ctypes.byref(err)) == 0
    assert_rows_equal(out, want, "rs_encode after errors")
