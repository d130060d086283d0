"""CPU-only checks of the product library (no GPU calls).

* the C-ABI library loads and exports every function include/rs_mi355x.h declares;
* its GF tables equal the oracle's (reference tables.rs semantics);
* the byte-permute multiply format used by the HIP kernels, emulated here in
  numpy exactly as rs_kernels.hip gf_muladd4 computes it, equals the oracle's
  scalar multiply (reference tables.rs:172-178);
* the reduced 2^u-point eval_poly of k_eval_poly, emulated in numpy, equals the
  oracle's full 65536-point eval_poly (reference utils.rs:20-31) on the values
  the decoder uses;
* rate selection / support / validation / work counts (reference rate tests).
"""
import ctypes
import os
import re

import numpy as np
import pytest

import oracle_lib as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "rs_mi355x.h")


@pytest.fixture(scope="module")
def rs():
    import reed_solomon_simd
    return reed_solomon_simd


def test_library_exports_every_header_symbol(rs):
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    names = set(re.findall(r"\b(rs_[a-z0-9_]+)\s*\(", text))
    assert len(names) > 40
    missing = [n for n in sorted(names) if not hasattr(rs._lib, n)]
    assert not missing, missing


def test_tables_match_oracle(rs):
    for name, n in (("exp", 65536), ("log", 65536), ("skew", 65535), ("log_walsh", 65536)):
        assert np.array_equal(rs.table(name, n), O.table(name, n)), name


def _perm(s0, s1, sel):
    """v_perm_b32 for selector bytes 0..7: byte k of {s0:s1}."""
    both = (s0.astype(np.uint64) << 32) | s1.astype(np.uint64)
    out = np.zeros_like(sel, dtype=np.uint32)
    for b in range(4):
        k = (sel >> (8 * b)) & 0xFF
        assert np.all(k < 8)
        out |= (((both >> (8 * k.astype(np.uint64))) & 0xFF).astype(np.uint32)) << (8 * b)
    return out


def _mul4(t, xl, xh):
    """numpy restatement of rs_kernels.hip gf_muladd4 with acc = 0."""
    t = t.astype(np.uint32)
    l0, l1, l2 = xl & 0x07070707, (xl >> 3) & 0x07070707, (xl >> 6) & 0x03030303
    h0, h1, h2 = xh & 0x07070707, (xh >> 3) & 0x07070707, (xh >> 6) & 0x03030303
    pl = (_perm(t[1], t[0], l0) ^ _perm(t[3], t[2], l1) ^ _perm(t[4], t[4], l2) ^ _perm(t[11], t[10], h0)
          ^ _perm(t[13], t[12], h1) ^ _perm(t[14], t[14], h2))
    ph = (_perm(t[6], t[5], l0) ^ _perm(t[8], t[7], l1) ^ _perm(t[9], t[9], l2) ^ _perm(t[16], t[15], h0)
          ^ _perm(t[18], t[17], h1) ^ _perm(t[19], t[19], h2))
    return pl, ph


def test_perm_multiply_format_matches_oracle(rs):
    perm = np.ctypeslib.as_array(rs._lib.rs_table_perm_by_log(), shape=(65536 * 20,)).reshape(65536, 20)
    rng = np.random.default_rng(7)
    logs = np.concatenate([[0, 1, 65534, 65535], rng.integers(0, 65536, 60)])
    for lm in logs:
        x = rng.integers(0, 65536, 4096, dtype=np.uint32)
        x[:3] = [0, 1, 65535]
        lo, hi = x & 0xFF, x >> 8
        xl = (lo[0::4] | lo[1::4] << 8 | lo[2::4] << 16 | lo[3::4] << 24).astype(np.uint32)
        xh = (hi[0::4] | hi[1::4] << 8 | hi[2::4] << 16 | hi[3::4] << 24).astype(np.uint32)
        pl, ph = _mul4(perm[lm], xl, xh)
        got = np.zeros_like(x)
        for k in range(4):
            got[k::4] = ((pl >> (8 * k)) & 0xFF) | (((ph >> (8 * k)) & 0xFF) << 8)
        want = np.array([O.lib().orc_gf_mul(int(v), int(lm)) for v in x], dtype=np.uint32)
        assert np.array_equal(got, want), int(lm)


def test_skew_tables_zero_means_no_multiply(rs):
    sk = np.ctypeslib.as_array(rs._lib.rs_table_perm_by_skew(), shape=(65536 * 20,)).reshape(65536, 20)
    bl = np.ctypeslib.as_array(rs._lib.rs_table_perm_by_log(), shape=(65536 * 20,)).reshape(65536, 20)
    skew = O.table("skew", 65535)
    zero = np.where(skew == 65535)[0]
    assert len(zero) > 0
    assert not sk[zero].any()
    idx = np.where(skew != 65535)[0][:2000]
    assert np.array_equal(sk[idx], bl[skew[idx]])


def _walsh(v):
    v = v.astype(np.int64).copy()
    h = 1
    while h < len(v):
        v = v.reshape(-1, 2, h)
        a, b = v[:, 0, :].copy(), v[:, 1, :].copy()
        v[:, 0, :], v[:, 1, :] = (a + b) % 65535, (a - b) % 65535
        v = v.reshape(-1)
        h *= 2
    return v


def _reduced_eval(e_vec_low, u, low_rate, end, lw):
    """numpy restatement of k_eval_poly (rs_kernels.hip)."""
    n = 1 << u
    fold = lw.astype(np.int64).reshape(-1, n).sum(axis=0) % 65535
    if low_rate:
        v = np.where(np.arange(n) < end, np.where(e_vec_low == 1, 0, 65534), 0)
    else:
        v = e_vec_low.astype(np.int64)
    f = _walsh(v)
    p = (f * fold) % 65535
    if low_rate:
        p[0] = (p[0] + int(lw[0])) % 65535
    return _walsh(p)


@pytest.mark.parametrize("high,N,M", [(1, 3, 2), (1, 100, 37), (1, 1000, 1000), (0, 2, 3), (0, 37, 100),
                                      (0, 1000, 3000), (1, 61440, 4096)])
def test_reduced_eval_poly_matches_full(high, N, M):
    rng = np.random.default_rng(N * 7 + M)
    lw = O.table("log_walsh", 65536)
    p2 = lambda x: 1 << (x - 1).bit_length()
    chunk = p2(M) if high else p2(N)
    end = chunk + (N if high else M)
    nd = p2(end)
    u = nd.bit_length() - 1
    er = np.zeros(65536, np.uint16)
    miss = rng.random(end) < 0.3
    if high:
        er[:M] = miss[:M]
        er[M:chunk] = 1
        er[chunk:end] = miss[chunk:end]
    else:
        er[:N] = miss[:N]
        er[chunk:end] = miss[chunk:end]
        er[end:] = 1
    full = er.copy()
    O.lib().orc_eval_poly(O.ptr(full), 65536)
    red = _reduced_eval(er[:nd], u, not high, end, lw)
    # compare as residues mod 65535 (0 and 65535 are the same residue; both mean x1)
    assert np.array_equal(full[:nd].astype(np.int64) % 65535, red % 65535)


def test_host_eval_poly_matches_oracle(rs):
    rng = np.random.default_rng(3)
    er = (rng.random(65536) < 0.1).astype(np.uint16)
    er[5000:] = 0
    want = er.copy()
    O.lib().orc_eval_poly(O.ptr(want), 5000)
    got = rs.engine.eval_poly(er.copy(), 5000)
    assert np.array_equal(got, want)


def test_rate_selection(rs):
    M = 2**64 - 1
    for n, m, want in ((0, 1, -1), (1, 0, -1), (3, 3, 1), (3, 4, 1), (3, 5, 0), (4, 3, 0), (5, 3, 1),
                       (4096, 61440, 0), (4096, 61441, -1), (4097, 61440, -1), (61440, 4096, 1),
                       (61440, 4097, -1), (61441, 4096, -1), (M, M, -1)):
        assert rs.use_high_rate(n, m) == want


def test_supports_and_validate(rs):
    H, L = rs.rate.HighRateEncoder, rs.rate.LowRateEncoder
    # rate_high.rs:476-489 / rate_low.rs equivalents
    assert not H.supports(0, 1) and not H.supports(1, 0)
    assert not H.supports(4096, 61440) and H.supports(61440, 4096)
    assert not H.supports(61440, 4097) and not H.supports(61441, 4096)
    assert L.supports(4096, 61440) and not L.supports(61440, 4096)
    assert rs.ReedSolomonEncoder.supports(4096, 61440) and rs.ReedSolomonEncoder.supports(61440, 4096)
    with pytest.raises(rs.InvalidShardSize) as e:
        H.validate(1, 1, 123)
    assert e.value == rs.InvalidShardSize(shard_bytes=123)
    with pytest.raises(rs.UnsupportedShardCount) as e:
        H.validate(4096, 61440, 64)
    assert e.value == rs.UnsupportedShardCount(original_count=4096, recovery_count=61440)
    H.validate(61440, 4096, 64)


def test_work_counts(rs):
    HE, HD = rs.rate.HighRateEncoder, rs.rate.HighRateDecoder
    # rate_high.rs:560-567, 618-626
    assert [HE.work_count(*x) for x in ((1, 1), (4096, 1024), (4097, 1024), (4097, 1025), (32768, 32768))] == \
        [1, 4096, 5120, 6144, 32768]
    assert [HD.work_count(*x) for x in ((1, 1), (2048, 1025), (2049, 1025), (3072, 1024), (3073, 1024),
                                         (32768, 32768))] == [2, 4096, 8192, 4096, 8192, 65536]
    LE, LD = rs.rate.LowRateEncoder, rs.rate.LowRateDecoder
    assert [LE.work_count(*x) for x in ((1, 1), (1024, 4096), (1024, 4097), (1025, 4097), (32768, 32768))] == \
        [1, 4096, 5120, 6144, 32768]
    assert [LD.work_count(*x) for x in ((1, 1), (1025, 2048), (1025, 2049), (1024, 3072), (1024, 3073),
                                         (32768, 32768))] == [2, 4096, 8192, 4096, 8192, 65536]


def test_python_binding_declares_every_signature():
    """Every C function the Python mirror calls has ctypes argtypes/restype declared
    (an undeclared one silently truncates 64-bit pointers to int)."""
    import re
    import reed_solomon_simd as rs
    src = open(rs.__file__).read()
    used = set(re.findall(r"_lib\.(rs_\w+)", src))
    assert used
    for name in sorted(used):
        f = getattr(rs._lib, name)
        assert f.argtypes is not None, f"{name} has no declared argtypes"


def test_batch_entry_points_validate_before_any_device_work(rs):
    """rs_*_device_batch reject bad arguments like the single-stripe calls (no GPU needed)."""
    import ctypes
    err = rs._RsError()
    # null context / pointers
    assert rs._lib.rs_encode_device_batch(None, 0, 1024, 1024, 1024, 3, 0, 0, 0, 0, 0, 0, None,
                                          ctypes.byref(err)) == 101
    op = bytes([1] * 4)
    assert rs._lib.rs_decode_device_batch(None, 0, 4, 4, 64, 2, 0, 0, 0, op, 0, 0, 0, op, 0, 0, 0, None,
                                          ctypes.byref(err)) == 101


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="a GPU is present on this host")
def test_no_cpu_fallback_without_a_gpu(rs):
    """The product path has no CPU fallback: with no device every compute entry point
    (one-shot API, encoder objects, device context) raises DeviceError instead of computing."""
    with pytest.raises(rs.DeviceError):
        rs.Context()
    with pytest.raises(rs.DeviceError):
        rs.encode(3, 5, [bytes(64)] * 3)
    with pytest.raises(rs.DeviceError):
        rs.ReedSolomonEncoder(3, 5, 64)
