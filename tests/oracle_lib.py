"""ctypes handle on the CPU oracle (test infrastructure; oracle/rs_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ODIR = os.path.join(ROOT, "oracle")
SO = os.path.join(ODIR, "_build", "liboracle.so")


RATES = {"default": 0, "high": 1, "low": 2}
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ODIR], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(SO):
            build()
        _lib = ctypes.CDLL(SO)
        sz = ctypes.c_size_t
        vp = ctypes.c_void_p
        _lib.orc_generate_original.argtypes = [sz, sz, ctypes.c_uint8, vp]
        _lib.orc_encode.argtypes = [ctypes.c_int, sz, sz, sz, vp, vp]
        _lib.orc_decode.argtypes = [ctypes.c_int, sz, sz, sz, vp, vp, vp, vp, vp]
        _lib.orc_fft.argtypes = [vp, sz, sz, sz, sz, sz]
        _lib.orc_ifft.argtypes = [vp, sz, sz, sz, sz, sz]
        _lib.orc_mul.argtypes = [vp, sz, ctypes.c_uint16]
        _lib.orc_formal_derivative.argtypes = [vp, sz, sz]
        _lib.orc_eval_poly.argtypes = [vp, sz]
        _lib.orc_use_high_rate.argtypes = [sz, sz]
        _lib.orc_select_engine.argtypes = [ctypes.c_int]
        for t in ("exp", "log", "skew", "log_walsh"):
            getattr(_lib, f"orc_{t}_table").restype = ctypes.POINTER(ctypes.c_uint16)
    return _lib


def ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def table(name, n):
    return np.ctypeslib.as_array(getattr(lib(), f"orc_{name}_table")(), shape=(n,)).copy()


def generate_original(count, shard_bytes, seed):
    out = np.zeros((count, shard_bytes), np.uint8)
    lib().orc_generate_original(count, shard_bytes, seed, ptr(out))
    return out


def encode(rate, orig, recovery_count):
    n, s = orig.shape
    rec = np.zeros((recovery_count, s), np.uint8)
    err = lib().orc_encode(RATES[rate], n, recovery_count, s, ptr(np.ascontiguousarray(orig)), ptr(rec))
    if err:
        raise RuntimeError(f"oracle encode error {err}")
    return rec


def decode(rate, orig, orig_present, rec, rec_present):
    n, s = orig.shape
    m = rec.shape[0]
    out = np.zeros((n, s), np.uint8)
    op = np.asarray(orig_present, np.uint8)
    rp = np.asarray(rec_present, np.uint8)
    err = lib().orc_decode(RATES[rate], n, m, s, ptr(np.ascontiguousarray(orig)), ptr(op),
                           ptr(np.ascontiguousarray(rec)), ptr(rp), ptr(out))
    if err:
        raise RuntimeError(f"oracle decode error {err}")
    return out


def ranges_mask(ranges, count):
    m = np.zeros(count, np.uint8)
    for a, b in ranges:
        m[a:b] = 1
    return m
