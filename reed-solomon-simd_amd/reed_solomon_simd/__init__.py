"""reed_solomon_simd -- MI355X-native drop-in for the reed-solomon-simd API.

Python mirror of the reference crate's public interface (AndersTrier/
reed-solomon-simd v3.1.0, /root/reference):

    encode(original_count, recovery_count, original)            src/lib.rs:251-290
    decode(original_count, recovery_count, original, recovery)  src/lib.rs:292-353
    ReedSolomonEncoder / ReedSolomonDecoder                      src/reed_solomon.rs
    EncoderResult / DecoderResult                                src/encoder_result.rs, decoder_result.rs
    Error (one subclass per variant, same fields)               src/lib.rs:48-231
    rate.{DefaultRate, HighRate, LowRate}{Encoder,Decoder}       src/rate/*.rs

plus the device-resident batch path `encode_device` / `decode_device` that
works on HIP device pointers (e.g. torch tensors on cuda:0).

Everything runs through the C ABI of librs_mi355x.so (include/rs_mi355x.h);
there is no CPU fallback: importing fails loudly if the library is missing.
"""
from __future__ import annotations

import ctypes
import os
from typing import Dict, Iterable, List, Optional, Tuple

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(os.path.dirname(_HERE), "lib", "librs_mi355x.so")

if not os.path.exists(LIB_PATH):
    raise ImportError(
        f"{LIB_PATH} not built; run `python -c 'import __graft_entry__ as g; g.build()'` (HIP extension required)"
    )

_lib = ctypes.CDLL(LIB_PATH)

_u64 = ctypes.c_uint64
_vp = ctypes.c_void_p
_int = ctypes.c_int


class _RsError(ctypes.Structure):
    _fields_ = [
        ("code", ctypes.c_int32),
        ("original_count", _u64),
        ("recovery_count", _u64),
        ("shard_bytes", _u64),
        ("got", _u64),
        ("index", _u64),
        ("original_received_count", _u64),
        ("recovery_received_count", _u64),
    ]


_E = ctypes.POINTER(_RsError)


def _sig(name, restype, *args):
    f = getattr(_lib, name)
    f.restype = restype
    f.argtypes = list(args)
    return f


_sig("rs_context_create", _int, _int, ctypes.POINTER(_vp))
_sig("rs_context_destroy", None, _vp)
_sig("rs_last_device_error", ctypes.c_char_p)
_sig("rs_version", ctypes.c_char_p)
_sig("rs_supports", _int, _int, _u64, _u64)
_sig("rs_use_high_rate", _int, _u64, _u64)
_sig("rs_validate", _int, _int, _u64, _u64, _u64, _E)
_sig("rs_encoder_work_count", _u64, _int, _u64, _u64)
_sig("rs_decoder_work_count", _u64, _int, _u64, _u64)
_sig("rs_encoder_new", _int, _vp, _int, _u64, _u64, _u64, ctypes.POINTER(_vp), _E)
_sig("rs_encoder_reset", _int, _vp, _u64, _u64, _u64, _E)
_sig("rs_encoder_add_original_shard", _int, _vp, ctypes.c_char_p, _u64, _E)
_sig("rs_encoder_encode", _int, _vp, _E)
_sig("rs_encoder_recovery", ctypes.POINTER(ctypes.c_uint8), _vp, _u64)
_sig("rs_encoder_result_drop", None, _vp)
_sig("rs_encoder_is_high_rate", _int, _vp)
_sig("rs_encoder_free", None, _vp)
_sig("rs_decoder_new", _int, _vp, _int, _u64, _u64, _u64, ctypes.POINTER(_vp), _E)
_sig("rs_encoder_new_with_work", _int, _vp, _int, _u64, _u64, _u64, _vp, ctypes.POINTER(_vp), _E)
_sig("rs_decoder_new_with_work", _int, _vp, _int, _u64, _u64, _u64, _vp, ctypes.POINTER(_vp), _E)
_sig("rs_encoder_into_parts", _int, _vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp))
_sig("rs_decoder_into_parts", _int, _vp, ctypes.POINTER(_vp), ctypes.POINTER(_vp))
_sig("rs_encoder_work_free", None, _vp)
_sig("rs_decoder_work_free", None, _vp)
_sig("rs_decoder_reset", _int, _vp, _u64, _u64, _u64, _E)
_sig("rs_decoder_add_original_shard", _int, _vp, _u64, ctypes.c_char_p, _u64, _E)
_sig("rs_decoder_add_recovery_shard", _int, _vp, _u64, ctypes.c_char_p, _u64, _E)
_sig("rs_decoder_decode", _int, _vp, _E)
_sig("rs_decoder_restored_original", ctypes.POINTER(ctypes.c_uint8), _vp, _u64)
_sig("rs_decoder_restored_count", _u64, _vp)
_sig("rs_decoder_result_drop", None, _vp)
_sig("rs_decoder_is_high_rate", _int, _vp)
_sig("rs_decoder_free", None, _vp)
_sig("rs_encode_device", _int, _vp, _int, _u64, _u64, _u64, _vp, _vp, _vp, _E)
_sig("rs_decode_device", _int, _vp, _int, _u64, _u64, _u64, _vp, ctypes.c_char_p, _vp, ctypes.c_char_p, _vp, _vp, _E)
_sig("rs_encode_device_strided", _int, _vp, _int, _u64, _u64, _u64, _vp, _u64, _vp, _u64, _vp, _E)
_sig("rs_decode_device_strided", _int, _vp, _int, _u64, _u64, _u64, _vp, _u64, ctypes.c_char_p, _vp, _u64,
     ctypes.c_char_p, _vp, _u64, _vp, _E)
_sig("rs_encode_device_batch", _int, _vp, _int, _u64, _u64, _u64, _u64, _vp, _u64, _u64, _vp, _u64, _u64, _vp, _E)
_sig("rs_decode_device_batch", _int, _vp, _int, _u64, _u64, _u64, _u64, _vp, _u64, _u64, ctypes.c_char_p, _vp, _u64,
     _u64, ctypes.c_char_p, _vp, _u64, _u64, _vp, _E)
_sig("rs_engine_fft", _int, _vp, _vp, _u64, _u64, _u64, _u64, _u64, _u64, _vp)
_sig("rs_engine_ifft", _int, _vp, _vp, _u64, _u64, _u64, _u64, _u64, _u64, _vp)
_sig("rs_engine_mul", _int, _vp, _vp, _u64, ctypes.c_uint16, _vp)
_sig("rs_engine_eval_poly", None, ctypes.POINTER(ctypes.c_uint16), _u64)
_sig("rs_engine_formal_derivative", _int, _vp, _vp, _u64, _u64, _vp)
_sig("rs_engine_fft_host", _int, _vp, _vp, _u64, _u64, _u64, _u64, _u64, _u64)
_sig("rs_engine_ifft_host", _int, _vp, _vp, _u64, _u64, _u64, _u64, _u64, _u64)
_sig("rs_engine_mul_host", _int, _vp, _vp, _u64, ctypes.c_uint16)
for _t in ("exp", "log", "skew", "log_walsh"):
    _sig(f"rs_table_{_t}", ctypes.POINTER(ctypes.c_uint16))
for _t in ("perm_by_log", "perm_by_skew"):
    _sig(f"rs_table_{_t}", ctypes.POINTER(ctypes.c_uint32))
_sig("rs_profile_enable", _int, _vp, _int)
_sig("rs_profile_collect", _int, _vp, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(_u64),
     ctypes.POINTER(ctypes.c_char_p), _int)


def profile_enable(enable: bool = True, ctx=None) -> None:
    """Bracket every kernel launch of `ctx` with HIP events (bench instrumentation)."""
    ctx = ctx or default_context()
    _lib.rs_profile_enable(ctx.handle, 1 if enable else 0)


def profile_collect(ctx=None, max_records: int = 1 << 16):
    """[(kernel_name, ms, algorithmic_bytes)] of the launches since the last collect."""
    ctx = ctx or default_context()
    ms = (ctypes.c_float * max_records)()
    by = (_u64 * max_records)()
    nm = (ctypes.c_char_p * max_records)()
    n = _lib.rs_profile_collect(ctx.handle, ms, by, nm, max_records)
    return [(nm[i].decode(), float(ms[i]), int(by[i])) for i in range(max(n, 0))]


_sig("rs_check_device", _int, _vp)


_sig("rs_mono_enable", _int, _vp, _int)
_sig("rs_release_stream_scratch", _int, _vp, _vp)


def release_stream_scratch(stream=None, ctx=None) -> None:
    """Synchronize `stream` and free the context's device scratch for it (rs_release_stream_scratch)."""
    ctx = ctx or default_context()
    st = _lib.rs_release_stream_scratch(ctx.handle, _stream(stream))
    if st != 0:
        raise DeviceError(_lib.rs_last_device_error().decode())


def mono_enable(enable=True, ctx=None) -> None:
    """Column kernel (one workgroup per pack): False = never, True = where fastest (default),
    2 = also multi-chunk and 2^11 / 2^12-row transforms; + 4 no split decode plan, + 8 4-element
    packs only, + 16 2-element packs everywhere (rs_mono_enable)."""
    ctx = ctx or default_context()
    _lib.rs_mono_enable(ctx.handle, int(enable))


def check_device(ctx=None) -> None:
    """Synchronize the context's device; raise DeviceError if an earlier asynchronous launch failed."""
    ctx = ctx or default_context()
    st = _lib.rs_check_device(ctx.handle)
    if st != 0:
        raise DeviceError(_lib.rs_last_device_error().decode())

GF_BITS = 16
GF_ORDER = 65536
GF_MODULUS = 65535

RATE_DEFAULT, RATE_HIGH, RATE_LOW = 0, 1, 2


# ---------------------------------------------------------------------------
# Errors (src/lib.rs:48-142)

class Error(Exception):
    """Base of the reference's `Error` variants; fields as attributes."""

    fields: Tuple[str, ...] = ()

    def __init__(self, **kw):
        for f in self.fields:
            setattr(self, f, kw.get(f))
        super().__init__(self._msg())

    def _msg(self):
        return type(self).__name__

    def __eq__(self, other):
        return type(self) is type(other) and all(getattr(self, f) == getattr(other, f) for f in self.fields)

    def __hash__(self):
        return hash((type(self).__name__,) + tuple(getattr(self, f) for f in self.fields))

    def __repr__(self):
        return f"{type(self).__name__}({', '.join(f'{f}={getattr(self, f)}' for f in self.fields)})"


class DifferentShardSize(Error):
    fields = ("shard_bytes", "got")

    def _msg(self):
        return f"different shard size: expected {self.shard_bytes} bytes, got {self.got} bytes"


class DuplicateOriginalShardIndex(Error):
    fields = ("index",)

    def _msg(self):
        return f"duplicate original shard index: {self.index}"


class DuplicateRecoveryShardIndex(Error):
    fields = ("index",)

    def _msg(self):
        return f"duplicate recovery shard index: {self.index}"


class InvalidOriginalShardIndex(Error):
    fields = ("original_count", "index")

    def _msg(self):
        return f"invalid original shard index: {self.index} >= original_count {self.original_count}"


class InvalidRecoveryShardIndex(Error):
    fields = ("recovery_count", "index")

    def _msg(self):
        return f"invalid recovery shard index: {self.index} >= recovery_count {self.recovery_count}"


class InvalidShardSize(Error):
    fields = ("shard_bytes",)

    def _msg(self):
        return f"invalid shard size: {self.shard_bytes} bytes (must non-zero and multiple of 2)"


class NotEnoughShards(Error):
    fields = ("original_count", "original_received_count", "recovery_received_count")

    def _msg(self):
        return (f"not enough shards: {self.original_received_count} original + {self.recovery_received_count} "
                f"recovery < {self.original_count} original_count")


class TooFewOriginalShards(Error):
    fields = ("original_count", "original_received_count")

    def _msg(self):
        return (f"too few original shards: got {self.original_received_count} shards while original_count is "
                f"{self.original_count}")


class TooManyOriginalShards(Error):
    fields = ("original_count",)

    def _msg(self):
        return f"too many original shards: got more than original_count ({self.original_count}) shards"


class UnsupportedShardCount(Error):
    fields = ("original_count", "recovery_count")

    def _msg(self):
        return (f"unsupported shard count: {self.original_count} original shards with {self.recovery_count} "
                f"recovery shards")


class DeviceError(RuntimeError):
    pass


_BY_CODE = {1: DifferentShardSize, 2: DuplicateOriginalShardIndex, 3: DuplicateRecoveryShardIndex,
            4: InvalidOriginalShardIndex, 5: InvalidRecoveryShardIndex, 6: InvalidShardSize, 7: NotEnoughShards,
            8: TooFewOriginalShards, 9: TooManyOriginalShards, 10: UnsupportedShardCount}


def _raise(code: int, err: _RsError):
    if code == 0:
        return
    cls = _BY_CODE.get(code)
    if cls is not None:
        raise cls(**{f: int(getattr(err, f)) for f in cls.fields})
    if code == 100:
        raise DeviceError(_lib.rs_last_device_error().decode())
    raise ValueError(f"invalid argument (rs_status {code})")


# ---------------------------------------------------------------------------
# Context: one per device (GF tables live in HBM)

class Context:
    def __init__(self, device: int = 0):
        h = _vp()
        code = _lib.rs_context_create(device, ctypes.byref(h))
        if code:
            raise DeviceError(_lib.rs_last_device_error().decode())
        self._h = h
        self.device = device

    @property
    def handle(self):
        return self._h

    def close(self):
        if self._h:
            _lib.rs_context_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_default_ctx: Dict[int, Context] = {}


def default_context(device: int = 0) -> Context:
    if device not in _default_ctx:
        _default_ctx[device] = Context(device)
    return _default_ctx[device]


def version() -> str:
    return _lib.rs_version().decode()


# ---------------------------------------------------------------------------
# Encoder / decoder objects (src/reed_solomon.rs, src/rate.rs)

class EncoderResult:
    """Borrowed view of the recovery shards (src/encoder_result.rs)."""

    def __init__(self, enc: "_EncoderBase"):
        self._enc = enc
        self._alive = True

    def recovery(self, index: int) -> Optional[bytes]:
        if not self._alive:
            raise RuntimeError("EncoderResult used after drop")
        p = _lib.rs_encoder_recovery(self._enc._h, index)
        if not p:
            return None
        return ctypes.string_at(p, self._enc.shard_bytes)

    def recovery_iter(self):
        i = 0
        while True:
            r = self.recovery(i)
            if r is None:
                return
            yield r
            i += 1

    def drop(self):
        """EncoderResult::drop -> reset_received (encoder_result.rs:48-52)."""
        if self._alive:
            self._alive = False
            _lib.rs_encoder_result_drop(self._enc._h)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.drop()

    def __del__(self):
        try:
            self.drop()
        except Exception:
            pass


class DecoderResult:
    """Borrowed view of the restored originals (src/decoder_result.rs)."""

    def __init__(self, dec: "_DecoderBase"):
        self._dec = dec
        self._alive = True

    def restored_original(self, index: int) -> Optional[bytes]:
        if not self._alive:
            raise RuntimeError("DecoderResult used after drop")
        p = _lib.rs_decoder_restored_original(self._dec._h, index)
        if not p:
            return None
        return ctypes.string_at(p, self._dec.shard_bytes)

    def restored_original_iter(self):
        for i in range(self._dec.original_count):
            r = self.restored_original(i)
            if r is not None:
                yield i, r

    def __len__(self):
        return int(_lib.rs_decoder_restored_count(self._dec._h))

    def drop(self):
        if self._alive:
            self._alive = False
            _lib.rs_decoder_result_drop(self._dec._h)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.drop()

    def __del__(self):
        try:
            self.drop()
        except Exception:
            pass


class _Work:
    """EncoderWork / DecoderWork (src/rate.rs:129-131, 206-208): the buffers of a consumed
    encoder / decoder (into_parts), reusable by a new one of any rate and shape (work=...)."""
    _FREE = None

    def __init__(self, handle):
        self._h = handle

    def _take(self):
        h, self._h = self._h, None
        if h is None:
            raise ValueError("this work object was already handed to an encoder / decoder")
        return h

    def __del__(self):
        try:
            if self._h:
                getattr(_lib, self._FREE)(self._h)
                self._h = None
        except Exception:
            pass


class EncoderWork(_Work):
    _FREE = "rs_encoder_work_free"


class DecoderWork(_Work):
    _FREE = "rs_decoder_work_free"


class _EncoderBase:
    RATE = RATE_DEFAULT

    def __init__(self, original_count: int, recovery_count: int, shard_bytes: int, ctx: Optional[Context] = None,
                 work: Optional[EncoderWork] = None):
        self._ctx = ctx or default_context()
        h = _vp()
        err = _RsError()
        w = work._take() if work is not None else None  # consumed in every case (rate_high.rs:93-103)
        code = _lib.rs_encoder_new_with_work(self._ctx.handle, self.RATE, original_count, recovery_count,
                                             shard_bytes, w, ctypes.byref(h), ctypes.byref(err))
        _raise(code, err)
        self._h = h
        self.original_count, self.recovery_count, self.shard_bytes = original_count, recovery_count, shard_bytes
        self._result: Optional[EncoderResult] = None

    @classmethod
    def supports(cls, original_count: int, recovery_count: int) -> bool:
        return bool(_lib.rs_supports(cls.RATE, original_count, recovery_count))

    @classmethod
    def validate(cls, original_count: int, recovery_count: int, shard_bytes: int) -> None:
        err = _RsError()
        _raise(_lib.rs_validate(cls.RATE, original_count, recovery_count, shard_bytes, ctypes.byref(err)), err)

    @classmethod
    def work_count(cls, original_count: int, recovery_count: int) -> int:
        return int(_lib.rs_encoder_work_count(cls.RATE, original_count, recovery_count))

    def _drop_result(self):
        if self._result is not None:
            self._result.drop()
            self._result = None

    def add_original_shard(self, shard) -> None:
        self._drop_result()
        b = bytes(shard)
        err = _RsError()
        _raise(_lib.rs_encoder_add_original_shard(self._h, b, len(b), ctypes.byref(err)), err)

    def encode(self) -> EncoderResult:
        err = _RsError()
        _raise(_lib.rs_encoder_encode(self._h, ctypes.byref(err)), err)
        self._result = EncoderResult(self)
        return self._result

    def reset(self, original_count: int, recovery_count: int, shard_bytes: int) -> None:
        self._drop_result()
        err = _RsError()
        _raise(_lib.rs_encoder_reset(self._h, original_count, recovery_count, shard_bytes, ctypes.byref(err)), err)
        self.original_count, self.recovery_count, self.shard_bytes = original_count, recovery_count, shard_bytes

    @property
    def is_high_rate(self) -> bool:
        return bool(_lib.rs_encoder_is_high_rate(self._h))

    def into_parts(self):
        """RateEncoder::into_parts (src/rate.rs:129-131): consumes this encoder, returns
        (engine context, EncoderWork)."""
        self._drop_result()
        w = _vp()
        _lib.rs_encoder_into_parts(self._h, None, ctypes.byref(w))
        self._h = None
        return self._ctx, EncoderWork(w)

    def __del__(self):
        try:
            if self._h:
                _lib.rs_encoder_free(self._h)
                self._h = None
        except Exception:
            pass


class _DecoderBase:
    RATE = RATE_DEFAULT

    def __init__(self, original_count: int, recovery_count: int, shard_bytes: int, ctx: Optional[Context] = None,
                 work: Optional[DecoderWork] = None):
        self._ctx = ctx or default_context()
        h = _vp()
        err = _RsError()
        w = work._take() if work is not None else None
        code = _lib.rs_decoder_new_with_work(self._ctx.handle, self.RATE, original_count, recovery_count,
                                             shard_bytes, w, ctypes.byref(h), ctypes.byref(err))
        _raise(code, err)
        self._h = h
        self.original_count, self.recovery_count, self.shard_bytes = original_count, recovery_count, shard_bytes
        self._result: Optional[DecoderResult] = None

    supports = classmethod(lambda cls, n, m: bool(_lib.rs_supports(cls.RATE, n, m)))

    @classmethod
    def validate(cls, original_count: int, recovery_count: int, shard_bytes: int) -> None:
        err = _RsError()
        _raise(_lib.rs_validate(cls.RATE, original_count, recovery_count, shard_bytes, ctypes.byref(err)), err)

    @classmethod
    def work_count(cls, original_count: int, recovery_count: int) -> int:
        return int(_lib.rs_decoder_work_count(cls.RATE, original_count, recovery_count))

    def _drop_result(self):
        if self._result is not None:
            self._result.drop()
            self._result = None

    def add_original_shard(self, index: int, shard) -> None:
        self._drop_result()
        b = bytes(shard)
        err = _RsError()
        _raise(_lib.rs_decoder_add_original_shard(self._h, index, b, len(b), ctypes.byref(err)), err)

    def add_recovery_shard(self, index: int, shard) -> None:
        self._drop_result()
        b = bytes(shard)
        err = _RsError()
        _raise(_lib.rs_decoder_add_recovery_shard(self._h, index, b, len(b), ctypes.byref(err)), err)

    def decode(self) -> DecoderResult:
        err = _RsError()
        _raise(_lib.rs_decoder_decode(self._h, ctypes.byref(err)), err)
        self._result = DecoderResult(self)
        return self._result

    def reset(self, original_count: int, recovery_count: int, shard_bytes: int) -> None:
        self._drop_result()
        err = _RsError()
        _raise(_lib.rs_decoder_reset(self._h, original_count, recovery_count, shard_bytes, ctypes.byref(err)), err)
        self.original_count, self.recovery_count, self.shard_bytes = original_count, recovery_count, shard_bytes

    @property
    def is_high_rate(self) -> bool:
        return bool(_lib.rs_decoder_is_high_rate(self._h))

    def into_parts(self):
        """RateDecoder::into_parts (src/rate.rs:206-208): consumes this decoder, returns
        (engine context, DecoderWork)."""
        self._drop_result()
        w = _vp()
        _lib.rs_decoder_into_parts(self._h, None, ctypes.byref(w))
        self._h = None
        return self._ctx, DecoderWork(w)

    def __del__(self):
        try:
            if self._h:
                _lib.rs_decoder_free(self._h)
                self._h = None
        except Exception:
            pass


class ReedSolomonEncoder(_EncoderBase):
    """src/reed_solomon.rs:13-81 (DefaultRate + the MI355X engine)."""


class ReedSolomonDecoder(_DecoderBase):
    """src/reed_solomon.rs:83-183."""


class _RateNS:
    pass


rate = _RateNS()
for _name, _r in (("Default", RATE_DEFAULT), ("High", RATE_HIGH), ("Low", RATE_LOW)):
    setattr(rate, f"{_name}RateEncoder", type(f"{_name}RateEncoder", (_EncoderBase,), {"RATE": _r}))
    setattr(rate, f"{_name}RateDecoder", type(f"{_name}RateDecoder", (_DecoderBase,), {"RATE": _r}))


# ---------------------------------------------------------------------------
# one-shot (src/lib.rs:251-353)
#
# Each call builds an encoder / decoder as the reference does, on the working space
# the previous one-shot call left (into_parts -> work=): pinned staging, device
# buffers and stream are reused, so a call allocates (and frees) nothing when the
# shapes repeat -- a hipHostFree or hipFree per call would synchronize the device.
_oneshot_work: Dict[str, _Work] = {}

def encode(original_count: int, recovery_count: int, original: Iterable) -> List[bytes]:
    if not ReedSolomonEncoder.supports(original_count, recovery_count):
        raise UnsupportedShardCount(original_count=original_count, recovery_count=recovery_count)
    it = iter(original)
    try:
        first = bytes(next(it))
    except StopIteration:
        raise TooFewOriginalShards(original_count=original_count, original_received_count=0) from None
    enc = ReedSolomonEncoder(original_count, recovery_count, len(first), work=_oneshot_work.pop("enc", None))
    try:
        enc.add_original_shard(first)
        for s in it:
            enc.add_original_shard(s)
        res = enc.encode()
        out = list(res.recovery_iter())
        res.drop()
    finally:
        _oneshot_work["enc"] = enc.into_parts()[1]
    return out


def decode(original_count: int, recovery_count: int, original: Iterable[Tuple[int, bytes]],
           recovery: Iterable[Tuple[int, bytes]]) -> Dict[int, bytes]:
    if not ReedSolomonDecoder.supports(original_count, recovery_count):
        raise UnsupportedShardCount(original_count=original_count, recovery_count=recovery_count)
    original = list(original)
    rit = iter(recovery)
    try:
        first = next(rit)
    except StopIteration:
        if len(original) == original_count:
            return {}
        raise NotEnoughShards(original_count=original_count, original_received_count=len(original),
                              recovery_received_count=0) from None
    shard_bytes = len(bytes(first[1]))
    dec = ReedSolomonDecoder(original_count, recovery_count, shard_bytes, work=_oneshot_work.pop("dec", None))
    try:
        for i, s in original:
            dec.add_original_shard(i, s)
        dec.add_recovery_shard(first[0], first[1])
        for i, s in rit:
            dec.add_recovery_shard(i, s)
        res = dec.decode()
        out = dict(res.restored_original_iter())
        res.drop()
    finally:
        _oneshot_work["dec"] = dec.into_parts()[1]
    return out


# ---------------------------------------------------------------------------
# device-resident path (HIP device pointers; torch tensors accepted)

def _ptr(x) -> int:
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    return int(x)


def _stream(stream) -> Optional[int]:
    if stream is None:
        return None
    if hasattr(stream, "cuda_stream"):
        return stream.cuda_stream
    return int(stream)


def _row_stride(x) -> int:
    """Row stride in bytes of a 2-D uint8 tensor view (0 = contiguous / raw pointer)."""
    if hasattr(x, "stride") and callable(x.stride) and x.dim() == 2:
        if x.stride(1) != 1:
            raise ValueError("shard rows must be contiguous (stride(1) == 1)")
        return 0 if x.is_contiguous() else int(x.stride(0)) * x.element_size()
    return 0


def _check_matrix(x, rows: int, shard_bytes: int, what: str, dims: int = 2, on_device: bool = True) -> None:
    """A tensor argument must be a uint8 device tensor [.., >= rows, shard_bytes]: the kernels
    address rows * stride bytes, so an undersized tensor would be written past its end (the
    reference rejects wrong sizes with DifferentShardSize).  Raw pointers are the caller's
    responsibility."""
    if not hasattr(x, "data_ptr"):
        return
    if str(x.dtype) != "torch.uint8":
        raise ValueError(f"{what}: dtype must be uint8, got {x.dtype}")
    if on_device and not x.is_cuda:
        raise ValueError(f"{what}: must be a device (cuda/HIP) tensor")
    if x.dim() != dims:
        raise ValueError(f"{what}: expected a {dims}-D tensor, got shape {tuple(x.shape)}")
    if x.shape[-2] < rows or x.shape[-1] != shard_bytes:
        raise ValueError(f"{what}: shape {tuple(x.shape)} does not hold {rows} rows of {shard_bytes} bytes")


def _validate(rate_: int, original_count: int, recovery_count: int, shard_bytes: int) -> None:
    """The reference's own checks first (UnsupportedShardCount, then InvalidShardSize:
    src/rate.rs:91-106), so argument-shape errors never mask them."""
    err = _RsError()
    _raise(_lib.rs_validate(rate_, original_count, recovery_count, shard_bytes, ctypes.byref(err)), err)


def _check_mask(mask: bytes, count: int, what: str) -> bytes:
    if len(mask) != count:
        raise ValueError(f"{what}: {len(mask)} flags for {count} shards")
    return mask


def encode_device(original_count: int, recovery_count: int, shard_bytes: int, d_original, d_recovery,
                  stream=None, rate_: int = RATE_DEFAULT, ctx: Optional[Context] = None) -> None:
    """Encode shard matrices resident in device memory (rs_encode_device[_strided]).

    d_original / d_recovery: torch uint8 tensors [count, shard_bytes] (column-slice views of wider
    matrices allowed) or raw device pointers to contiguous rows."""
    ctx = ctx or default_context()
    _validate(rate_, original_count, recovery_count, shard_bytes)
    _check_matrix(d_original, original_count, shard_bytes, "d_original")
    _check_matrix(d_recovery, recovery_count, shard_bytes, "d_recovery")
    err = _RsError()
    _raise(_lib.rs_encode_device_strided(ctx.handle, rate_, original_count, recovery_count, shard_bytes,
                                         _ptr(d_original), _row_stride(d_original), _ptr(d_recovery),
                                         _row_stride(d_recovery), _stream(stream), ctypes.byref(err)), err)


def _batch_strides(x):
    """(row stride, stripe stride) in bytes of a 3-D uint8 tensor [stripes, rows, shard_bytes]
    whose rows are contiguous (0 = packed)."""
    if x.dim() != 3 or x.stride(2) != 1:
        raise ValueError("batch matrices must be [stripes, rows, shard_bytes] with contiguous rows")
    return int(x.stride(1)) * x.element_size(), int(x.stride(0)) * x.element_size()


def encode_device_batch(original_count: int, recovery_count: int, shard_bytes: int, d_original, d_recovery,
                        stream=None, rate_: int = RATE_DEFAULT, ctx: Optional[Context] = None) -> None:
    """Encode a batch of stripes of one shape (rs_encode_device_batch): d_original
    [stripes, original_count, shard_bytes], d_recovery [stripes, recovery_count, shard_bytes]."""
    ctx = ctx or default_context()
    _validate(rate_, original_count, recovery_count, shard_bytes)
    _check_matrix(d_original, original_count, shard_bytes, "d_original", 3)
    _check_matrix(d_recovery, recovery_count, shard_bytes, "d_recovery", 3)
    if d_original.shape[0] != d_recovery.shape[0]:
        raise ValueError("original and recovery batches differ in stripe count")
    (o_row, o_b), (r_row, r_b) = _batch_strides(d_original), _batch_strides(d_recovery)
    err = _RsError()
    _raise(_lib.rs_encode_device_batch(ctx.handle, rate_, original_count, recovery_count, shard_bytes,
                                       d_original.shape[0], d_original.data_ptr(), o_row, o_b, d_recovery.data_ptr(),
                                       r_row, r_b, _stream(stream), ctypes.byref(err)), err)


def decode_device_batch(original_count: int, recovery_count: int, shard_bytes: int, d_original, original_present,
                        d_recovery, recovery_present, d_restored, stream=None, rate_: int = RATE_DEFAULT,
                        ctx: Optional[Context] = None) -> None:
    """Decode a batch of stripes sharing ONE erasure pattern (rs_decode_device_batch); tensors
    [stripes, rows, shard_bytes]; only missing originals of d_restored are written."""
    ctx = ctx or default_context()
    _validate(rate_, original_count, recovery_count, shard_bytes)
    _check_matrix(d_original, original_count, shard_bytes, "d_original", 3)
    _check_matrix(d_recovery, recovery_count, shard_bytes, "d_recovery", 3)
    _check_matrix(d_restored, original_count, shard_bytes, "d_restored", 3)
    n = d_original.shape[0]
    if d_recovery.shape[0] != n or d_restored.shape[0] != n:
        raise ValueError("batches differ in stripe count")
    (o_row, o_b), (r_row, r_b), (x_row, x_b) = (_batch_strides(d_original), _batch_strides(d_recovery),
                                                _batch_strides(d_restored))
    err = _RsError()
    _raise(_lib.rs_decode_device_batch(ctx.handle, rate_, original_count, recovery_count, shard_bytes, n,
                                       d_original.data_ptr(), o_row, o_b,
                                       _check_mask(present_mask(original_present), original_count, "original_present"),
                                       d_recovery.data_ptr(), r_row, r_b,
                                       _check_mask(present_mask(recovery_present), recovery_count, "recovery_present"),
                                       d_restored.data_ptr(), x_row, x_b, _stream(stream), ctypes.byref(err)), err)


def present_mask(flags) -> bytes:
    """0/1 byte mask; bytes pass through unchanged (pre-build it once in hot loops)."""
    if isinstance(flags, (bytes, bytearray)):
        return bytes(flags)
    if hasattr(flags, "astype"):
        return (flags != 0).astype("uint8").tobytes()
    return bytes(bytearray(1 if x else 0 for x in flags))


def decode_device(original_count: int, recovery_count: int, shard_bytes: int, d_original, original_present,
                  d_recovery, recovery_present, d_restored, stream=None, rate_: int = RATE_DEFAULT,
                  ctx: Optional[Context] = None) -> None:
    ctx = ctx or default_context()
    _validate(rate_, original_count, recovery_count, shard_bytes)
    op = _check_mask(present_mask(original_present), original_count, "original_present")
    rp = _check_mask(present_mask(recovery_present), recovery_count, "recovery_present")
    _check_matrix(d_original, original_count, shard_bytes, "d_original")
    _check_matrix(d_recovery, recovery_count, shard_bytes, "d_recovery")
    _check_matrix(d_restored, original_count, shard_bytes, "d_restored")
    err = _RsError()
    _raise(_lib.rs_decode_device_strided(ctx.handle, rate_, original_count, recovery_count, shard_bytes,
                                         _ptr(d_original), _row_stride(d_original), op, _ptr(d_recovery),
                                         _row_stride(d_recovery), rp, _ptr(d_restored), _row_stride(d_restored),
                                         _stream(stream), ctypes.byref(err)), err)


class DeviceCall:
    """A device encode / decode bound once to fixed shapes, buffers and stream
    (`encode_device_call` / `decode_device_call`): each call is one C-ABI call
    (rs_encode_device_strided / rs_decode_device_strided) with pre-converted
    arguments, ≈1 µs of Python instead of ≈4 µs for the keyword wrappers --
    what a storage server coding many stripes through fixed staging buffers
    does, and what a Rust / C caller of the ABI pays (nothing).  The buffers
    and masks are kept alive by the object."""

    def __init__(self, fn, args, keep):
        self._fn = fn
        self._err = _RsError()
        self._args = tuple(args) + (ctypes.byref(self._err),)
        self._keep = keep

    def __call__(self) -> None:
        code = self._fn(*self._args)
        if code:
            _raise(code, self._err)


def encode_device_call(original_count: int, recovery_count: int, shard_bytes: int, d_original, d_recovery,
                       stream=None, rate_: int = RATE_DEFAULT, ctx: Optional[Context] = None) -> DeviceCall:
    """encode_device(...) bound once; call the result to encode."""
    ctx = ctx or default_context()
    _validate(rate_, original_count, recovery_count, shard_bytes)
    _check_matrix(d_original, original_count, shard_bytes, "d_original")
    _check_matrix(d_recovery, recovery_count, shard_bytes, "d_recovery")
    u = ctypes.c_uint64
    args = (_vp(ctx.handle.value), _int(rate_), u(original_count), u(recovery_count), u(shard_bytes),
            _vp(_ptr(d_original)), u(_row_stride(d_original)), _vp(_ptr(d_recovery)), u(_row_stride(d_recovery)),
            _vp(_stream(stream)))
    return DeviceCall(_lib.rs_encode_device_strided, args, (d_original, d_recovery, ctx))


def decode_device_call(original_count: int, recovery_count: int, shard_bytes: int, d_original, original_present,
                       d_recovery, recovery_present, d_restored, stream=None, rate_: int = RATE_DEFAULT,
                       ctx: Optional[Context] = None) -> DeviceCall:
    """decode_device(...) bound once; call the result to decode."""
    ctx = ctx or default_context()
    _validate(rate_, original_count, recovery_count, shard_bytes)
    op = _check_mask(present_mask(original_present), original_count, "original_present")
    rp = _check_mask(present_mask(recovery_present), recovery_count, "recovery_present")
    _check_matrix(d_original, original_count, shard_bytes, "d_original")
    _check_matrix(d_recovery, recovery_count, shard_bytes, "d_recovery")
    _check_matrix(d_restored, original_count, shard_bytes, "d_restored")
    u = ctypes.c_uint64
    args = (_vp(ctx.handle.value), _int(rate_), u(original_count), u(recovery_count), u(shard_bytes),
            _vp(_ptr(d_original)), u(_row_stride(d_original)), op, _vp(_ptr(d_recovery)),
            u(_row_stride(d_recovery)), rp, _vp(_ptr(d_restored)), u(_row_stride(d_restored)), _vp(_stream(stream)))
    return DeviceCall(_lib.rs_decode_device_strided, args, (d_original, d_recovery, d_restored, op, rp, ctx))


_sig("rs_host_alloc", ctypes.c_void_p, _u64)
_sig("rs_host_free", None, ctypes.c_void_p)
_sig("rs_encode_host", _int, _vp, _int, _u64, _u64, _u64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32,
     ctypes.POINTER(_RsError))
_sig("rs_decode_host", _int, _vp, _int, _u64, _u64, _u64, ctypes.c_void_p, ctypes.c_char_p, ctypes.c_void_p,
     ctypes.c_char_p, ctypes.c_void_p, ctypes.c_uint32, ctypes.POINTER(_RsError))


def _host_ptr(x) -> int:
    """Address of a contiguous host buffer: numpy array, torch CPU tensor (pinned for full rate) or int."""
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        if x.is_cuda or not x.is_contiguous():
            raise ValueError("host buffers must be contiguous CPU tensors")
        return x.data_ptr()
    if not x.flags["C_CONTIGUOUS"]:
        raise ValueError("host buffers must be C-contiguous")
    return x.ctypes.data


def encode_host(original_count: int, recovery_count: int, shard_bytes: int, h_original, h_recovery,
                slices: int = 4, rate_: int = RATE_DEFAULT, ctx: Optional[Context] = None) -> None:
    """Encode shard matrices in HOST memory (rs_encode_host): column slices pipelined over
    H2D copy / kernels / D2H copy on several streams.  Blocks until h_recovery is filled."""
    ctx = ctx or default_context()
    err = _RsError()
    _raise(_lib.rs_encode_host(ctx.handle, rate_, original_count, recovery_count, shard_bytes,
                               _host_ptr(h_original), _host_ptr(h_recovery), slices, ctypes.byref(err)), err)


def decode_host(original_count: int, recovery_count: int, shard_bytes: int, h_original, original_present,
                h_recovery, recovery_present, h_restored, slices: int = 4, rate_: int = RATE_DEFAULT,
                ctx: Optional[Context] = None) -> None:
    """Decode from HOST memory (rs_decode_host); only missing originals of h_restored are written."""
    ctx = ctx or default_context()
    err = _RsError()
    _raise(_lib.rs_decode_host(ctx.handle, rate_, original_count, recovery_count, shard_bytes,
                               _host_ptr(h_original),
                               _check_mask(present_mask(original_present), original_count, "original_present"),
                               _host_ptr(h_recovery),
                               _check_mask(present_mask(recovery_present), recovery_count, "recovery_present"),
                               _host_ptr(h_restored), slices,
                               ctypes.byref(err)), err)


class _ColumnSplit:
    """Shared plumbing of the column-partitioned encode and decode of ONE stripe over the ranks
    of a process group, one GPU per rank.  Rank r owns byte
    columns [r*w, (r+1)*w) of every shard, w = shard_bytes / world (whole 64-byte blocks).
    Every engine op is column-wise (src/engine/utils.rs:35-43, src/engine/engine_naive.rs:107-146),
    so a rank's slice is coded on its own device with no exchange, and the all-gathered slices
    equal the single-device result.

    The slice is coded in `chunks` column pieces: piece c's all-gather (asynchronous, on the
    collective's own stream for RCCL) runs while piece c+1 is coded and piece c-1 is
    re-interleaved.  `force_collective` keeps that path at world 1 (the all-gather of one rank
    is a copy through the backend), so RCCL's stream ordering is exercised on one GPU."""

    def __init__(self, original_count, recovery_count, shard_bytes, device, group, stream, rate_, ctx, chunks,
                 force_collective):
        import torch
        import torch.distributed as dist

        self.group = group
        self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        if shard_bytes % (64 * self.world):
            raise ValueError(f"shard_bytes {shard_bytes} must split into whole 64-byte blocks over "
                             f"{self.world} ranks")
        self.N, self.M, self.S = original_count, recovery_count, shard_bytes
        self.w = shard_bytes // self.world
        self.collective = self.world > 1 or bool(force_collective)
        if chunks is None:  # pieces of at least 2 KiB of columns, at most 4
            chunks = max(c for c in (1, 2, 4) if self.w % (64 * c) == 0 and (c == 1 or self.w // c >= 2048))
        if chunks < 1 or self.w % (64 * chunks):
            raise ValueError(f"{chunks} pieces do not split a {self.w}-byte column slice into whole 64-byte blocks")
        self.chunks, self.cw = chunks, self.w // chunks
        self.stream, self.rate, self.ctx = stream, rate_, ctx
        self.nccl = dist.get_backend(group) == "nccl"
        self.dev = torch.device(device) if device is not None else (
            torch.device("cuda", torch.cuda.current_device()) if self.nccl else torch.device("cpu"))

    def columns(self, d_matrix):
        """This rank's column slice of a full [rows x S] shard matrix (a strided view)."""
        return d_matrix[:, self.rank * self.w:(self.rank + 1) * self.w]

    def _piece(self, c):
        return slice(c * self.cw, (c + 1) * self.cw)

    def _on_stream(self, call) -> None:
        """Run a device call on the caller-supplied stream, ordered against the current one:
        the call waits for what the current stream has queued (the writes of its inputs and,
        through the previous call's work.wait(), the all-gathers still reading its output),
        and the collectives, which follow the current stream, wait for the call."""
        if self.stream is None:
            call(None)
            return
        import torch
        cur = torch.cuda.current_stream()
        self.stream.wait_stream(cur)
        call(self.stream)
        cur.wait_stream(self.stream)

    def _all_gather(self, out, inp):
        import torch.distributed as dist

        if self.nccl:
            return dist.all_gather_into_tensor(out, inp, group=self.group, async_op=True)
        return dist.all_gather(list(out.unbind(0)), inp, group=self.group, async_op=True)

    def _pipeline(self, code, start, finish) -> None:
        pending = None
        for c in range(self.chunks):
            code(c)
            work = start(c)
            if pending is not None:  # piece c-1's interleave behind piece c's coding
                finish(*pending)
            pending = (c, work)
        finish(*pending)


class ShardedEncoder(_ColumnSplit):
    """Column-partitioned encode of ONE stripe (_ColumnSplit): rank r encodes its [N x w]
    columns (rs_encode_device_strided) into [M x w] recovery slices, and an all-gather (RCCL
    over xGMI for the "nccl" backend) plus a re-interleave assembles the whole [M x S] recovery
    matrix on every rank.  `encode_slice(orig_cols, rec_slice)` replaces the per-piece device
    encode (tests drive the plumbing on CPU with a stand-in)."""

    def __init__(self, original_count: int, recovery_count: int, shard_bytes: int, device=None, group=None,
                 stream=None, rate_: int = RATE_DEFAULT, ctx: Optional[Context] = None, encode_slice=None,
                 chunks: Optional[int] = None, force_collective: bool = False):
        import torch

        super().__init__(original_count, recovery_count, shard_bytes, device, group, stream, rate_, ctx, chunks,
                         force_collective)
        self._encode_slice = encode_slice
        M, dev = recovery_count, self.dev
        self._part = None
        self.pieces = ([torch.empty((M, self.cw), dtype=torch.uint8, device=dev) for _ in range(self.chunks)]
                       if self.collective else [])
        self.gathered = ([torch.empty((self.world, M, self.cw), dtype=torch.uint8, device=dev)
                          for _ in range(self.chunks)] if self.collective else [])

    def _encode(self, cols, out) -> None:
        if self._encode_slice is not None:
            self._encode_slice(cols, out)
            return
        self._on_stream(lambda s: encode_device(self.N, self.M, cols.shape[1], cols, out, stream=s, rate_=self.rate,
                                                ctx=self.ctx))

    @property
    def part(self):
        """This rank's [M x w] recovery slice (encode_local / gather; allocated on first use)."""
        if self._part is None:
            import torch
            self._part = torch.empty((self.M, self.w), dtype=torch.uint8, device=self.dev)
        return self._part

    def encode_local(self, orig_cols) -> None:
        """Encode this rank's [N x w] columns into self.part (one device call)."""
        self._encode(orig_cols, self.part)

    def gather(self, d_recovery) -> None:
        """All-gather every rank's self.part and re-interleave into d_recovery [M x S]."""
        if not self.collective:
            d_recovery.copy_(self.part)
            return
        for c in range(self.chunks):
            self.pieces[c].copy_(self.part[:, self._piece(c)])
        works = [(c, self._start_gather(c)) for c in range(self.chunks)]
        for c, work in works:
            self._finish_gather(c, work, d_recovery)

    def _start_gather(self, c):
        return self._all_gather(self.gathered[c], self.pieces[c])

    def _finish_gather(self, c, work, d_recovery) -> None:
        work.wait()  # (nccl: the current stream waits for the collective's stream)
        out = d_recovery.view(self.M, self.world, self.w)[:, :, self._piece(c)]
        out.copy_(self.gathered[c].permute(1, 0, 2))

    def __call__(self, orig_cols, d_recovery) -> None:
        """Encode this rank's [N x w] columns and assemble d_recovery [M x S] on every rank."""
        if not self.collective:
            self._encode(orig_cols, d_recovery)
            return
        self._pipeline(lambda c: self._encode(orig_cols[:, self._piece(c)], self.pieces[c]), self._start_gather,
                       lambda c, work: self._finish_gather(c, work, d_recovery))


class ShardedDecoder(_ColumnSplit):
    """Column-partitioned decode of ONE stripe (_ColumnSplit).  The erasure
    pattern is the same on every rank, so eval_poly (src/rate/rate_high.rs:186-204) is
    replicated: each rank decodes its [N x w] / [M x w] column slices
    (rs_decode_device_strided, src/rate/rate_high.rs:172-254 per column) into a slice buffer,
    packs the restored (= missing original) rows of each piece, and an all-gather plus a
    re-interleave writes the missing originals' full rows into d_restored [N x S] on every
    rank; present rows of d_restored are never written, as in the single-device decode.
    `decode_slice(orig_cols, original_present, rec_cols, recovery_present, out)` replaces the
    per-piece device decode (CPU tests)."""

    def __init__(self, original_count: int, recovery_count: int, shard_bytes: int, device=None, group=None,
                 stream=None, rate_: int = RATE_DEFAULT, ctx: Optional[Context] = None, decode_slice=None,
                 chunks: Optional[int] = None, force_collective: bool = False):
        import torch

        super().__init__(original_count, recovery_count, shard_bytes, device, group, stream, rate_, ctx, chunks,
                         force_collective)
        self._decode_slice = decode_slice
        N, dev = original_count, self.dev
        self.part = torch.empty((N, self.w), dtype=torch.uint8, device=dev) if self.collective else None
        # packed / gathered restored rows of each piece, allocated once for the most rows a
        # pattern can restore (N) and narrowed per pattern: a loss pattern that changes from
        # stripe to stripe costs no allocation
        self._packed = [torch.empty(N * self.cw, dtype=torch.uint8, device=dev) for _ in range(self.chunks)] \
            if self.collective else []
        self._gathered = [torch.empty(self.world * N * self.cw, dtype=torch.uint8, device=dev)
                          for _ in range(self.chunks)] if self.collective else []
        self._pattern = None  # (original mask, missing-row index, its host copy, packed, gathered)
        self._check_masks = os.environ.get("RS_MI355X_DEBUG_MASKS") == "1"

    def _same_on_every_rank(self, op: bytes) -> None:
        """Debug (RS_MI355X_DEBUG_MASKS=1): every rank must pass the same erasure pattern --
        the gathers are sized by its loss count, so ranks that differ would hang in them."""
        import hashlib
        import torch
        import torch.distributed as dist

        h = int.from_bytes(hashlib.sha256(op).digest()[:7], "little")
        t = torch.tensor([h, -h], dtype=torch.int64, device=self.dev if self.nccl else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        if int(t[0]) != h or -int(t[1]) != h:
            raise ValueError("ShardedDecoder: the ranks passed different original_present masks")

    def _prepare(self, op: bytes):
        """Missing-row index and gather views of one erasure pattern (kept while it repeats)."""
        if self._pattern is not None and self._pattern[0] == op:
            return self._pattern
        import numpy as np
        import torch

        if self._check_masks:
            self._same_on_every_rank(op)
        miss = np.flatnonzero(np.frombuffer(op, dtype=np.uint8) == 0).astype(np.int64)
        L, dev = len(miss), self.dev
        host = torch.from_numpy(miss)
        if dev.type == "cuda":  # pinned, so the index goes up without blocking the host
            host = host.pin_memory()
        idx = host.to(dev, non_blocking=True)
        cw, world = self.cw, self.world
        packed = [b[:L * cw].view(L, cw) for b in self._packed]
        gathered = [b[:world * L * cw].view(world, L, cw) for b in self._gathered]
        self._pattern = (op, idx, host, packed, gathered)
        return self._pattern

    def _decode(self, orig_cols, op, rec_cols, rp, out) -> None:
        if self._decode_slice is not None:
            self._decode_slice(orig_cols, op, rec_cols, rp, out)
            return
        self._on_stream(lambda s: decode_device(self.N, self.M, out.shape[1], orig_cols, op, rec_cols, rp, out,
                                                stream=s, rate_=self.rate, ctx=self.ctx))

    def __call__(self, orig_cols, original_present, rec_cols, recovery_present, d_restored) -> None:
        """Decode this rank's column slices (orig_cols [N x w], rec_cols [M x w]; rows not
        present are ignored) and write every missing original's full row of d_restored
        [N x S] on every rank."""
        import torch

        op = _check_mask(present_mask(original_present), self.N, "original_present")
        rp = _check_mask(present_mask(recovery_present), self.M, "recovery_present")
        if not self.collective:
            self._decode(orig_cols, op, rec_cols, rp, d_restored)
            return
        _, idx, _, packed, gathered = self._prepare(op)
        if idx.numel() == 0:  # nothing to restore (decoder_work.rs:131-132); the call still validates
            self._decode(orig_cols[:, self._piece(0)], op, rec_cols[:, self._piece(0)], rp,
                         self.part[:, self._piece(0)])
            return

        def code(c):
            sl = self._piece(c)
            self._decode(orig_cols[:, sl], op, rec_cols[:, sl], rp, self.part[:, sl])
            torch.index_select(self.part[:, sl], 0, idx, out=packed[c])

        def finish(c, work):
            work.wait()
            out = d_restored.view(self.N, self.world, self.w)[:, :, self._piece(c)]
            out.index_copy_(0, idx, gathered[c].permute(1, 0, 2))

        self._pipeline(code, lambda c: self._all_gather(gathered[c], packed[c]), finish)


_sharded_cache: Dict[tuple, _ColumnSplit] = {}


def _sharded(cls, original_count, recovery_count, shard_bytes, device, group, stream, rate_, ctx):
    key = (cls.__name__, original_count, recovery_count, shard_bytes, id(group), str(device), _stream(stream), rate_,
           id(ctx))
    obj = _sharded_cache.get(key)
    if obj is None:
        obj = _sharded_cache[key] = cls(original_count, recovery_count, shard_bytes, device=device, group=group,
                                        stream=stream, rate_=rate_, ctx=ctx)
    return obj


def encode_device_sharded(original_count: int, recovery_count: int, shard_bytes: int, d_original, d_recovery,
                          group=None, stream=None, rate_: int = RATE_DEFAULT, ctx: Optional[Context] = None) -> None:
    """Multi-GPU encode of one large stripe: each rank (one GPU each) encodes its column slice of
    d_original [N x S] on its device, then an all-gather assembles d_recovery [M x S] everywhere
    (ShardedEncoder, cached per shape / group / device)."""
    enc = _sharded(ShardedEncoder, original_count, recovery_count, shard_bytes, d_recovery.device, group, stream,
                   rate_, ctx)
    _check_matrix(d_recovery, recovery_count, shard_bytes, "d_recovery", on_device=False)
    _check_matrix(d_original, original_count, shard_bytes, "d_original", on_device=False)
    enc(enc.columns(d_original), d_recovery)


def decode_device_sharded(original_count: int, recovery_count: int, shard_bytes: int, d_original, original_present,
                          d_recovery, recovery_present, d_restored, group=None, stream=None,
                          rate_: int = RATE_DEFAULT, ctx: Optional[Context] = None) -> None:
    """Multi-GPU decode of one large stripe (ShardedDecoder, cached per shape / group / device):
    each rank decodes its column slice of d_original [N x S] / d_recovery [M x S] with the
    erasure pattern evaluated on its own device, and an all-gather writes the missing originals'
    full rows into d_restored [N x S] on every rank."""
    dec = _sharded(ShardedDecoder, original_count, recovery_count, shard_bytes, d_restored.device, group, stream,
                   rate_, ctx)
    _check_matrix(d_original, original_count, shard_bytes, "d_original", on_device=False)
    _check_matrix(d_recovery, recovery_count, shard_bytes, "d_recovery", on_device=False)
    _check_matrix(d_restored, original_count, shard_bytes, "d_restored", on_device=False)
    dec(dec.columns(d_original), original_present, dec.columns(d_recovery), recovery_present, d_restored)


class engine:
    """trait Engine over device shard matrices (src/engine.rs:234-291)."""

    @staticmethod
    def fft(d_rows, shard_count, shard_len_64, pos, size, truncated_size, skew_delta, stream=None, ctx=None):
        ctx = ctx or default_context()
        code = _lib.rs_engine_fft(ctx.handle, _ptr(d_rows), shard_count, shard_len_64, pos, size, truncated_size,
                                  skew_delta, _stream(stream))
        _raise(code, _RsError())

    @staticmethod
    def ifft(d_rows, shard_count, shard_len_64, pos, size, truncated_size, skew_delta, stream=None, ctx=None):
        ctx = ctx or default_context()
        code = _lib.rs_engine_ifft(ctx.handle, _ptr(d_rows), shard_count, shard_len_64, pos, size, truncated_size,
                                   skew_delta, _stream(stream))
        _raise(code, _RsError())

    @staticmethod
    def mul(d_rows, block_count, log_m, stream=None, ctx=None):
        ctx = ctx or default_context()
        _raise(_lib.rs_engine_mul(ctx.handle, _ptr(d_rows), block_count, log_m, _stream(stream)), _RsError())

    @staticmethod
    def formal_derivative(d_rows, shard_count, shard_len_64, stream=None, ctx=None):
        ctx = ctx or default_context()
        _raise(_lib.rs_engine_formal_derivative(ctx.handle, _ptr(d_rows), shard_count, shard_len_64,
                                                _stream(stream)), _RsError())

    # the same ops on a HOST array (numpy uint8 [shard_count, shard_len_64 * 64], C-contiguous,
    # writable), the reference's own calling convention (rs_engine_*_host; blocking)
    @staticmethod
    def fft_host(rows, shard_count, shard_len_64, pos, size, truncated_size, skew_delta, ctx=None):
        ctx = ctx or default_context()
        _raise(_lib.rs_engine_fft_host(ctx.handle, _host_ptr(rows), shard_count, shard_len_64, pos, size,
                                       truncated_size, skew_delta), _RsError())

    @staticmethod
    def ifft_host(rows, shard_count, shard_len_64, pos, size, truncated_size, skew_delta, ctx=None):
        ctx = ctx or default_context()
        _raise(_lib.rs_engine_ifft_host(ctx.handle, _host_ptr(rows), shard_count, shard_len_64, pos, size,
                                        truncated_size, skew_delta), _RsError())

    @staticmethod
    def mul_host(blocks, block_count, log_m, ctx=None):
        ctx = ctx or default_context()
        _raise(_lib.rs_engine_mul_host(ctx.handle, _host_ptr(blocks), block_count, log_m), _RsError())

    @staticmethod
    def eval_poly(erasures, truncated_size):
        """In place on a writable buffer of 65536 uint16 (e.g. numpy array)."""
        import numpy as np
        a = np.ascontiguousarray(erasures, dtype=np.uint16)
        _lib.rs_engine_eval_poly(a.ctypes.data_as(ctypes.POINTER(ctypes.c_uint16)), truncated_size)
        return a


def table(name: str, count: int):
    import numpy as np
    p = getattr(_lib, f"rs_table_{name}")()
    return np.ctypeslib.as_array(p, shape=(count,)).copy()


def use_high_rate(original_count: int, recovery_count: int) -> int:
    return int(_lib.rs_use_high_rate(original_count, recovery_count))
