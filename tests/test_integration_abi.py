"""The reference-side binding in INTEGRATION.md matches the C ABI (CPU only, no GPU).

Every `extern "C" { ... }` block of INTEGRATION.md's Rust code is parsed, its Rust types are
mapped to C, and the prototypes are compiled as redeclarations against include/rs_mi355x.h:
a binding whose signature drifts from the header fails here at compile time ("conflicting
types").  The `#[repr(C)] RsError` mirror is checked field by field against `rs_error`
(names, offsets, size).  The functions named in those blocks must also be exported by the
built library.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DOC = os.path.join(ROOT, "INTEGRATION.md")
HEADER = os.path.join(ROOT, "include", "rs_mi355x.h")

TYPES = {
    "*mut *mut RsContext": "rs_context **", "*mut RsContext": "rs_context *", "*mut c_void": "void *",
    "*const c_void": "const void *", "*const u8": "const uint8_t *", "*mut u8": "uint8_t *",
    "*mut u16": "uint16_t *", "*const c_char": "const char *", "*mut RsError": "rs_error *",
    "u64": "uint64_t", "u32": "uint32_t", "u16": "uint16_t", "u8": "uint8_t", "i32": "int32_t",
    "c_int": "int", "RsStatus": "rs_status", "RsRate": "rs_rate",
    "*mut RsEncoder": "rs_encoder *", "*mut *mut RsEncoder": "rs_encoder **",
    "*mut RsDecoder": "rs_decoder *", "*mut *mut RsDecoder": "rs_decoder **",
    "*mut RsEncoderWork": "rs_encoder_work *", "*mut *mut RsEncoderWork": "rs_encoder_work **",
    "*mut RsDecoderWork": "rs_decoder_work *", "*mut *mut RsDecoderWork": "rs_decoder_work **",
    "*mut *mut RsContext": "rs_context **",
}


def _rust_blocks():
    text = open(DOC).read()
    return re.findall(r"```rust\n(.*?)```", text, flags=re.S)


def _extern_fns():
    fns = []
    for block in _rust_blocks():
        for body in re.findall(r'extern "C" \{(.*?)\n\}', block, flags=re.S):
            body = re.sub(r"//[^\n]*", "", body)
            for m in re.finditer(r"fn\s+(\w+)\s*\((.*?)\)\s*(?:->\s*([^;]+))?;", body, flags=re.S):
                name, args, ret = m.group(1), " ".join(m.group(2).split()), (m.group(3) or "").strip()
                fns.append((name, args, ret))
    return fns


def _ctype(t):
    t = " ".join(t.split())
    if t not in TYPES:
        raise AssertionError(f"unmapped Rust type in INTEGRATION.md binding: {t!r}")
    return TYPES[t]


def _prototype(name, args, ret):
    params = []
    for a in filter(None, (x.strip() for x in args.split(","))):
        pname, ptype = (x.strip() for x in a.split(":", 1))
        params.append(f"{_ctype(ptype)} {pname}")
    return f"{_ctype(ret) if ret else 'void'} {name}({', '.join(params) or 'void'});"


def _rs_error_fields():
    for block in _rust_blocks():
        m = re.search(r"pub struct RsError \{(.*?)\}", block, flags=re.S)
        if m:
            return re.findall(r"pub (\w+): (\w+),", m.group(1))
    raise AssertionError("INTEGRATION.md has no RsError mirror")


def test_integration_bindings_compile_against_header(tmp_path):
    fns = _extern_fns()
    names = {f[0] for f in fns}
    # the Engine shim, the device path, the batch forms and the host pipeline are all bound
    for must in ("rs_engine_fft_host", "rs_engine_ifft_host", "rs_engine_mul_host", "rs_engine_eval_poly",
                 "rs_context_create", "rs_encode_device", "rs_decode_device", "rs_encode_device_batch",
                 "rs_decode_device_batch", "rs_encode_host", "rs_decode_host"):
        assert must in names, must
    fields = _rs_error_fields()
    src = ["#include <stddef.h>", "#include <stdint.h>", f'#include "{HEADER}"', ""]
    src += [_prototype(*f) for f in fns]
    src += ["", "struct rust_rs_error {"] + [f"    {_ctype(t)} {n};" for n, t in fields] + ["};"]
    src += [f"_Static_assert(offsetof(struct rust_rs_error, {n}) == offsetof(rs_error, {n}), \"{n}\");"
            for n, _ in fields]
    src += ["_Static_assert(sizeof(struct rust_rs_error) == sizeof(rs_error), \"size\");"]
    c = tmp_path / "bindings.c"
    c.write_text("\n".join(src) + "\n")
    r = subprocess.run(["gcc", "-std=c11", "-Wall", "-Werror", "-c", str(c), "-o", str(tmp_path / "b.o")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr + "\n" + c.read_text()


def test_integration_bindings_detect_drift(tmp_path):
    """The check itself works: a binding with a wrong parameter type does not compile."""
    src = ["#include <stdint.h>", f'#include "{HEADER}"',
           _prototype("rs_engine_mul_host", "ctx: *mut RsContext, blocks: *mut u8, block_count: u64, log_m: u64",
                      "RsStatus")]
    c = tmp_path / "drift.c"
    c.write_text("\n".join(src) + "\n")
    r = subprocess.run(["gcc", "-std=c11", "-c", str(c), "-o", str(tmp_path / "d.o")], capture_output=True,
                       text=True)
    assert r.returncode != 0 and "conflicting types" in r.stderr


def test_integration_bound_symbols_are_exported():
    import reed_solomon_simd as rs

    missing = [n for n, _, _ in _extern_fns() if not hasattr(rs._lib, n)]
    assert not missing, missing
