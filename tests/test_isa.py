"""Checks of the built gfx950 code object (CPU: disassembly, no GPU).

rs_mono.hip's staged decode loads lw_fold first, with a plain load the compiler
tracks, and lets the compiler place the wait for it at its first use, after
eval_poly's first transform.  On the path that issues the row and table loads
that wait must leave them in flight: vmcnt(13) in the headline decode (1
shared-table load, 4 row loads, 8 phase-1 table loads issued after lw_fold).
A smaller count would still be correct but would hold eval_poly until the rows
land (the former hand-counted inline-asm wait).
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "reed-solomon-simd_amd", "lib", "librs_mi355x.so")
LLVM = "/opt/rocm/lib/llvm/bin"


def _disassemble(tmp_path_factory):
    tools = [os.path.join(LLVM, t) for t in ("llvm-objcopy", "clang-offload-bundler", "llvm-objdump")]
    if not all(os.path.exists(t) for t in tools) or not os.path.exists(LIB):
        pytest.skip("ROCm LLVM tools or the built library missing")
    d = tmp_path_factory.mktemp("isa")
    fat = str(d / "fat")
    subprocess.run([tools[0], "-O", "binary", "--only-section=.hip_fatbin", LIB, fat], check=True)
    # the section holds one offload bundle per translation unit, each opening with the magic
    data = open(fat, "rb").read()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)]
    out = ""
    for k, a in enumerate(starts):
        part, co = str(d / ("b%d" % k)), str(d / ("co%d" % k))
        with open(part, "wb") as f:
            f.write(data[a:starts[k + 1] if k + 1 < len(starts) else len(data)])
        subprocess.run([tools[1], "--unbundle", "--type=o", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950",
                        "--input=" + part, "--output=" + co], check=True)
        out += subprocess.run([tools[2], "-d", co], check=True, capture_output=True, text=True).stdout
    # per kernel: [(address, instruction, branch target or None)]
    kernels, name, body, base = {}, None, [], 0
    for line in out.splitlines():
        m = re.match(r"^([0-9a-f]+) <(\S+)>:$", line)
        if m:
            if name:
                kernels[name] = body
            name, body, base = m.group(2), [], int(m.group(1), 16)
        elif name and line.startswith("\t"):
            ins, _, comment = line.partition("//")
            a = re.match(r"\s*([0-9A-Fa-f]+):", comment)
            t = re.search(r"<\S+\+0x([0-9a-f]+)>", comment)
            body.append((int(a.group(1), 16) if a else None, ins.strip(),
                         base + int(t.group(1), 16) if t else None))
    if name:
        kernels[name] = body
    return kernels


@pytest.fixture(scope="module")
def kernels(tmp_path_factory):
    return _disassemble(tmp_path_factory)


def test_headline_decode_leaves_row_loads_in_flight(kernels):
    name = next((k for k in kernels if "k_monoILi11ELi1ELi2ELb1ELb0ELb1ELi2E" in k), None)
    assert name, "headline decode kernel k_mono<11, 1, 2, true, false, true, 2> not found"
    body = [ins for _, ins, _ in kernels[name]]
    first = next(i for i, ins in enumerate(body) if ins.startswith("global_load_dword "))
    reg = body[first].split()[1].rstrip(",")  # the lw_fold destination
    waits = []
    for i in range(first + 1, len(body)):
        ins = body[i]
        if ins.startswith("v_mul") and re.search(r"\b%s\b" % re.escape(reg), ins):  # x * lw_fold
            # the wait in force at this read of lw_fold: the last vmcnt before it
            for j in range(i - 1, first, -1):
                m = re.match(r"s_waitcnt vmcnt\((\d+)\)", body[j])
                if m:
                    waits.append(int(m.group(1)))
                    break
    # skip path (the shared-table load only after it: 1), live path (13 loads after it)
    assert 13 in waits, waits


def test_every_staged_decode_waits_for_lw_fold(kernels):
    """Every staged decode instantiation (L = 7..11, plain and split plans, 2- and 4-element
    packs): each multiply that reads the lw_fold register (the first vector load's
    destination) comes after an s_waitcnt vmcnt, placed by the compiler."""
    dec = [k for k in kernels if re.search(r"k_monoILi\d+ELi1ELi2ELb1E", k)]
    assert len(dec) >= 10, sorted(dec)
    for name in dec:
        body = [ins for _, ins, _ in kernels[name]]
        first = next(i for i, ins in enumerate(body) if ins.startswith("global_load_dword "))
        reg = body[first].split()[1].rstrip(",")
        uses = [i for i in range(first + 1, len(body))
                if body[i].startswith("v_mul") and re.search(r"\b%s\b" % re.escape(reg), body[i])]
        assert uses, name
        for i in uses:
            assert any(re.match(r"s_waitcnt vmcnt\(\d+\)", body[j]) for j in range(first + 1, i)), (name, i)
