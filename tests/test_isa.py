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


def _vmem(ins):
    """Instructions counted by vmcnt on gfx950 (GFX9: vector loads and stores alike)."""
    return re.match(r"(global|buffer|flat)_(load|store|atomic)", ins) is not None


def _lw_fold_covered_on_every_path(body, first, reg):
    """Walk every control-flow path from the lw_fold load (body[first]) and check that at
    each v_mul reading its register an s_waitcnt vmcnt(k) has retired it: k <= the vector
    memory instructions issued after it on that path.  Returns the counts n of the waits
    that retired it (by wait: the largest n - k over the paths through it).  Branch targets come from the
    disassembler's comments, so the check is path-exact rather than a linear scan."""
    index = {addr: i for i, (addr, _, _) in enumerate(body) if addr is not None}
    slack = {}  # wait instruction -> loads after lw_fold it leaves in flight beyond need
    seen = set()
    stack = [(first + 1, 0, False)]  # (instruction, vmem ops after lw_fold (capped), retired)
    while stack:
        i, n, done = stack.pop()
        while i < len(body):
            key = (i, n, done)
            if key in seen:
                break
            seen.add(key)
            _, ins, target = body[i]
            if ins.startswith("s_endpgm"):
                break
            m = re.match(r"s_waitcnt\s.*vmcnt\((\d+)\)", ins)
            if m and not done and int(m.group(1)) <= n:
                done = True
                slack[i] = max(slack.get(i, 0), n - int(m.group(1)))
                n = 0  # (no longer tracked once retired)
            if ins.startswith("v_mul") and re.search(r"\b%s\b" % re.escape(reg), ins):
                assert done, "lw_fold read at %d before a covering vmcnt wait (%d vector ops after it)" % (i, n)
            if _vmem(ins) and not done:
                n = min(n + 1, 64)
            if ins.startswith("s_cbranch") and target is not None and target in index:
                stack.append((index[target], n, done))
            if ins.startswith("s_branch") and target is not None and target in index:
                i = index[target]
                continue
            i += 1
    return slack


def test_every_staged_decode_waits_for_lw_fold(kernels):
    """Every staged decode instantiation (L = 7..11, plain and split plans, 2- and 4-element
    packs): on every path from the lw_fold load (the first vector load) to a multiply that
    reads it, a vmcnt wait placed by the compiler retires it (the count is
    checked per path, not merely present)."""
    dec = [k for k in kernels if re.search(r"k_monoILi\d+ELi1ELi2ELb1E", k)]
    assert len(dec) >= 10, sorted(dec)
    for name in dec:
        body = kernels[name]
        first = next(i for i, (_, ins, _) in enumerate(body) if ins.startswith("global_load_dword "))
        reg = body[first][1].split()[1].rstrip(",")
        uses = [i for i in range(first + 1, len(body))
                if body[i][1].startswith("v_mul") and re.search(r"\b%s\b" % re.escape(reg), body[i][1])]
        assert uses, name
        _lw_fold_covered_on_every_path(body, first, reg)


def test_headline_decode_wait_is_exact_on_every_path(kernels):
    """Performance pin (tied to this toolchain's scheduling): in the headline decode the first
    waits that retire lw_fold -- on the path that skips the row loads and on the one that issues
    them -- leave every later load in flight on every path through them (k = n: vmcnt(1) after
    the one shared-table load, vmcnt(13) after 13 loads).  Later copies (the byte-wise row
    access variant) are only checked for correctness above."""
    name = next(k for k in kernels if "k_monoILi11ELi1ELi2ELb1ELb0ELb1ELi2E" in k)
    body = kernels[name]
    first = next(i for i, (_, ins, _) in enumerate(body) if ins.startswith("global_load_dword "))
    reg = body[first][1].split()[1].rstrip(",")
    slack = _lw_fold_covered_on_every_path(body, first, reg)
    firsts = sorted(slack)[:2]
    assert [re.search(r"vmcnt\((\d+)\)", body[i][1]).group(1) for i in firsts] == ["1", "13"], firsts
    assert [slack[i] for i in firsts] == [0, 0], slack
