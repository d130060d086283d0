"""Contexts used from several threads, and work handed between devices.

Kernel attributes (the dynamic LDS size of the column, pass and eval kernels)
are set once per device on first use (rs_device.hpp lds_attr_once: a per-device
bit set with an atomic OR after hipFuncSetAttribute succeeds).  The first test
runs in a fresh interpreter, so no kernel of this library has run on the device
yet: two threads each create their own Context on device 0, meet at a barrier
and launch at once -- the column-kernel encode and decode and the multi-pass
encode, each needing more than the default LDS -- and every result must equal
the oracle.  A second physical device is not testable on the 1-GPU pool; the
cross-device work hand-off test skips there.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

# (N, M, S, loss): column-kernel encode + decode (L = 11), multi-pass encode (L = 13)
THREAD_CASES = [(1024, 1024, 1024, 10), (4096, 4096, 512, 0), (1000, 3000, 256, 500)]

_CHILD = r"""
import json, sys, threading
import numpy as np
import torch
import reed_solomon_simd as rs
import oracle_lib as O
cases = json.loads(sys.argv[1])
T = 2
bar = threading.Barrier(T)
out, err = {}, []
def work(t):
    try:
        ctx = rs.Context(0)
        torch.cuda.set_device(0)
        inputs = []
        for (N, M, S, loss) in cases:
            orig = O.generate_original(N, S, N + M + S + t)
            inputs.append(torch.from_numpy(orig).cuda())
        torch.cuda.synchronize()
        bar.wait()
        for k, (N, M, S, loss) in enumerate(cases):
            d_orig = inputs[k]
            d_rec = torch.empty((M, S), dtype=torch.uint8, device="cuda")
            rs.encode_device(N, M, S, d_orig, d_rec, rate_=1, ctx=ctx)
            res = {"rec": d_rec.cpu().numpy().tobytes().hex()}
            if loss:
                op = np.ones(N, np.uint8); op[:loss] = 0
                rp = np.zeros(M, np.uint8); rp[:loss] = 1
                d_in = d_orig.clone(); d_in[:loss] = 0
                d_out = torch.zeros_like(d_orig)
                rs.decode_device(N, M, S, d_in, op, d_rec, rp, d_out, rate_=1, ctx=ctx)
                res["ok"] = bool(torch.equal(d_out[:loss], d_orig[:loss]))
            torch.cuda.synchronize()
            out["%d:%d" % (t, k)] = res
        rs.check_device(ctx)
        ctx.close()
    except Exception as e:
        err.append("%s: %r" % (t, e))
ths = [threading.Thread(target=work, args=(t,)) for t in range(T)]
[th.start() for th in ths]
[th.join() for th in ths]
print(json.dumps({"out": out, "err": err}))
"""


def _gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch


def test_two_contexts_two_threads_first_launch():
    _gpu()
    env = dict(os.environ)
    env["PYTHONPATH"] = os.pathsep.join([os.path.join(ROOT, "reed-solomon-simd_amd"), os.path.join(ROOT, "tests"),
                                         env.get("PYTHONPATH", "")])
    p = subprocess.run([sys.executable, "-c", _CHILD, json.dumps(THREAD_CASES)], env=env, capture_output=True,
                       text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads(p.stdout.strip().splitlines()[-1])
    assert not res["err"], res["err"]
    for t in range(2):
        for k, (N, M, S, loss) in enumerate(THREAD_CASES):
            r = res["out"]["%d:%d" % (t, k)]
            want = O.encode("high", O.generate_original(N, S, N + M + S + t), M)
            assert bytes.fromhex(r["rec"]) == want.tobytes(), (t, k)
            if loss:
                assert r["ok"], (t, k)


def test_work_moves_between_devices():
    """EncoderWork / DecoderWork handed from Context(0) to Context(1) (rs_codec.cpp's
    cross-device branch: host copies swapped, device buffers of device 0 freed)."""
    torch = _gpu()
    if torch.cuda.device_count() < 2:
        pytest.skip("one GPU: a second physical device is not testable on this pool")
    import reed_solomon_simd as rs
    c1 = rs.Context(1)
    try:
        orig = O.generate_original(300, 1024, 9)
        want = O.encode("high", orig, 200)
        enc = rs.rate.HighRateEncoder(300, 200, 1024)
        for row in orig:
            enc.add_original_shard(row.tobytes())
        assert b"".join(enc.encode().recovery_iter()) == want.tobytes()
        _, work = enc.into_parts()
        enc2 = rs.rate.HighRateEncoder(300, 200, 1024, ctx=c1, work=work)
        for row in orig:
            enc2.add_original_shard(row.tobytes())
        assert b"".join(enc2.encode().recovery_iter()) == want.tobytes()
        dec = rs.rate.HighRateDecoder(300, 200, 1024, ctx=c1)
        for i in range(100, 300):
            dec.add_original_shard(i, orig[i].tobytes())
        for i in range(100):
            dec.add_recovery_shard(i, want[i].tobytes())
        assert all(v == orig[i].tobytes() for i, v in dec.decode().restored_original_iter())
        _, dwork = dec.into_parts()
        dec0 = rs.rate.HighRateDecoder(300, 200, 1024, work=dwork)
        for i in range(100, 300):
            dec0.add_original_shard(i, orig[i].tobytes())
        for i in range(100):
            dec0.add_recovery_shard(i, want[i].tobytes())
        got = dict(dec0.decode().restored_original_iter())
        assert sorted(got) == list(range(100)) and all(got[i] == orig[i].tobytes() for i in got)
        rs.check_device(c1)
    finally:
        c1.close()
