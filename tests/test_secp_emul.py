"""CPU checks of the secp256k1 kernel code (lachain_amd/csrc/k_secp.hip) compiled for the host by
tools/emul/secp_emul.cpp and run lane by lane (the kernels use no LDS or barriers, so that is exact), against the oracle
(oracle/secp.c) and Python integers.  TEST INFRASTRUCTURE: catches logic errors in the device code without a GPU; the
GPU itself is covered by tests/test_gpu_ecdsa.py, and tools/emul/secp_stage_dump.hip diffs every intermediate buffer of
a GPU run against this emulation (profiles/r02/secp_stage_diff.txt)."""
import ctypes
import os
import random
import subprocess
import sys

import pytest

import oracle as o

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tools", "emul", "secp_emul.cpp")
LIB = os.path.join(ROOT, "tools", "emul", "libsecp_emul.so")
DEPS = [SRC, os.path.join(ROOT, "lachain_amd", "csrc", "k_secp.hip"), os.path.join(ROOT, "lachain_amd", "csrc", "secp.hpp")]
P, N = o.SECP_P, o.SECP_N


@pytest.fixture(scope="module")
def emu():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(d) for d in DEPS):
        subprocess.run(["g++", "-O1", "-std=c++17", "-fPIC", "-shared", "-o", LIB, SRC], check=True)
    return ctypes.CDLL(LIB)


def _le(x):
    return (x % 2 ** 256).to_bytes(32, "little")


def test_field_and_scalar_ops(emu):
    rng = random.Random(1)
    b = ctypes.create_string_buffer(32)
    for i in range(3000):
        a, c = rng.randrange(2 ** 256), rng.randrange(2 ** 256)
        if i % 5 == 0:
            a = P - rng.randrange(3)
        if i % 7 == 0:
            c = 2 ** 256 - 1 - rng.randrange(3)
        for f, want in ((emu.emu_fe_mul, a * c), (emu.emu_fe_add, a + c), (emu.emu_fe_sub, a - c)):
            f(b, _le(a), _le(c))
            assert int.from_bytes(b.raw, "little") % P == want % P
        emu.emu_fe_sqr(b, _le(a))
        assert int.from_bytes(b.raw, "little") % P == a * a % P
        emu.emu_fe_canon(b, _le(a))
        assert int.from_bytes(b.raw, "little") == a % P
    a = rng.randrange(1, P)
    emu.emu_fe_inv(b, _le(a))
    assert int.from_bytes(b.raw, "little") % P == pow(a, -1, P)
    R = 2 ** 256 % N
    for _ in range(2000):
        x, y = rng.randrange(N), rng.randrange(N)
        emu.emu_sc_mont_mul(b, _le(x), _le(y))
        assert int.from_bytes(b.raw, "little") == x * y * pow(R, -1, N) % N
    emu.emu_sc_mont_inv(b, _le(x * R % N))
    assert int.from_bytes(b.raw, "little") == pow(x, -1, N) * R % N


@pytest.mark.parametrize("chain,new", [(25, False), (225, True)])
def test_pipeline_vs_oracle(emu, chain, new):
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from test_gpu_ecdsa import _mixed_batch
    keys, hs, sigs, idx = _mixed_batch(random.Random(1000 + chain), chain, new, n=400)
    L = 66 if new else 65
    H, S, PK = b"".join(hs), b"".join(sigs), b"".join(keys)
    want = o.ecdsa_verify_batch(H, S, L, PK, 33, idx, len(hs), new, chain)
    acc = ctypes.create_string_buffer(len(hs))
    ia = (ctypes.c_int32 * len(idx))(*idx)
    emu.emu_verify(acc, H, None, ctypes.c_uint64(0), S, L, PK, 33, len(keys), ia, len(hs), int(new), chain)
    assert acc.raw[:len(hs)] == want
