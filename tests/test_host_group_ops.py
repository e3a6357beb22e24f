"""The host-side G1 / G2 / GT surface of liblachain_bls.so (csrc/fp_host.hpp: add, sub, neg, dbl, normalize, isEqual,
isValid, (de)serialization, generators, GT product and (de)serialization) against the oracle and the reference's
serialization known answers (SerializationTest.cs:20-57).  These entry points do O(1) field work on the host, like the
Fr surface, so they run here without a GPU; the library is loaded without mclBn_init (only host code is called).
Every scalar multiplication below is the oracle's (the library's runs on the GPU, tests/test_gpu_parity.py)."""
import ctypes
import os
import subprocess
import sys

import pytest

import oracle as o
from helpers import Drbg, kats

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB


@pytest.fixture(scope="module")
def mcl():
    from lachain_amd import native
    native.load(False)._inited = True       # host entry points only: no device is opened
    from lachain_amd import mcl as m
    return m


def _points(d, n):
    g1s = [o.g1_mul(o.g1_gen(), d.fr()) for _ in range(n)]
    g2s = [o.g2_mul(o.g2_gen(), d.fr()) for _ in range(n)]
    return g1s, g2s


def test_generators_and_kats(mcl):
    k = kats()
    G1, G2 = mcl.G1, mcl.G2
    assert G1.Zero().ToBytes().hex() == k["g1_zero"]["hex"]
    assert G1.Generator().ToBytes().hex() == k["g1_generator"]["hex"]
    assert G2.Zero().ToBytes().hex() == k["g2_zero"]["hex"]
    assert G2.Generator().ToBytes().hex() == k["g2_generator"]["hex"]
    g1x2 = G1.Generator() + G1.Generator()
    assert g1x2.ToBytes().hex() == k["g1_generator_x2"]["hex"]
    g2x2 = G2.Generator() + G2.Generator()
    assert g2x2.ToBytes().hex() == k["g2_generator_x2"]["hex"]
    for key, G in (("g1_generator_x2", G1), ("g2_generator_x2", G2), ("g1_generator", G1), ("g2_generator", G2)):
        b = bytes.fromhex(k[key]["hex"])
        assert G.FromBytes(b).ToBytes() == b


@pytest.mark.parametrize("g", [1, 2])
def test_group_ops_match_oracle(mcl, g):
    d = Drbg(b"host-group-ops-%d" % g)
    g1s, g2s = _points(d, 6)
    pts = g1s if g == 1 else g2s
    G = mcl.G1 if g == 1 else mcl.G2
    add = o.g1_add if g == 1 else o.g2_add
    neg = o.g1_neg if g == 1 else o.g2_neg
    for a, b in zip(pts, pts[1:]):
        A, B = G.FromBytes(a), G.FromBytes(b)
        assert A.ToBytes() == a
        assert (A + B).ToBytes() == add(a, b)
        assert (A - B).ToBytes() == add(a, neg(b))
        assert (-A).ToBytes() == neg(a)
        assert (A + A).ToBytes() == add(a, a)                # doubling through add's equal-points case
        assert (A + (-A)).IsZero() and (A + (-A)).ToBytes() == bytes(len(a))
        assert (A + G.Zero()).ToBytes() == a and (G.Zero() + A).ToBytes() == a
        s = (A + B) + A                                      # Jacobian with z != 1, equal to (A + A) + B
        t = (A + A) + B
        assert s == t and s.ToBytes() == t.ToBytes() and s.IsValid()
        assert s != A
    assert G.Zero().IsValid() and G.Zero() == G.Zero() and G.Zero() != G.FromBytes(pts[0])


@pytest.mark.parametrize("g", [1, 2])
def test_dbl_normalize_and_struct_words(mcl, g):
    """mclBn*_dbl / _normalize: the same group element, and normalize gives z = 1 (Montgomery one) with the affine
    coordinates in the struct"""
    d = Drbg(b"host-dbl-%d" % g)
    g1s, g2s = _points(d, 2)
    G = mcl.G1 if g == 1 else mcl.G2
    T = G._T
    lib = mcl.native.lib()
    dbl = lib["mclBn%s_dbl" % G._P]
    nrm = lib["mclBn%s_normalize" % G._P]
    for f in (dbl, nrm):
        f.restype, f.argtypes = None, [ctypes.POINTER(T), ctypes.POINTER(T)]
    A = G.FromBytes((g1s if g == 1 else g2s)[0])
    D = G()
    dbl(ctypes.byref(D.v), ctypes.byref(A.v))
    assert D == A + A
    J = D + A                                               # z != 1
    N = G()
    nrm(ctypes.byref(N.v), ctypes.byref(J.v))
    assert N == J and N.ToBytes() == J.ToBytes()
    one = G.Generator().v.z                                 # generators are stored with z = 1
    assert bytes(N.v.z) == bytes(one)
    Z = G()
    nrm(ctypes.byref(Z.v), ctypes.byref(G.Zero().v))
    assert Z.IsZero()


@pytest.mark.parametrize("g", [1, 2])
def test_invalid_encodings_rejected(mcl, g):
    G = mcl.G1 if g == 1 else mcl.G2
    n = G.ByteSize
    valid = o.g1_valid if g == 1 else o.g2_valid
    bad = []
    x = (P + 5).to_bytes(48, "little")                     # x >= p
    bad.append(x + bytes(n - 48) if g == 1 else x + bytes(48))
    d = Drbg(b"host-invalid-%d" % g)
    tries = 0
    while len(bad) < 6 and tries < 200:                     # x values with no point on the curve
        tries += 1
        b = bytearray(d.bytes(n))
        b[n - 1] &= 0x1F
        if g == 2:
            b[47] &= 0x1F
        if not valid(bytes(b)):
            bad.append(bytes(b))
    assert len(bad) >= 4
    for b in bad:
        with pytest.raises(ValueError):
            G.FromBytes(b)
    # random valid encodings round-trip, including the sign flag of y
    for _ in range(8):
        b = bytearray(d.bytes(n))
        b[n - 1] &= 0x1F
        if g == 2:
            b[47] &= 0x1F
        b[n - 1] |= 0x80 if d.bytes(1)[0] & 1 else 0
        b = bytes(b)
        if valid(b):
            assert G.FromBytes(b).ToBytes() == b


def test_is_valid_rejects_off_curve_and_non_canonical(mcl):
    G1 = mcl.G1
    A = G1.Generator() + G1.Generator()
    assert A.IsValid()
    B = G1(type(A.v).from_buffer_copy(bytes(A.v)))
    raw = bytearray(bytes(B.v))
    raw[0] ^= 1                                             # x changed: off the curve
    C = G1(type(A.v).from_buffer_copy(bytes(raw)))
    assert not C.IsValid()
    raw = bytearray(bytes(A.v))
    raw[44:48] = b"\xff\xff\xff\xff"                         # x >= p
    assert not G1(type(A.v).from_buffer_copy(bytes(raw))).IsValid()


def test_gt_mul_and_serialization(mcl):
    d = Drbg(b"host-gt")
    g1s, g2s = _points(d, 2)
    a = o.pairing(g1s[0], g2s[0])
    b = o.pairing(g1s[1], g2s[1])
    lib = mcl.native.lib()
    des = lib["mclBnGT_deserialize"]
    des.restype, des.argtypes = ctypes.c_size_t, [ctypes.POINTER(mcl.mclBnGT), ctypes.c_char_p, ctypes.c_size_t]
    A, B = mcl.GT(), mcl.GT()
    assert des(ctypes.byref(A.v), a, 576) == 576 and des(ctypes.byref(B.v), b, 576) == 576
    assert A.ToBytes() == a
    assert (A * B).ToBytes() == o.gt_mul(a, b)
    assert (A * B) == (B * A)
    big = (P + 1).to_bytes(48, "little") + a[48:]
    C = mcl.GT()
    assert des(ctypes.byref(C.v), big, 576) == 0


def test_host_ops_from_16_threads():
    """the host surface is re-entrant (no shared state): 16 threads adding and (de)serializing at once"""
    code = r"""
import sys, threading
sys.path.insert(0, sys.argv[1]); sys.path.insert(0, sys.argv[1] + "/oracle")
from lachain_amd import native
native.load(False)._inited = True
from lachain_amd import mcl
import oracle as o
pts = [o.g1_mul(o.g1_gen(), (7 + i).to_bytes(32, "little")) for i in range(4)]
want = [o.g1_add(p, p) for p in pts]
start = threading.Barrier(16); bad = []; done = []
def work(i):
    start.wait()
    for k in range(300):
        j = (i + k) % 4
        A = mcl.G1.FromBytes(pts[j])
        if (A + A).ToBytes() != want[j]:
            bad.append(j)
    done.append(i)
ts = [threading.Thread(target=work, args=(i,)) for i in range(16)]
for t in ts: t.start()
for t in ts: t.join()
sys.exit(1 if bad or len(done) != 16 else 0)
"""
    r = subprocess.run([sys.executable, "-X", "faulthandler", "-c", code, ROOT], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
