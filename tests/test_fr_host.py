"""Scalar-field (Fr) arithmetic of the mcl surface (lachain_amd/csrc/fr_host.hpp) against the oracle and Python
integers — CPU test: the mclBnFr_* entry points run on the host and need no device, so the library is loaded
directly (mclBn_init, which opens the GPU, is not called).  Bit-exact 32-byte canonical encodings.
"""
import ctypes
import os

import pytest

import oracle as o
from helpers import Drbg, R

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SO = os.path.join(ROOT, "lachain_amd", "liblachain_bls.so")


class Fr(ctypes.Structure):
    _fields_ = [("d", ctypes.c_uint64 * 4)]


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(SO):
        pytest.skip("liblachain_bls.so not built")
    L = ctypes.CDLL(SO)
    P = ctypes.POINTER(Fr)
    for n in ("add", "sub", "mul", "div"):
        getattr(L, "mclBnFr_" + n).argtypes = [P, P, P]
    for n in ("neg", "inv", "sqr"):
        getattr(L, "mclBnFr_" + n).argtypes = [P, P]
    L.mclBnFr_deserialize.argtypes = [P, ctypes.c_char_p, ctypes.c_size_t]
    L.mclBnFr_deserialize.restype = ctypes.c_size_t
    L.mclBnFr_serialize.argtypes = [ctypes.c_char_p, ctypes.c_size_t, P]
    L.mclBnFr_serialize.restype = ctypes.c_size_t
    L.mclBnFr_setInt.argtypes = [P, ctypes.c_int64]
    L.mclBnFr_setLittleEndian.argtypes = [P, ctypes.c_char_p, ctypes.c_size_t]
    L.mclBnFr_setByCSPRNG.argtypes = [P]
    for n in ("isValid", "isZero", "isOne"):
        getattr(L, "mclBnFr_" + n).argtypes = [P]
    L.mclBnFr_isEqual.argtypes = [P, P]
    L.mclBn_FrLagrangeInterpolation.argtypes = [P, P, P, ctypes.c_size_t]
    L.mclBn_FrEvaluatePolynomial.argtypes = [P, P, ctypes.c_size_t, P]
    return L


def fr_of(L, b):
    x = Fr()
    assert L.mclBnFr_deserialize(ctypes.byref(x), b, 32) == 32
    return x


def enc(L, x):
    buf = ctypes.create_string_buffer(32)
    assert L.mclBnFr_serialize(buf, 32, ctypes.byref(x)) == 32
    return buf.raw


def i2b(v):
    return (v % R).to_bytes(32, "little")


def test_field_ops_match_oracle(lib):
    d = Drbg(b"fr-host")
    vals = [0, 1, 2, R - 1, R - 2, (1 << 128) + 7] + [d.fr_int() for _ in range(60)]
    for i, a in enumerate(vals):
        b = vals[(i * 7 + 3) % len(vals)]
        fa, fb, z = fr_of(lib, i2b(a)), fr_of(lib, i2b(b)), Fr()
        lib.mclBnFr_mul(ctypes.byref(z), ctypes.byref(fa), ctypes.byref(fb))
        assert enc(lib, z) == o.fr_mul(i2b(a), i2b(b)) == i2b(a * b)
        lib.mclBnFr_add(ctypes.byref(z), ctypes.byref(fa), ctypes.byref(fb))
        assert enc(lib, z) == o.fr_add(i2b(a), i2b(b))
        lib.mclBnFr_sub(ctypes.byref(z), ctypes.byref(fa), ctypes.byref(fb))
        assert enc(lib, z) == i2b(a - b)
        lib.mclBnFr_neg(ctypes.byref(z), ctypes.byref(fa))
        assert enc(lib, z) == i2b(-a)
        lib.mclBnFr_sqr(ctypes.byref(z), ctypes.byref(fa))
        assert enc(lib, z) == i2b(a * a)
        lib.mclBnFr_inv(ctypes.byref(z), ctypes.byref(fa))
        assert enc(lib, z) == i2b(pow(a, R - 2, R))          # mcl: the inverse of zero is zero
        if b % R:
            lib.mclBnFr_div(ctypes.byref(z), ctypes.byref(fa), ctypes.byref(fb))
            assert enc(lib, z) == i2b(a * pow(b, R - 2, R))
        assert lib.mclBnFr_isZero(ctypes.byref(fa)) == (a % R == 0)
        assert lib.mclBnFr_isOne(ctypes.byref(fa)) == (a % R == 1)
        assert lib.mclBnFr_isValid(ctypes.byref(fa)) == 1


def test_encodings_and_setters(lib):
    x = Fr()
    for v in (0, 1, -1, -5, 2 ** 62, -(2 ** 63), 2 ** 63 - 1):
        assert lib.mclBnFr_setInt(ctypes.byref(x), v) == 0
        assert enc(lib, x) == o.fr_from_int(v) == i2b(v)
    # non-canonical encodings are rejected (mcl deserialize)
    for bad in (R, R + 1, 2 ** 256 - 1):
        assert lib.mclBnFr_deserialize(ctypes.byref(x), bad.to_bytes(32, "little"), 32) == 0
    assert lib.mclBnFr_deserialize(ctypes.byref(x), b"\x01" * 31, 31) == 0
    # setLittleEndian (mcl setArrayMask): 255-bit mask, then 254 bits if still >= r
    d = Drbg(b"fr-le")
    for n in (0, 1, 16, 31, 32, 40, 64):
        for _ in range(8):
            buf = d.bytes(n)
            v = int.from_bytes(buf[:32], "little") & ((1 << 255) - 1)
            if v >= R:
                v &= (1 << 254) - 1
            assert lib.mclBnFr_setLittleEndian(ctypes.byref(x), buf, n) == 0
            assert enc(lib, x) == v.to_bytes(32, "little")
    for _ in range(32):
        assert lib.mclBnFr_setByCSPRNG(ctypes.byref(x)) == 0
        assert lib.mclBnFr_isValid(ctypes.byref(x)) == 1
        assert int.from_bytes(enc(lib, x), "little") < R


def test_lagrange_and_polynomial_match_oracle(lib):
    d = Drbg(b"fr-lagr")
    for k in (1, 2, 5, 17):
        xs = [i2b(d.fr_int() or 1) for _ in range(k)]
        ys = [d.fr() for _ in range(k)]
        xa = (Fr * k)(*[fr_of(lib, b) for b in xs])
        ya = (Fr * k)(*[fr_of(lib, b) for b in ys])
        out = Fr()
        assert lib.mclBn_FrLagrangeInterpolation(ctypes.byref(out), xa, ya, k) == 0
        assert enc(lib, out) == o.fr_lagrange(xs, ys)
        coeffs = [d.fr() for _ in range(k)]
        ca = (Fr * k)(*[fr_of(lib, b) for b in coeffs])
        x = d.fr()
        assert lib.mclBn_FrEvaluatePolynomial(ctypes.byref(out), ca, k, ctypes.byref(fr_of(lib, x))) == 0
        assert enc(lib, out) == o.fr_eval_poly(coeffs, x)
    # zero or repeated abscissae fail, as mcl's
    xa = (Fr * 2)(fr_of(lib, i2b(3)), fr_of(lib, i2b(3)))
    assert lib.mclBn_FrLagrangeInterpolation(ctypes.byref(out), xa, xa, 2) != 0
    xa = (Fr * 2)(fr_of(lib, i2b(0)), fr_of(lib, i2b(3)))
    assert lib.mclBn_FrLagrangeInterpolation(ctypes.byref(out), xa, xa, 2) != 0
    assert lib.mclBn_FrEvaluatePolynomial(ctypes.byref(out), xa, 0, ctypes.byref(out)) != 0
