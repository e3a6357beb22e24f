"""The device's binary-GCD Fp inversion (field.hpp fp_inv_gcd) restated step for step in Python integers: 26 outer
iterations of 30 divsteps on the 62-bit approximations (low 30 bits, top 32 bits below the common bit length), the
exact signed updates of a, b, the coefficients u, v with one 32-bit Montgomery reduction each, and the final
Montgomery product by LCB_BINV_C.  Checks the bound the device code relies on (|f|, |g| <= 2^30; the reduced
coefficient in (-p/2, 3p/2)), that b ends at 1, that the result is the Montgomery form of the inverse, and that the
generated constant equals 2^52 R^3 mod p (CPU test)."""
import os
import random
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = 0x1a0111ea397fe69a4b1ba7b6434bacd764774b84f38512bf6730d2a0f6b0f6241eabfffeb153ffffb9feffffffffaaab
R = 1 << 384
PINV32 = (-pow(P, -1, 1 << 32)) % (1 << 32)


def _const(name):
    text = open(os.path.join(ROOT, "lachain_amd", "csrc", "bls_constants.hpp")).read()
    words = re.search(name + r"\[12\] = \{([^}]*)\}", text).group(1)
    return sum(int(w.strip().rstrip("u"), 16) << (32 * i) for i, w in enumerate(words.split(",")))


def _mont_lin(u, v, f, g):
    t = u * f + v * g
    q = ((t & 0xffffffff) * PINV32) & 0xffffffff
    t += q * P
    assert t % (1 << 32) == 0
    t >>= 32
    assert -P // 2 - 1 < t < 3 * P // 2 + 1
    return t + P if t < 0 else (t - P if t >= P else t)


def fp_inv_gcd(x_mont, c):
    if x_mont == 0:
        return 0
    a, b, u, v = x_mont, P, 1, 0
    for _ in range(26):
        n = max(a.bit_length(), b.bit_length(), 62)
        s = n - 32
        ab = (a & ((1 << 30) - 1)) | (((a >> s) & 0xffffffff) << 30)
        bb = (b & ((1 << 30) - 1)) | (((b >> s) & 0xffffffff) << 30)
        f0, g0, f1, g1 = 1, 0, 0, 1
        for _ in range(30):
            odd = ab & 1
            if odd and ab < bb:
                ab, bb, f0, g0, f1, g1 = bb, ab, f1, g1, f0, g0
            if odd:
                ab, f0, g0 = ab - bb, f0 - f1, g0 - g1
            ab, f1, g1 = ab >> 1, f1 * 2, g1 * 2
            assert max(abs(f0), abs(g0), abs(f1), abs(g1)) <= 1 << 30
        na, nb = (a * f0 + b * g0) >> 30, (a * f1 + b * g1) >> 30
        assert (a * f0 + b * g0) % (1 << 30) == 0 and (a * f1 + b * g1) % (1 << 30) == 0
        if na < 0:
            na, f0, g0 = -na, -f0, -g0
        if nb < 0:
            nb, f1, g1 = -nb, -f1, -g1
        u, v, a, b = _mont_lin(u, v, f0, g0), _mont_lin(u, v, f1, g1), na, nb
    assert b == 1
    return v * c * pow(R, -1, P) % P              # the Montgomery product fp_mul(v, LCB_BINV_C)


def test_constant_is_2_52_r3():
    assert _const("LCB_BINV_C") == pow(2, 52, P) * pow(R, 3, P) % P


def test_restated_inversion_matches_fermat():
    c = _const("LCB_BINV_C")
    rng = random.Random(20261018)
    xs = [1, 2, 3, P - 1, P - 2, (P - 1) // 2, 1 << 380, (1 << 381) % P] + [rng.randrange(1, P) for _ in range(400)]
    for x in xs:
        xm = x * R % P
        assert fp_inv_gcd(xm, c) == pow(x, -1, P) * R % P, hex(x)
    assert fp_inv_gcd(0, c) == 0
