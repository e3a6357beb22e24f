"""tests/pyref/bls12_381.py — TEST INFRASTRUCTURE: an independent pure-Python restatement of the BLS12-381 pieces the
TPKE / threshold-signature path uses, written to cross-check the C oracle (oracle/bls.c) with different algorithms:

  * Fp12 is the flat ring Fp[w] / (w^12 - 2 w^6 + 2) (w^6 = xi = 1 + i), not the oracle's Fp2/Fp6/Fp12 tower; the
    tower form appears only when serialising GT elements in mcl's layout (c0.c0, c0.c1, c0.c2, c1.c0, c1.c1, c1.c2).
  * Points are affine with Python-integer field inverses; the Miller loop keeps T on the twist and evaluates each line
    in Fp12 through the untwist (x, y) -> (x / w^2, y / w^3); the final exponentiation is one plain power by
    (p^12 - 1) / r (no easy / hard split, no cyclotomic squaring).
  * psi (untwist - Frobenius - twist) is computed from its definition with powers of xi.
  * Hash-to-G2 follows mcl's MapTo::calcBN description (SW map on y^2 = x^3 + 4(1 + i), t = (Fp::setHashOf(msg), 0))
    and Budroni-Pintore cofactor clearing; like the oracle it is parity-unpinned against MCL itself.

Serialisation follows SURVEY.md Appendix A (pinned by the reference's SerializationTest vectors).  Slow (a pairing
check is ~1 s); used on small transcript samples only.
"""
import hashlib

P = 0x1A0111EA397FE69A4B1BA7B6434BACD764774B84F38512BF6730D2A0F6B0F6241EABFFFEB153FFFFB9FEFFFFFFFFAAAB
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
Z = -0xD201000000010000


# ------------------------------------------------------------------------------------------------ Fp, Fp2
def inv(a):
    return pow(a, P - 2, P)


def sqrt_fp(a):
    """mcl Fp::squareRoot for p = 3 mod 4: a^((p+1)/4), or None"""
    y = pow(a % P, (P + 1) // 4, P)
    return y if y * y % P == a % P else None


def f2add(x, y): return ((x[0] + y[0]) % P, (x[1] + y[1]) % P)
def f2sub(x, y): return ((x[0] - y[0]) % P, (x[1] - y[1]) % P)
def f2neg(x): return ((-x[0]) % P, (-x[1]) % P)
def f2mul(x, y): return ((x[0] * y[0] - x[1] * y[1]) % P, (x[0] * y[1] + x[1] * y[0]) % P)
def f2conj(x): return (x[0], (-x[1]) % P)
def f2inv(x):
    n = inv((x[0] * x[0] + x[1] * x[1]) % P)
    return (x[0] * n % P, (-x[1]) * n % P)


def f2pow(x, e):
    r = (1, 0)
    while e:
        if e & 1:
            r = f2mul(r, x)
        x = f2mul(x, x)
        e >>= 1
    return r


def f2sqrt(x):
    """mcl Fp2::squareRoot root choice (norm method): b == 0 -> (sqrt a, 0) or (0, sqrt -a); otherwise
    c = sqrt(a^2 + b^2), d = sqrt((a + c) / 2) or sqrt((a - c) / 2), root = (d, b / 2d)"""
    a, b = x
    if b == 0:
        s = sqrt_fp(a)
        if s is not None:
            return (s, 0)
        s = sqrt_fp(-a)
        return None if s is None else (0, s)
    c = sqrt_fp(a * a + b * b)
    if c is None:
        return None
    half = inv(2)
    d = sqrt_fp((a + c) * half)
    if d is None:
        d = sqrt_fp((a - c) * half)
        if d is None:
            return None
    return (d, b * inv(2 * d) % P)


XI = (1, 1)
B1 = 4
B2 = (4, 4)          # 4 xi


# ------------------------------------------------------------------------------------------------ flat Fp12
def e_zero(): return [0] * 12
def e_one():
    e = [0] * 12
    e[0] = 1
    return e


def e_mul(a, b):
    t = [0] * 23
    for i, ai in enumerate(a):
        if ai:
            for j, bj in enumerate(b):
                if bj:
                    t[i + j] += ai * bj
    for k in range(22, 11, -1):           # w^12 = 2 w^6 - 2
        c = t[k]
        if c:
            t[k - 6] += 2 * c
            t[k - 12] -= 2 * c
    return [x % P for x in t[:12]]


def e_pow(a, e):
    r = e_one()
    for bit in bin(e)[2:]:
        r = e_mul(r, r)
        if bit == "1":
            r = e_mul(r, a)
    return r


def e_from_f2(x, k=0):
    """(a + b i) w^k with i = w^6 - 1"""
    e = [0] * 12
    a, b = x
    for kk, c in ((k, a - b), (k + 6, b)):
        if kk < 12:
            e[kk] = (e[kk] + c) % P
        else:                             # w^12 = 2 w^6 - 2
            e[kk - 6] = (e[kk - 6] + 2 * c) % P
            e[kk - 12] = (e[kk - 12] - 2 * c) % P
    return e


def e_add(a, b): return [(x + y) % P for x, y in zip(a, b)]


def e_conj(a):
    """w -> -w (the p^6 Frobenius: w^(p^6) = -w)"""
    return [c if k % 2 == 0 else (-c) % P for k, c in enumerate(a)]


def gt_bytes(e):
    """mcl GT layout: Fp12 = c0 + c1 w over Fp6 = Fp2[v] (v = w^2); Fp2 coefficient of w^j is x_j + y_j i with
    c_j = x_j - y_j, c_(j+6) = y_j; serialised j = 0, 2, 4, 1, 3, 5, each as a (48 B LE), b (48 B LE)"""
    out = b""
    for j in (0, 2, 4, 1, 3, 5):
        y = e[j + 6]
        x = (e[j] + y) % P
        out += x.to_bytes(48, "little") + y.to_bytes(48, "little")
    return out


# ------------------------------------------------------------------------------------------------ curves (affine)
def g1_add(p, q):
    if p is None:
        return q
    if q is None:
        return p
    if p[0] == q[0]:
        if (p[1] + q[1]) % P == 0:
            return None
        lam = 3 * p[0] * p[0] * inv(2 * p[1]) % P
    else:
        lam = (q[1] - p[1]) * inv(q[0] - p[0]) % P
    x = (lam * lam - p[0] - q[0]) % P
    return x, (lam * (p[0] - x) - p[1]) % P


def g1_neg(p): return None if p is None else (p[0], (-p[1]) % P)


def g1_mul(p, k):
    if k < 0:
        return g1_mul(g1_neg(p), -k)
    r = None
    while k:
        if k & 1:
            r = g1_add(r, p)
        p = g1_add(p, p)
        k >>= 1
    return r


def g2_add(p, q):
    if p is None:
        return q
    if q is None:
        return p
    if p[0] == q[0]:
        if f2add(p[1], q[1]) == (0, 0):
            return None
        lam = f2mul(f2mul((3, 0), f2mul(p[0], p[0])), f2inv(f2add(p[1], p[1])))
    else:
        lam = f2mul(f2sub(q[1], p[1]), f2inv(f2sub(q[0], p[0])))
    x = f2sub(f2sub(f2mul(lam, lam), p[0]), q[0])
    return x, f2sub(f2mul(lam, f2sub(p[0], x)), p[1])


def g2_neg(p): return None if p is None else (p[0], f2neg(p[1]))


def g2_mul(p, k):
    if k < 0:
        return g2_mul(g2_neg(p), -k)
    r = None
    while k:
        if k & 1:
            r = g2_add(r, p)
        p = g2_add(p, p)
        k >>= 1
    return r


# psi = twist o Frobenius o untwist: (x, y) -> (conj(x) xi^((1-p)/3), conj(y) xi^((1-p)/2))
_PSI_X = f2inv(f2pow(XI, (P - 1) // 3))
_PSI_Y = f2inv(f2pow(XI, (P - 1) // 2))


def g2_psi(p):
    return None if p is None else (f2mul(f2conj(p[0]), _PSI_X), f2mul(f2conj(p[1]), _PSI_Y))


# ------------------------------------------------------------------------------------------------ serialisation
def g1_from_bytes(b):
    if b == bytes(48):
        return None
    odd = b[47] >> 7
    x = int.from_bytes(b[:47] + bytes([b[47] & 0x7F]), "little")
    if x >= P:
        raise ValueError("x >= p")
    y = sqrt_fp(x ** 3 + B1)
    if y is None:
        raise ValueError("not on curve")
    if (y & 1) != odd:
        y = (-y) % P
    return (x, y)


def g1_to_bytes(p):
    if p is None:
        return bytes(48)
    b = bytearray(p[0].to_bytes(48, "little"))
    if p[1] & 1:
        b[47] |= 0x80
    return bytes(b)


def g2_from_bytes(b):
    if b == bytes(96):
        return None
    odd = b[95] >> 7
    xa = int.from_bytes(b[:48], "little")
    xb = int.from_bytes(b[48:95] + bytes([b[95] & 0x7F]), "little")
    if xa >= P or xb >= P:
        raise ValueError("x >= p")
    x = (xa, xb)
    y = f2sqrt(f2add(f2mul(f2mul(x, x), x), B2))
    if y is None:
        raise ValueError("not on curve")
    if (y[0] & 1) != odd:                  # sign flag = parity of y.a
        y = f2neg(y)
    return (x, y)


def g2_to_bytes(p):
    if p is None:
        return bytes(96)
    b = bytearray(p[0][0].to_bytes(48, "little") + p[0][1].to_bytes(48, "little"))
    if p[1][0] & 1:
        b[95] |= 0x80
    return bytes(b)


# ------------------------------------------------------------------------------------------------ hash to G2
_SQRT_M3 = pow((-3) % P, (P + 1) // 4, P)
_HALF_M1_SQRT_M3 = (_SQRT_M3 - 1) * inv(2) % P


def fp_hash_of(msg):
    """mcl Fp::setHashOf: SHA-512, first 48 bytes little-endian, keep 381 bits, 380 if still >= p"""
    d = hashlib.sha512(msg).digest()
    v = int.from_bytes(d[:48], "little") & ((1 << 381) - 1)
    if v >= P:
        v &= (1 << 380) - 1
    return v


def _legendre(a):
    a %= P
    if a == 0:
        return 0
    return 1 if pow(a, (P - 1) // 2, P) == 1 else -1


def map_to_g2_bn(t):
    """SW map of mcl calcBN for y^2 = x^3 + b, b = 4 xi: w = sqrt(-3) t / (1 + b + t^2); candidates
    x1 = (-1 + sqrt(-3)) / 2 - t w, x2 = -1 - x1, x3 = 1 + 1 / w^2; y negated when the norm of t is a non-residue"""
    leg = _legendre(t[0] * t[0] + t[1] * t[1])
    if leg == 0:
        return None
    den = f2add(f2add(f2mul(t, t), B2), (1, 0))
    if den == (0, 0):
        return None
    w = f2mul(f2mul(f2inv(den), (_SQRT_M3, 0)), t)
    x1 = f2add(f2neg(f2mul(t, w)), (_HALF_M1_SQRT_M3, 0))
    x2 = f2sub(f2neg(x1), (1, 0))
    x3 = f2add(f2inv(f2mul(w, w)), (1, 0))
    for x in (x1, x2, x3):
        y = f2sqrt(f2add(f2mul(f2mul(x, x), x), B2))
        if y is not None:
            return (x, f2neg(y) if leg < 0 else y)
    return None


def clear_cofactor_g2(p):
    """Budroni-Pintore: (z^2 - z - 1) P + psi((z - 1) P) + psi^2(2 P)"""
    t1 = g2_mul(p, Z * Z - Z - 1)
    t2 = g2_psi(g2_mul(p, Z - 1))
    t3 = g2_psi(g2_psi(g2_add(p, p)))
    return g2_add(g2_add(t1, t2), t3)


def hash_to_g2(msg):
    q = map_to_g2_bn((fp_hash_of(msg), 0))
    if q is None:
        raise ValueError("map failed")
    return clear_cofactor_g2(q)


# ------------------------------------------------------------------------------------------------ pairing
def _line(lam, xt, yt, p):
    """line through T (on the twist, slope lam) evaluated at P = (xp, yp), multiplied by w^3 (an Fp4 factor that the
    final exponentiation removes): yp w^3 - lam xp w^2 + (lam xt - yt)"""
    xp, yp = p
    e = e_zero()
    e[3] = yp % P
    e = e_add(e, e_from_f2(f2neg((lam[0] * xp % P, lam[1] * xp % P)), 2))
    return e_add(e, e_from_f2(f2sub(f2mul(lam, xt), yt), 0))


def miller(p, q):
    """f_{|z|,Q}(P) conjugated (z < 0); vertical lines omitted (they lie in a proper subfield)"""
    if p is None or q is None:
        return e_one()
    f = e_one()
    t = q
    for bit in bin(-Z)[3:]:
        lam = f2mul(f2mul((3, 0), f2mul(t[0], t[0])), f2inv(f2add(t[1], t[1])))
        f = e_mul(e_mul(f, f), _line(lam, t[0], t[1], p))
        t = g2_add(t, t)
        if bit == "1":
            lam = f2mul(f2sub(q[1], t[1]), f2inv(f2sub(q[0], t[0])))
            f = e_mul(f, _line(lam, t[0], t[1], p))
            t = g2_add(t, q)
    return e_conj(f)


FE_EXP = (P ** 12 - 1) // R


def pairing(p, q):
    """the reduced Tate-style optimal-ate pairing f^((p^12 - 1) / r) (the oracle and mcl return its cube)"""
    return e_pow(miller(p, q), FE_EXP)


def pairing_check(p1, q1, p2, q2):
    """e(p1, q1) == e(p2, q2), as one product of Miller loops and one final exponentiation"""
    f = e_mul(miller(p1, q1), miller(g1_neg(p2), q2))
    return e_pow(f, FE_EXP) == e_one()


# ------------------------------------------------------------------------------------------------ Lagrange
def lagrange_coeffs(xs):
    out = []
    for i, xi in enumerate(xs):
        num, den = 1, 1
        for j, xj in enumerate(xs):
            if j != i:
                num = num * xj % R
                den = den * (xj - xi) % R
        out.append(num * pow(den, R - 2, R) % R)
    return out
