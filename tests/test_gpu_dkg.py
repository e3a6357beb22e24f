"""Trustless-DKG G1 work on the GPU against the oracle's literal restatement of
Commitment.Evaluate (src/Lachain.Consensus/ThresholdKeygen/Data/Commitment.cs:23-53: (D+1)^2 G1 x Fr products)
and against known answers G * f(x, y) computed from the polynomial's Fr coefficients.  N=256, F=85 (degree 85,
3,741 commitment coefficients) as in BASELINE configs[4]'s validator set, plus small degrees and edge cases
(x = 0 for TryGetKeys' Evaluate(0), negative x, a malformed coefficient)."""
import pytest

import oracle as o
from helpers import Drbg, R, gpu_native

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nat():
    return gpu_native()


def index(i, j):
    if i > j:
        i, j = j, i
    return i * (i + 1) // 2 + j


def commitment(nat, d, degree):
    """a symmetric bivariate polynomial's coefficients (Fr) and its G1 commitment (ThresholdKeygen/Data/State.cs)"""
    n = (degree + 1) * (degree + 2) // 2
    c = [d.fr_int() for _ in range(n)]
    pts = nat.mul_batch(1, None, [o.fr(v) for v in c], generator=True)
    return c, pts


def f_xy(c, degree, x, y):
    return sum(c[index(i, j)] * pow(x, i, R) * pow(y, j, R) for i in range(degree + 1) for j in range(degree + 1)) % R


def test_commitment_eval_n256_f85(nat):
    n, degree = 256, 85
    d = Drbg(b"gpu-dkg-n256")
    c, pts = commitment(nat, d, degree)
    x0 = 6                                          # HandleSendValue: Evaluate(myIdx + 1, sender + 1), myIdx = 5
    queries = [(0, x0, s + 1) for s in range(n)]
    got = nat.dkg_commitment_eval([pts], degree, queries)
    G = o.g1_gen()
    for (_, x, y), g in zip(queries, got):
        assert g == o.g1_mul(G, o.fr(f_xy(c, degree, x, y))), y
    # the reference's own (D+1)^2-product evaluation, once
    assert got[17] == o.dkg_commitment_eval(pts, degree, x0, 18)
    # HandleCommit's row Evaluate(myIdx + 1) and TryGetKeys' Evaluate(0)
    rows = nat.dkg_commitment_rows([pts], degree, [(0, x0), (0, 0)])
    for q, x in enumerate((x0, 0)):
        for i in range(degree + 1):
            e = sum(c[index(i, j)] * pow(x, j, R) for j in range(degree + 1)) % R
            assert rows[q][i] == o.g1_mul(G, o.fr(e)), (x, i)
    assert rows[0] == o.dkg_commitment_row(pts, degree, x0)


def test_commitment_eval_small_degrees_and_edges(nat):
    d = Drbg(b"gpu-dkg-small")
    for degree in (0, 1, 2, 7):
        comms = [commitment(nat, d, degree) for _ in range(3)]
        pts = [p for _, p in comms]
        queries = [(k % 3, x, y) for k, (x, y) in enumerate([(1, 1), (2, 5), (0, 3), (7, 0), (-3, 4), (256, 255),
                                                             (5, -2), (100000, 3)])]
        got = nat.dkg_commitment_eval(pts, degree, queries)
        for (ci, x, y), g in zip(queries, got):
            assert g == o.dkg_commitment_eval(pts[ci], degree, x, y), (degree, x, y)
        rows = nat.dkg_commitment_rows(pts, degree, [(1, 3), (2, -1)])
        assert rows[0] == o.dkg_commitment_row(pts[1], degree, 3)
        assert rows[1] == o.dkg_commitment_row(pts[2], degree, -1)
    # a malformed coefficient fails only the queries of its commitment; an out-of-range commitment index fails too
    c, p = commitment(nat, d, 2)
    bad = list(p)
    bad[3] = b"\xff" * 47 + b"\x1f"   # x >= p: G1.FromBytes rejects it
    assert not o.g1_valid(bad[3])
    got = nat.dkg_commitment_eval([p, bad], 2, [(0, 1, 2), (1, 1, 2), (2, 1, 2)])
    assert got[0] == o.g1_mul(o.g1_gen(), o.fr(f_xy(c, 2, 1, 2))) and got[1] is None and got[2] is None


def test_g1_eval_poly_batch(nat):
    # TryGetKeys: pubKeys[i] = EvaluatePolynomial(pubKeyPoly, i), i = 0..N (TrustlessKeygen.cs:172-174)
    d = Drbg(b"gpu-dkg-poly")
    a = [d.fr_int() for _ in range(86)]
    coeffs = nat.mul_batch(1, None, [o.fr(v) for v in a], generator=True)
    xs = list(range(257)) + [-5, 70000]
    got = nat.g1_eval_poly_batch(coeffs, xs)
    G = o.g1_gen()
    for x, g in zip(xs, got):
        assert g == o.g1_mul(G, o.fr(sum(c * pow(x, k, R) for k, c in enumerate(a)) % R)), x
    for x in (0, 1, 256, -5):
        assert got[xs.index(x)] == o.g1_eval_poly(coeffs, o.fr(x))


def test_commitment_off_subgroup_coefficients(nat):
    """A Byzantine dealer's commitment with coefficients outside G1 (G1.FromBytes accepts them, SURVEY A.8;
    TrustlessKeygen never calls Commitment.IsValid): one coefficient carries the order-3 point (0, -2), one is a random
    on-curve point.  With x^i y^j >= r the powers' reduction mod r changes the result, so the GPU must take the
    reference's own form [y^j mod r]([x^i mod r] C) (Commitment.cs:23-37) — equal to the oracle's literal evaluation —
    and the rows (Commitment.cs:39-53) likewise; an honest commitment in the same call is unaffected."""
    from test_gpu_batched import off_subgroup_g1
    d = Drbg(b"gpu-dkg-off-subgroup")
    degree = 40
    c, pts = commitment(nat, d, degree)
    t3 = bytes(47) + b"\x80"                        # x = 0, odd y: (0, p - 2), order 3
    assert o.g1_valid(t3) and not o.g1_in_subgroup(t3)
    bad = list(pts)
    bad[index(3, 5)] = o.g1_add(pts[index(3, 5)], t3)
    bad[index(0, 7)] = off_subgroup_g1(d)
    queries = [(1, 200, 150), (1, 7, 230), (0, 200, 150), (1, 255, 255)]
    got = nat.dkg_commitment_eval([pts, bad], degree, queries)
    for (k, x, y), g in zip(queries, got):
        assert g == o.dkg_commitment_eval([pts, bad][k], degree, x, y), (k, x, y)
    # the honest commitment's value is still G * f(x, y)
    assert got[2] == o.g1_mul(o.g1_gen(), o.fr(f_xy(c, degree, 200, 150)))
    rows = nat.dkg_commitment_rows([pts, bad], degree, [(1, 200), (0, 200)])
    assert rows[0] == o.dkg_commitment_row(bad, degree, 200)
    assert rows[1] == o.dkg_commitment_row(pts, degree, 200)
    # MclBls12381.EvaluatePolynomial with a negative x: Fr.FromInt(x) = r - |x| multiplies the off-subgroup terms
    coeffs = bad[:12]
    for x in (-3, 5):
        xb = o.fr(x % R)
        assert nat.g1_eval_poly_batch(coeffs, [x]) == [o.g1_eval_poly(coeffs, xb)], x
