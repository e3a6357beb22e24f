"""The mcl single-element surface on its batch / cooperative kernels (lcb_host.cpp "mcl surface" section):
mclBn_pairing (one-group nine-lane check), mclBn_finalExp, mclBnG1_mulVec, G1 / G2 Lagrange interpolation and
G1 / G2 EvaluatePolynomial against the oracle, bit-exact on the wire encodings; and the per-thread staging
(single operations from several threads at once).
"""
import ctypes
import threading

import pytest

import oracle as o
from helpers import Drbg, R, gpu_native

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def mcl():
    gpu_native()
    from lachain_amd import mcl as m
    return m


def _mul_vec(mcl, pts, scs):
    from lachain_amd.native import mclBnG1, mclBnFr
    n = len(pts)
    pa = (mclBnG1 * max(1, n))(*[p.v for p in pts])
    sa = (mclBnFr * max(1, n))(*[s.v for s in scs])
    out = mcl.G1()
    f = mcl._f("mclBnG1_mulVec", None, [ctypes.POINTER(mclBnG1), ctypes.POINTER(mclBnG1), ctypes.POINTER(mclBnFr),
                                       ctypes.c_size_t])
    f(ctypes.byref(out.v), pa, sa, n)
    return out


def test_pairing_edge_cases_and_bilinearity(mcl):
    Fr, G1, G2, GT = mcl.Fr, mcl.G1, mcl.G2, mcl.GT
    d = Drbg(b"mcl-pairing")
    for _ in range(3):
        a, b = d.fr(), d.fr()
        A, B = G1.Generator() * Fr.FromBytes(a), G2.Generator() * Fr.FromBytes(b)
        assert GT.Pairing(A, B).ToBytes() == o.pairing(A.ToBytes(), B.ToBytes())
        assert GT.Pairing(-A, B) * GT.Pairing(A, B) == GT.Pairing(G1.Zero(), B)
    assert GT.Pairing(G1.Zero(), G2.Generator()).IsOne()
    assert GT.Pairing(G1.Generator(), G2.Zero()).IsOne()
    assert GT.Pairing(G1.Zero(), G2.Zero()).IsOne()
    # Jacobian inputs (z != 1) give the same value as their affine forms
    A = G1.Generator() + G1.Generator() * Fr.FromInt(5)
    B = G2.Generator() + G2.Generator() * Fr.FromInt(9)
    assert GT.Pairing(A, B).ToBytes() == o.pairing(A.ToBytes(), B.ToBytes())


def test_final_exp_of_miller_loop_is_the_pairing(mcl):
    from lachain_amd.native import mclBnGT, mclBnG1, mclBnG2
    Fr, G1, G2, GT = mcl.Fr, mcl.G1, mcl.G2, mcl.GT
    P = ctypes.POINTER
    ml = mcl._f("mclBn_millerLoop", None, [P(mclBnGT), P(mclBnG1), P(mclBnG2)])
    fe = mcl._f("mclBn_finalExp", None, [P(mclBnGT), P(mclBnGT)])
    d = Drbg(b"mcl-fe")
    A, B = G1.Generator() * Fr.FromBytes(d.fr()), G2.Generator() * Fr.FromBytes(d.fr())
    f, e = GT(), GT()
    ml(ctypes.byref(f.v), ctypes.byref(A.v), ctypes.byref(B.v))
    fe(ctypes.byref(e.v), ctypes.byref(f.v))
    assert e == GT.Pairing(A, B)
    assert e.ToBytes() == o.final_exp(f.ToBytes())


@pytest.mark.parametrize("n", [0, 1, 2, 7, 300, 70000])
def test_mul_vec_matches_oracle(mcl, n):
    Fr, G1 = mcl.Fr, mcl.G1
    d = Drbg(b"mcl-mulvec-%d" % n)
    m = min(n, 24)                        # distinct points; larger n repeats them (the sum is still exact)
    base = [G1.Generator() * Fr.FromBytes(d.fr()) for _ in range(m)]
    if m > 3:
        base[2] = G1.Zero()               # a point at infinity
    pts = [base[i % m] for i in range(n)] if m else []
    scs = [Fr.FromBytes(d.fr()) for _ in range(n)]
    if n > 3:
        scs[1] = Fr.FromInt(0)
        scs[3] = Fr.FromInt(-1)
    got = _mul_vec(mcl, pts, scs)
    # oracle: sum_i s_i P_i with the scalars folded per distinct point
    fold = {}
    for i in range(n):
        fold[i % m] = (fold.get(i % m, 0) + int.from_bytes(scs[i].ToBytes(), "little")) % R
    want = G1.Zero().ToBytes()
    for j, s in fold.items():
        want = o.g1_add(want, o.g1_mul(base[j].ToBytes(), s.to_bytes(32, "little")))
    assert got.ToBytes() == want


def test_pairing_cache_survives_other_mcl_calls(mcl):
    """mclBn_pairing caches G2 line sets per thread; mulVec, Lagrange and EvaluatePolynomial stage their data on the
    same context and must not overwrite a cached set (a cached second pairing was wrong before the cache had a buffer
    of its own)."""
    Fr, G1, G2, GT = mcl.Fr, mcl.G1, mcl.G2, mcl.GT
    d = Drbg(b"mcl-pair-cache")
    A, B = G1.Generator() * Fr.FromBytes(d.fr()), G2.Generator() * Fr.FromBytes(d.fr())
    want = o.pairing(A.ToBytes(), B.ToBytes())
    assert GT.Pairing(A, B).ToBytes() == want
    pts = [G1.Generator() * Fr.FromBytes(d.fr()) for _ in range(22)]
    scs = [Fr.FromBytes(d.fr()) for _ in range(22)]
    _mul_vec(mcl, pts, scs)
    mcl.MclBls12381.LagrangeInterpolate([Fr.FromInt(i + 1) for i in range(8)], pts[:8])
    mcl.MclBls12381.EvaluatePolynomial(pts[:8], scs[0])
    _mul_vec(mcl, pts * 40, scs * 40)                 # 880 terms: the batch kernels' path
    assert GT.Pairing(A, B).ToBytes() == want
    assert GT.Pairing(-A, B) * GT.Pairing(A, B) == GT.Pairing(G1.Zero(), B)


def test_mul_vec_and_lagrange_with_points_outside_g1(mcl):
    """The cooperative ladders split scalars by GLV, valid in G1 only: a term outside G1 (the order-3 point, a random
    on-curve point) sends the call to the exact per-term path, so the result is sum_i [s_i] P_i for any on-curve
    input; the point at infinity and zero scalars are idle terms."""
    from test_gpu_batched import off_subgroup_g1
    Fr, G1 = mcl.Fr, mcl.G1
    d = Drbg(b"mcl-mulvec-off")
    t3 = G1.FromBytes(bytes(47) + b"\x80")
    off = G1.FromBytes(off_subgroup_g1(d))
    good = [G1.Generator() * Fr.FromBytes(d.fr()) for _ in range(6)]
    for case, pts in enumerate((good, good[:3] + [t3] + good[3:], good[:2] + [off], [G1.Zero()] + good[:2])):
        scs = [Fr.FromBytes(d.fr()) for _ in pts]
        scs[-1] = Fr.FromInt(0) if len(pts) == 3 else scs[-1]
        if case == 1:                               # [s] t3 = t3 for s = 1 mod 3: -t3 = (0, 2) serialises as all zeros,
            s3 = int.from_bytes(scs[3].ToBytes(), "little")   # the encoding of infinity, so the expected sum is
            scs[3] = Fr.FromBytes((s3 - s3 % 3 + 1).to_bytes(32, "little"))   # accumulated through t3 itself
        want = G1.Zero().ToBytes()
        for p, s in zip(pts, scs):
            want = o.g1_add(want, o.g1_mul(p.ToBytes(), s.ToBytes()))
        assert _mul_vec(mcl, pts, scs).ToBytes() == want, case
        xs = [Fr.FromInt(i + 1) for i in range(len(pts))]
        got = mcl.MclBls12381.LagrangeInterpolate(xs, pts)
        assert got.ToBytes() == o.g1_lagrange([x.ToBytes() for x in xs], [p.ToBytes() for p in pts]), case


def test_g2_lagrange_and_polynomial_with_points_outside_g2(mcl):
    """G2 Lagrange interpolation and EvaluatePolynomial run their terms on the cooperative GLS ladders when every point
    is in G2; a point outside G2 (on the twist, not in the subgroup) sends the call to its exact path."""
    from test_gpu_batched import off_subgroup_g2
    Fr, G2 = mcl.Fr, mcl.G2
    d = Drbg(b"mcl-g2-off")
    good = [G2.Generator() * Fr.FromBytes(d.fr()) for _ in range(5)]
    off = G2.FromBytes(off_subgroup_g2(d))
    for case, pts in enumerate((good, good[:2] + [off] + good[2:], [G2.Zero()] + good[:3])):
        xs = [Fr.FromInt(3 * i + 2) for i in range(len(pts))]
        got = mcl.MclBls12381.LagrangeInterpolate(xs, pts)
        assert got.ToBytes() == o.g2_lagrange([x.ToBytes() for x in xs], [p.ToBytes() for p in pts]), case
        x = Fr.FromBytes(d.fr())
        acc = pts[-1].ToBytes()
        for c in reversed(pts[:-1]):
            acc = o.g2_add(o.g2_mul(acc, x.ToBytes()), c.ToBytes())
        assert mcl.MclBls12381.EvaluatePolynomial(pts, x).ToBytes() == acc, case


@pytest.mark.parametrize("g", [1, 2])
def test_lagrange_points_match_oracle(mcl, g):
    Fr = mcl.Fr
    G = mcl.G1 if g == 1 else mcl.G2
    lag = o.g1_lagrange if g == 1 else o.g2_lagrange
    d = Drbg(b"mcl-lagr-%d" % g)
    for k in (2, 3, 8, 22):
        xs = [Fr.FromInt(i + 1) for i in range(k)]
        ys = [G.Generator() * Fr.FromBytes(d.fr()) for _ in range(k)]
        ys[0] = ys[0] + G.Generator()     # a Jacobian record with z != 1
        got = mcl.MclBls12381.LagrangeInterpolate(xs, ys)
        assert got.ToBytes() == lag([x.ToBytes() for x in xs], [y.ToBytes() for y in ys])
    with pytest.raises(ValueError):
        mcl.MclBls12381.LagrangeInterpolate([Fr.FromInt(1), Fr.FromInt(1)], [G.Generator(), G.Generator()])
    with pytest.raises(ValueError):
        mcl.MclBls12381.LagrangeInterpolate([Fr.FromInt(0), Fr.FromInt(1)], [G.Generator(), G.Generator()])


@pytest.mark.parametrize("g", [1, 2])
def test_evaluate_polynomial_matches_horner(mcl, g):
    Fr = mcl.Fr
    G = mcl.G1 if g == 1 else mcl.G2
    mul, add = (o.g1_mul, o.g1_add) if g == 1 else (o.g2_mul, o.g2_add)
    d = Drbg(b"mcl-eval-%d" % g)
    for n in (1, 2, 8):
        cs = [G.Generator() * Fr.FromBytes(d.fr()) for _ in range(n)]
        for x in (Fr.FromInt(0), Fr.FromInt(1), Fr.FromInt(-3), Fr.FromBytes(d.fr())):
            got = mcl.MclBls12381.EvaluatePolynomial(cs, x)
            acc = cs[-1].ToBytes()
            for c in reversed(cs[:-1]):
                acc = add(mul(acc, x.ToBytes()), c.ToBytes())
            assert got.ToBytes() == acc
    if g == 1:
        cs = [G.Generator() * Fr.FromBytes(d.fr()) for _ in range(4)]
        x = Fr.FromBytes(d.fr())
        assert mcl.MclBls12381.EvaluatePolynomial(cs, x).ToBytes() == o.g1_eval_poly([c.ToBytes() for c in cs],
                                                                                     x.ToBytes())


def test_g1_evaluate_polynomial_off_subgroup_and_long(mcl):
    """G1 EvaluatePolynomial runs as independent terms [x^i mod #E(Fp)] c_i (lcb_host.cpp eval_poly_g1_terms): the
    Horner value for coefficients outside G1 too (the order-3 point and a random on-curve point, G1.FromBytes accepts
    them), for x = 0, 1, -1, -3 and random x, for a polynomial longer than one block of terms, and with the point at
    infinity among the coefficients."""
    from test_gpu_batched import off_subgroup_g1
    Fr, G1 = mcl.Fr, mcl.G1
    d = Drbg(b"mcl-eval-off")
    t3 = bytes(47) + b"\x80"                        # (0, p - 2): order 3
    cs = [G1.Generator() * Fr.FromBytes(d.fr()) for _ in range(6)]
    cs[1] = G1.FromBytes(t3)
    cs[3] = G1.FromBytes(off_subgroup_g1(d))
    cs[4] = cs[4] + G1.FromBytes(t3)
    cs[5] = G1.Zero()                               # the point at infinity
    for x in (Fr.FromInt(0), Fr.FromInt(1), Fr.FromInt(-1), Fr.FromInt(-3), Fr.FromBytes(d.fr())):
        got = mcl.MclBls12381.EvaluatePolynomial(cs, x)
        assert got.ToBytes() == o.g1_eval_poly([c.ToBytes() for c in cs], x.ToBytes())
    long_cs = [G1.Generator() * Fr.FromBytes(d.fr()) for _ in range(300)]
    x = Fr.FromBytes(d.fr())
    got = mcl.MclBls12381.EvaluatePolynomial(long_cs, x)
    assert got.ToBytes() == o.g1_eval_poly([c.ToBytes() for c in long_cs], x.ToBytes())


def test_single_operations_from_many_threads(mcl):
    # each thread owns its staging buffers and stream: results never mix
    Fr, G1, G2, GT = mcl.Fr, mcl.G1, mcl.G2, mcl.GT
    d = Drbg(b"mcl-threads")
    jobs = [(d.fr(), d.fr()) for _ in range(8)]
    want = [o.pairing(o.g1_mul(o.g1_gen(), a), o.g2_mul(o.g2_gen(), b)) for a, b in jobs]
    got = [None] * len(jobs)
    errs = []

    def work(i):
        try:
            a, b = jobs[i]
            for _ in range(3):
                A = G1.Generator() * Fr.FromBytes(a)
                B = G2.Generator() * Fr.FromBytes(b)
                got[i] = GT.Pairing(A, B).ToBytes()
        except Exception as e:          # noqa: BLE001 — reported below
            errs.append(e)

    ts = [threading.Thread(target=work, args=(i,)) for i in range(len(jobs))]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    assert got == want


def test_thread_churn_reuses_retired_staging(mcl):
    """Threads that exit hand their staging and implicit contexts to the next threads (no HIP call at thread exit):
    four generations of six short-lived threads, each doing a scalar multiplication, all exact"""
    Fr, G1 = mcl.Fr, mcl.G1
    errs, got = [], {}

    def work(gen, i):
        try:
            k = 1000 * gen + i + 2
            got[(gen, i)] = (G1.Generator() * Fr.FromInt(k)).ToBytes()
        except Exception as e:          # noqa: BLE001 — reported below
            errs.append(e)

    for gen in range(4):
        ts = [threading.Thread(target=work, args=(gen, i)) for i in range(6)]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
    assert not errs, errs
    for (gen, i), b in got.items():
        assert b == o.g1_mul(o.g1_gen(), o.fr(1000 * gen + i + 2)), (gen, i)


def test_pairing_line_cache(mcl):
    """mclBn_pairing keeps the line sets of the last 32 distinct G2 arguments per thread: hits, misses and evictions
    (40 distinct Q, revisited out of order) all give the oracle's GT value"""
    Fr, G1, G2, GT = mcl.Fr, mcl.G1, mcl.G2, mcl.GT
    P = G1.Generator() * Fr.FromInt(7)
    Qs = [G2.Generator() * Fr.FromInt(i + 2) for i in range(40)]
    want = {}
    order = list(range(40)) + [39, 0, 5, 38, 1, 1, 20, 33, 8, 39]
    for i in order:
        if i not in want:
            want[i] = o.pairing(P.ToBytes(), Qs[i].ToBytes())
        assert GT.Pairing(P, Qs[i]).ToBytes() == want[i], i
    # the same Q with another P hits the cache
    P2 = G1.Generator() * Fr.FromInt(11)
    assert GT.Pairing(P2, Qs[39]).ToBytes() == o.pairing(P2.ToBytes(), Qs[39].ToBytes())
