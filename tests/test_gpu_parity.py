"""GPU parity tests: liblachain_bls.so (gfx950 kernels, called through the C ABI) against oracle/
(the C restatement of the MCL path, pinned by tests/test_oracle.py).  Integer/byte work: every
comparison is bit-exact (serialized G1/G2/GT bytes, accept/reject bitmaps).
"""
import pytest

import oracle as o
from helpers import Drbg, gpu_native, kats

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def nat():
    return gpu_native()


@pytest.fixture(scope="module")
def mcl(nat):
    from lachain_amd import mcl as m
    return m


# ------------------------------------------------------------------ MCL-shaped single operations
def test_serialization_kats(mcl):
    # test/Lachain.CryptoTest/SerializationTest.cs:20-57 through the mcl-shaped ABI
    k = kats()
    Fr, G1, G2 = mcl.Fr, mcl.G1, mcl.G2
    assert Fr.FromInt(0).ToBytes().hex() == k["fr_0"]["hex"]
    assert Fr.FromInt(1).ToBytes().hex() == k["fr_1"]["hex"]
    assert G1.Zero().ToBytes().hex() == k["g1_zero"]["hex"]
    assert G1.Generator().ToBytes().hex() == k["g1_generator"]["hex"]
    assert (G1.Generator() * Fr.FromInt(2)).ToBytes().hex() == k["g1_generator_x2"]["hex"]
    assert G2.Zero().ToBytes().hex() == k["g2_zero"]["hex"]
    assert G2.Generator().ToBytes().hex() == k["g2_generator"]["hex"]
    assert (G2.Generator() * Fr.FromInt(2)).ToBytes().hex() == k["g2_generator_x2"]["hex"]
    fr = Fr.GetRandom()
    assert Fr.FromBytes(fr.ToBytes()) == fr
    g1 = G1.Generator() * Fr.GetRandom()
    assert G1.FromBytes(g1.ToBytes()) == g1


def test_fr_and_group_ops_match_oracle(mcl):
    Fr, G1, G2 = mcl.Fr, mcl.G1, mcl.G2
    d = Drbg(b"gpu-fr-ops")
    for _ in range(4):
        a, b = d.fr(), d.fr()
        fa, fb = Fr.FromBytes(a), Fr.FromBytes(b)
        assert (fa + fb).ToBytes() == o.fr_add(a, b)
        assert (fa * fb).ToBytes() == o.fr_mul(a, b)
        assert (fa - fb).ToBytes() == (o.fr((int.from_bytes(a, "little") - int.from_bytes(b, "little"))))
        inv = fa.Inverse()
        assert (inv * fa).ToBytes() == o.fr(1)
        A = G1.Generator() * fa
        B = G2.Generator() * fb
        assert A.ToBytes() == o.g1_mul(o.g1_gen(), a)
        assert B.ToBytes() == o.g2_mul(o.g2_gen(), b)
        assert (A + A).ToBytes() == o.g1_add(A.ToBytes(), A.ToBytes())
        assert (B + G2.Generator()).ToBytes() == o.g2_add(B.ToBytes(), o.g2_gen())
        assert (-A).ToBytes() == o.g1_neg(A.ToBytes())
        assert A.IsValid() and B.IsValid()


def test_pairing_matches_oracle(mcl):
    Fr, G1, G2, GT = mcl.Fr, mcl.G1, mcl.G2, mcl.GT
    d = Drbg(b"gpu-pairing")
    a, b = d.fr(), d.fr()
    A = G1.Generator() * Fr.FromBytes(a)
    B = G2.Generator() * Fr.FromBytes(b)
    e = GT.Pairing(A, B)
    assert e.ToBytes() == o.pairing(A.ToBytes(), B.ToBytes())
    # MclTests.cs:64-75 bilinearity
    e0 = GT.Pairing(G1.Generator(), G2.Generator())
    assert GT.Pow(e0, Fr.FromBytes(a) * Fr.FromBytes(b)) == e


def test_hash_to_g2_matches_oracle(nat):
    d = Drbg(b"gpu-h2g2")
    msgs = [b"", b"\x00", b"lachain"] + [d.bytes(n) for n in (1, 24, 47, 48, 80, 111, 112, 200, 300)]
    got = nat.g2_hash_batch(msgs)
    for m, h in zip(msgs, got):
        assert h == o.g2_hash(m), m.hex()


def test_scalar_mul_batches_match_oracle(nat):
    d = Drbg(b"gpu-mul")
    n = 300
    ks = [d.fr() for _ in range(n)]
    ks[0] = o.fr(0)
    ks[1] = o.fr(1)
    g1s = nat.mul_batch(1, None, ks, generator=True)
    g2s = nat.mul_batch(2, None, ks[:40], generator=True)
    for i in range(0, n, 7):
        assert g1s[i] == o.g1_mul(o.g1_gen(), ks[i])
    for i in range(40):
        assert g2s[i] == o.g2_mul(o.g2_gen(), ks[i])
    # variable base
    pts = g1s[:50]
    ks2 = [d.fr() for _ in range(50)]
    out = nat.mul_batch(1, pts, ks2)
    for i in range(0, 50, 5):
        assert out[i] == o.g1_mul(pts[i], ks2[i])


# ------------------------------------------------------------------ TPKE
def _tpke_setup(d, n, f, n_cts, vlen=32):
    coeffs = [d.fr() for _ in range(f + 1)]  # DKG-style keys of degree F
    x = [o.fr_eval_poly(coeffs, o.fr(i + 1)) for i in range(n)]
    y = o.g1_mul(o.g1_gen(), o.fr_eval_poly(coeffs, o.fr(0)))
    yi = [o.g1_mul(o.g1_gen(), xi) for xi in x]
    cts = []
    for c in range(n_cts):
        data = d.bytes(vlen)
        cts.append(o.tpke_encrypt(y, data, d.fr()))
    return x, y, yi, cts


def test_tpke_verify_batch_matches_oracle(nat):
    d = Drbg(b"gpu-tpke-verify")
    n, f = 4, 1
    x, y, yi, cts = _tpke_setup(d, n, f, 3)
    shares, expect = [], []
    for c, (U, V, W) in enumerate(cts):
        for i in range(n):
            ui = o.tpke_decrypt(U, V, W, x[i])
            shares.append((c, i, ui))
    # corruptions: wrong decryptor key, Ui + G, reversed bytes (HoneyBadgerMalicious.cs:23), infinity
    shares.append((0, 1, shares[0][2]))
    shares.append((1, 2, o.g1_add(shares[6][2], o.g1_gen())))
    shares.append((2, 3, bytes(reversed(shares[11][2]))))
    shares.append((2, 0, bytes(48)))
    for c, i, ui in shares:
        U, V, W = cts[c]
        r = o.tpke_verify_share(yi[i], U, V, W, ui)
        expect.append(r == 1)
    got = nat.tpke_verify_shares(yi, cts, shares)
    assert got == expect
    assert sum(expect) == 12


def test_tpke_verify_n22(nat):
    d = Drbg(b"gpu-tpke-n22")
    n, f = 22, 7
    x, y, yi, cts = _tpke_setup(d, n, f, 2)
    shares = []
    for c, (U, V, W) in enumerate(cts):
        for i in range(n):
            shares.append((c, i, o.tpke_decrypt(U, V, W, x[i])))
    bad = {3, 17, 30}
    for j in bad:
        c, i, ui = shares[j]
        shares[j] = (c, i, o.g1_add(ui, o.g1_gen()))
    got = nat.tpke_verify_shares(yi, cts, shares)
    assert got == [j not in bad for j in range(len(shares))]


def test_tpke_partial_decrypt_and_encrypt_match_oracle(nat):
    d = Drbg(b"gpu-tpke-dec")
    x, y, yi, cts = _tpke_setup(d, 4, 1, 4)
    bad_ct = (cts[3][0], cts[3][1], o.g2_mul(cts[3][2], o.fr(2)))
    res = nat.tpke_partial_decrypt(x[2], cts[:3] + [bad_ct])
    for (ok, ui), (U, V, W) in zip(res[:3], cts[:3]):
        assert ok and ui == o.tpke_decrypt(U, V, W, x[2])
    assert res[3][0] is False
    # encrypt with fixed r matches the oracle transcript byte for byte
    r = d.fr()
    data = b"lachain tpke plaintext"
    us, ts = nat.tpke_encrypt_phase1(y, [r])
    v = nat.xor_with_hash(ts[0], data)
    (w,) = nat.tpke_encrypt_phase2(us, [r], [v])
    assert (us[0], v, w) == o.tpke_encrypt(y, data, r)


def test_tpke_mirror_roundtrip(nat):
    # test/Lachain.CryptoTest/TPKETest.cs:23-58 through the Python mirror of the C# classes
    from lachain_amd import tpke
    kg = tpke.TrustedKeyGen(7, 2)
    pub = kg.GetPubKey()
    priv = [kg.GetPrivKey(i) for i in range(7)]
    share = tpke.RawShare(b"\x01\x02\x03\x04\x05", 132)
    enc = pub.Encrypt(share)
    parts = []
    for i in (0, 3):
        dec = priv[i].Decrypt(enc)
        assert kg.GetVerificationPubKey(i).VerifyShare(enc, dec)
        parts.append(dec)
    out = pub.FullDecrypt(enc, parts)
    assert out.Id == 132 and out.Data == share.Data


# ------------------------------------------------------------------ threshold signatures
def test_ts_batch_matches_oracle(nat):
    d = Drbg(b"gpu-ts")
    n, f = 7, 2
    coeffs = [d.fr() for _ in range(f + 1)]
    sk = [o.fr_eval_poly(coeffs, o.fr(i + 1)) for i in range(n)]
    pk = [o.g1_mul(o.g1_gen(), s) for s in sk]
    msgs = [(0xdeadbeef).to_bytes(4, "little"), bytes(24)]
    sigs = nat.ts_sign(sk + sk, msgs, [0] * n + [1] * n)
    for i in range(n):
        assert sigs[i] == o.ts_sign(sk[i], msgs[0])
    items = [(0, i, sigs[i]) for i in range(n)] + [(1, i, sigs[n + i]) for i in range(n)]
    items.append((0, 0, sigs[1]))        # signature of another signer
    items.append((1, 3, sigs[3]))        # signature over another message
    got = nat.ts_verify_shares(pk, msgs, items)
    assert got == [True] * (2 * n) + [False, False]
    # G2 Lagrange assembly (PublicKeySet.AssembleSignature) and shared key
    xs = [o.fr(i + 1) for i in range(f + 1)]
    comb = nat.lagrange_batch(2, [(xs, sigs[: f + 1])])[0]
    assert comb == o.g2_lagrange(xs, sigs[: f + 1])
    shared = nat.lagrange_batch(1, [([o.fr(i + 1) for i in range(n)], pk)])[0]
    assert shared == o.g1_lagrange([o.fr(i + 1) for i in range(n)], pk)
    assert nat.ts_verify_shares([shared], [msgs[0]], [(0, 0, comb)]) == [True]


def test_threshold_signer_mirror(nat):
    # test/Lachain.CryptoTest/ThresholdSignatureTest.cs:11-43 through the Python mirror
    from lachain_amd import threshold_signature as ts
    n, f = 7, 2
    kg = ts.TrustedKeyGen(n, f)
    shares = kg.GetPrivateShares()
    data = (0xdeadbeef).to_bytes(4, "little")
    pks = ts.PublicKeySet([s.GetPublicKeyShare() for s in shares], f)
    signers = [ts.ThresholdSigner(data, shares[i], pks) for i in range(n)]
    sig_shares = [s.Sign() for s in signers]
    signer = signers[0]
    result = None
    for j in range(n):
        ok, sig = signer.AddShare(j, sig_shares[j])
        assert ok
        result = result or sig
    assert result is not None and pks.SharedPublicKey.ValidateSignature(result, data)


# ------------------------------------------------------------------ Lagrange / MSM edge cases
def test_lagrange_batch_edge_cases(nat):
    G1 = o.g1_gen()
    d = Drbg(b"gpu-lagrange")
    poly = [d.fr() for _ in range(5)]
    xs = [o.fr(10 + i) for i in range(5)]
    ys = [o.g1_mul(G1, o.fr_eval_poly(poly, x)) for x in xs]
    problems = [
        (xs, ys),                               # ok
        ([], []),                               # k == 0 -> error
        ([o.fr(0)] + xs[1:], ys),               # zero x -> error
        ([xs[0], xs[0]] + xs[2:], ys),          # duplicate x -> error
        (xs[:1], ys[:1]),                       # k == 1 -> y0
    ]
    got = nat.lagrange_batch(1, problems)
    assert got[0] == o.g1_mul(G1, poly[0])
    assert got[1] is None and got[2] is None and got[3] is None
    assert got[4] == ys[0]


def test_msm_known_answer(nat):
    d = Drbg(b"gpu-msm")
    n = 257
    a = [d.fr_int() for _ in range(n)]
    s = [d.fr_int() for _ in range(n)]
    pts = nat.mul_batch(1, None, [o.fr(v) for v in a], generator=True)
    got = nat.g1_msm(pts, [o.fr(v) for v in s])
    expect = o.g1_mul(o.g1_gen(), o.fr(sum(x * y for x, y in zip(a, s))))
    assert got == expect


def test_decompression_validity_matches_oracle(mcl):
    """G1/G2.FromBytes accept exactly the encodings the oracle accepts: random x under a valid point's flag
    bits exercises the square-root (Fp exponentiation) path on residues and non-residues alike, plus x >= p."""
    d = Drbg(b"gpu-decompress")
    for P, size, gen, valid in ((mcl.G1, 48, o.g1_gen(), o.g1_valid), (mcl.G2, 96, o.g2_gen(), o.g2_valid)):
        encs = [gen, o.g1_mul(gen, d.fr()) if size == 48 else o.g2_mul(gen, d.fr())]
        for i in range(24):
            b = bytearray(d.bytes(size))
            b[47] = (b[47] & 0x1f) | (gen[47] & 0xe0)   # keep the flag bits of a valid encoding
            if size == 96:
                b[95] = (b[95] & 0x1f) | (gen[95] & 0xe0)
            if i == 0:
                b[47] |= 0x1f                             # x >= p
            encs.append(bytes(b))
        n_ok = 0
        for b in encs:
            want = valid(b)
            try:
                got = P.FromBytes(b)
                ok = True
            except ValueError:
                ok = False
            assert ok == want, (P.__name__, b.hex())
            if ok:
                n_ok += 1
                assert got.ToBytes() == b
        assert n_ok >= 2
