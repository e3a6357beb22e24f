"""CPU tests: the oracle (oracle/liborc.so, a C restatement of the MCL path) against the reference's
known-answer vectors, plus its internal self-consistency.  These pin the checker before it is trusted.
"""
import random

import oracle as o
import pytest

from helpers import Drbg, R, kats


def test_serialization_kats():
    # test/Lachain.CryptoTest/SerializationTest.cs:20-57
    k = kats()
    assert o.fr_from_int(0).hex() == k["fr_0"]["hex"]
    assert o.fr_from_int(1).hex() == k["fr_1"]["hex"]
    g1, g2 = o.g1_gen(), o.g2_gen()
    assert g1.hex() == k["g1_generator"]["hex"]
    assert o.g1_mul(g1, o.fr(2)).hex() == k["g1_generator_x2"]["hex"]
    assert o.g2_gen().hex() == k["g2_generator"]["hex"]
    assert o.g2_mul(g2, o.fr(2)).hex() == k["g2_generator_x2"]["hex"]
    assert o.g1_mul(g1, o.fr(0)).hex() == k["g1_zero"]["hex"]
    assert o.g2_mul(g2, o.fr(0)).hex() == k["g2_zero"]["hex"]
    # the doubling formulas agree with the addition formulas on the vectors
    assert o.g1_add(g1, g1).hex() == k["g1_generator_x2"]["hex"]
    assert o.g2_add(g2, g2).hex() == k["g2_generator_x2"]["hex"]


def test_kdf_kat():
    # test/Lachain.CryptoTest/CryptographyTest.cs:103-113 (BouncyCastle DigestRandomGenerator(Sha3Digest))
    k = kats()["kdf_deadbeef_32"]
    assert o.drg_bytes(bytes.fromhex(k["seed_hex"]), 32).hex() == k["hex"]


def test_config_keys_decode():
    # every G1 key in the reference's sample / network configs decodes, and re-serializes identically
    for e in kats()["g1_config_keys"]:
        b = bytes.fromhex(e["hex"])
        assert o.g1_valid(b), e["source"]
        assert o.g1_in_subgroup(b), e["source"]
        assert o.g1_add(b, o.g1_mul(o.g1_gen(), o.fr(0))) == b


def test_sha_vectors():
    import hashlib
    for m in [b"", b"abc", bytes(range(200))]:
        assert o.sha256(m) == hashlib.sha256(m).digest()
        assert o.sha512(m) == hashlib.sha512(m).digest()
        assert o.sha3_256(m) == hashlib.sha3_256(m).digest()


def test_pairing_bilinear_and_paths_agree():
    d = Drbg(b"oracle-bilinear")
    G1, G2 = o.g1_gen(), o.g2_gen()
    e = o.pairing(G1, G2)
    for _ in range(3):
        a, b = d.fr_int(), d.fr_int()
        A, B = o.g1_mul(G1, o.fr(a)), o.g2_mul(G2, o.fr(b))
        eab = o.pairing(A, B)
        assert eab == o.gt_pow(e, o.fr(a * b))            # MclTests.cs:64-75
        assert eab == o.pairing_slow(A, B)                 # affine Miller loop + direct exponent
        f = o.miller_loop(A, B)
        assert o.final_exp(f) == o.final_exp_direct(f)     # addition chain == 3(p^4-p^2+1)/r power
    assert e != o.pairing(G1, o.g2_mul(G2, o.fr(0)))


def test_cyclotomic_and_sparse_helpers():
    import ctypes
    d = Drbg(b"oracle-helpers")
    A = o.g1_mul(o.g1_gen(), d.fr())
    B = o.g2_mul(o.g2_gen(), d.fr())
    f = o.miller_loop(A, B)
    out = ctypes.create_string_buffer(576)
    assert o.lib().orc_test_cyc_sqr(out, f) == 0
    rnd = random.Random(5)
    abc = b"".join(rnd.randrange(o.P).to_bytes(48, "little") for _ in range(6))
    assert o.lib().orc_test_sparse_line(f, abc) == 0


def test_hash_to_g2_properties():
    for m in [b"", b"\x00", b"lachain", bytes(range(100))]:
        h = o.g2_hash(m)
        assert o.g2_valid(h) and o.g2_in_subgroup(h)
    o.set_g2_original_cofactor(1)
    try:
        h2 = o.g2_hash(b"lachain")
        assert o.g2_in_subgroup(h2)
    finally:
        o.set_g2_original_cofactor(0)


def test_lagrange_and_poly():
    # MclTests.cs:90-118: evaluate a degree-9 polynomial at 100..110, interpolate the intercept
    d = Drbg(b"oracle-poly")
    poly = [d.fr() for _ in range(10)]
    xs = [o.fr(100 + i) for i in range(11)]
    ys = [o.fr_eval_poly(poly, x) for x in xs]
    assert o.fr_lagrange(xs, ys) == poly[0]
    # group versions: ys_i = poly(x_i) * G
    G1, G2 = o.g1_gen(), o.g2_gen()
    assert o.g1_lagrange(xs, [o.g1_mul(G1, y) for y in ys]) == o.g1_mul(G1, poly[0])
    assert o.g2_lagrange(xs[:5], [o.g2_mul(G2, y) for y in ys[:5]]) != o.g2_mul(G2, poly[0])
    # error cases: k == 0, zero x, duplicate x
    assert o.g1_lagrange([], []) is None
    assert o.g1_lagrange([o.fr(0), o.fr(1)], [G1, G1]) is None
    assert o.g1_lagrange([o.fr(3), o.fr(3)], [G1, G1]) is None


def test_tpke_roundtrip():
    # test/Lachain.CryptoTest/TPKETest.cs:23-58 with N=7, F=2, Id=132
    d = Drbg(b"oracle-tpke")
    n, f = 7, 2
    coeffs = [d.fr() for _ in range(f)]  # TPKE TrustedKeyGen: f coefficients
    x = [o.fr_eval_poly(coeffs, o.fr(i + 1)) for i in range(n)]
    y = o.g1_mul(o.g1_gen(), o.fr_eval_poly(coeffs, o.fr(0)))
    yi = [o.g1_mul(o.g1_gen(), xi) for xi in x]
    data = bytes(range(1, 10))
    U, V, W = o.tpke_encrypt(y, data, d.fr())
    parts = []
    for i in (1, 4):
        ui = o.tpke_decrypt(U, V, W, x[i])
        assert o.tpke_verify_share(yi[i], U, V, W, ui) == 1
        assert o.tpke_verify_share(yi[(i + 1) % n], U, V, W, ui) == 0
        parts.append((i, ui))
    assert o.tpke_full_decrypt(V, [i for i, _ in parts], [u for _, u in parts]) == data
    with pytest.raises(ValueError):
        o.tpke_decrypt(U, V, o.g2_mul(W, o.fr(2)), x[0])   # ciphertext validity check


def test_threshold_signature_roundtrip():
    # test/Lachain.CryptoTest/ThresholdSignatureTest.cs:11-43, n=7, f=2, msg = 0xdeadbeef LE
    d = Drbg(b"oracle-ts")
    n, f = 7, 2
    coeffs = [d.fr() for _ in range(f + 1)]
    sk = [o.fr_eval_poly(coeffs, o.fr(i + 1)) for i in range(n)]
    pk = [o.g1_mul(o.g1_gen(), s) for s in sk]
    msg = (0xdeadbeef).to_bytes(4, "little")
    sigs = [o.ts_sign(s, msg) for s in sk]
    for i in range(n):
        assert o.ts_validate(pk[i], sigs[i], msg) == 1
    assert o.ts_validate(pk[0], sigs[1], msg) == 0
    xs = [o.fr(i + 1) for i in range(f + 1)]
    combined = o.g2_lagrange(xs, sigs[: f + 1])
    shared_pk = o.g1_lagrange([o.fr(i + 1) for i in range(n)], pk)
    assert shared_pk == o.g1_mul(o.g1_gen(), coeffs[0])
    assert o.ts_validate(shared_pk, combined, msg) == 1
    assert combined == o.g2_lagrange([o.fr(i + 1) for i in range(2, 5)], sigs[2:5])


def test_malformed_encodings_rejected():
    g1 = bytearray(o.g1_gen())
    bad = bytearray(g1)
    bad[47] |= 0x60                      # x >= 2^381 > p
    assert not o.g1_valid(bytes(bad))
    # reversed bytes (HoneyBadgerMalicious.cs:23) are either rejected or a different point
    rev = bytes(reversed(g1))
    assert (not o.g1_valid(rev)) or rev != bytes(g1)
    # an x with no square root of x^3 + 4 is rejected
    x = 5
    while True:
        cand = x.to_bytes(48, "little")
        if not o.g1_valid(cand):
            break
        x += 1
    assert not o.g1_valid(cand)


def test_ts_validate_batch_matches_single():
    """orc_ts_validate_batch (the CommonCoin CPU baseline) decides like orc_ts_validate share by share."""
    import ctypes
    import numpy as np
    msgs = [b"coin-%d" % r for r in range(2)]
    sks = [o.fr(7), o.fr(9), o.fr(13)]
    pks = b"".join(o.g1_mul(o.g1_gen(), s) for s in sks)
    sigs = [o.ts_sign(sks[i], msgs[r]) for r in range(2) for i in range(3)]
    sigs[4] = sigs[3]                                   # round 1, share 1 carries share 0's signature
    moff = np.array([0, len(msgs[0]), len(msgs[0]) + len(msgs[1])], dtype=np.uint32)
    midx = np.array([0, 0, 0, 1, 1, 1], dtype=np.uint32)
    pidx = np.array([0, 1, 2, 0, 1, 2], dtype=np.uint32)
    acc = ctypes.create_string_buffer(6)
    assert o.lib().orc_ts_validate_batch(acc, ctypes.c_size_t(6), pks, b"".join(sigs), b"".join(msgs),
                                         moff.ctypes.data_as(ctypes.c_void_p), midx.ctypes.data_as(ctypes.c_void_p),
                                         pidx.ctypes.data_as(ctypes.c_void_p), 2) == 0
    single = [o.ts_validate(pks[48 * pidx[i]:48 * pidx[i] + 48], sigs[i], msgs[midx[i]]) == 1 for i in range(6)]
    assert [b == 1 for b in acc.raw] == single == [True, True, True, True, False, True]


def test_amortized_cpu_baselines_match_as_reference():
    """bench.py's amortized CPU legs (per-ciphertext H and Miller lines, one final exponentiation per share) decide
    exactly like the as-reference path (hash + two pairings + Equals per call, TPKE/PublicKey.cs:88-92,
    ThresholdSignature/PublicKey.cs:16-21), including malformed, wrong-key and infinity shares."""
    import ctypes
    import numpy as np
    from helpers import Drbg, R
    lib = o.lib()
    d = Drbg(b"oracle-amortized")
    n, f = 4, 1
    coeffs = [d.fr_int() for _ in range(f + 1)]
    poly = lambda x: sum(c * pow(x, i, R) for i, c in enumerate(coeffs)) % R
    xs = [poly(i + 1) for i in range(n)]
    yi = [o.g1_mul(o.g1_gen(), o.fr(x)) for x in xs]
    y = o.g1_mul(o.g1_gen(), o.fr(poly(0)))
    cts = [o.tpke_encrypt(y, d.bytes(32), o.fr(d.fr_int())) for _ in range(3)]
    shares = [o.g1_mul(cts[c][0], o.fr(xs[j])) for c in range(3) for j in range(n)]
    shares[1] = o.g1_add(shares[1], o.g1_gen())
    shares[5] = bytes(48)                   # infinity
    shares[6] = shares[6][::-1]             # reversed bytes (HoneyBadgerMalicious.cs:23)
    shares[9] = shares[10]                  # another decryptor's share
    m = len(shares)
    ct = np.repeat(np.arange(3, dtype=np.uint32), n)
    dec = np.tile(np.arange(n, dtype=np.uint32), 3)
    u = b"".join(c[0] for c in cts); v = b"".join(c[1] for c in cts); w = b"".join(c[2] for c in cts)
    a1 = ctypes.create_string_buffer(m); a2 = ctypes.create_string_buffer(m)
    p = lambda arr: arr.ctypes.data_as(ctypes.c_void_p)
    assert lib.orc_tpke_verify_batch(a1, ctypes.c_size_t(m), b"".join(yi), u, v, ctypes.c_size_t(32), w, p(ct), p(dec),
                                     b"".join(shares), 2) in (0, -1)
    assert lib.orc_tpke_verify_batch_amortized(a2, ctypes.c_size_t(m), b"".join(yi), ctypes.c_size_t(n), u, v,
                                               ctypes.c_size_t(32), w, ctypes.c_size_t(3), p(ct), p(dec),
                                               b"".join(shares), 2) == 0
    assert a1.raw == a2.raw and sum(a1.raw) == m - 4
    # threshold signatures
    sks = [d.fr_int() for _ in range(3)]
    pks = [o.g1_mul(o.g1_gen(), o.fr(s)) for s in sks]
    msgs = [b"coin a", b"coin bb"]
    sigs = [o.ts_sign(o.fr(sks[k]), msgs[mi]) for mi in range(2) for k in range(3)]
    sigs[1] = sigs[2]
    sigs[4] = bytes(96)
    mo = np.array([0, 6, 13], dtype=np.uint32)
    mi = np.repeat(np.arange(2, dtype=np.uint32), 3)
    pi = np.tile(np.arange(3, dtype=np.uint32), 2)
    b1 = ctypes.create_string_buffer(6); b2 = ctypes.create_string_buffer(6)
    lib.orc_ts_validate_batch(b1, ctypes.c_size_t(6), b"".join(pks), b"".join(sigs), b"".join(msgs), p(mo), p(mi),
                              p(pi), 2)
    assert lib.orc_ts_validate_batch_amortized(b2, ctypes.c_size_t(6), b"".join(pks), ctypes.c_size_t(3),
                                               b"".join(sigs), b"".join(msgs), p(mo), ctypes.c_size_t(2), p(mi), p(pi),
                                               2) == 0
    assert b1.raw == b2.raw and sum(b1.raw) == 4


def test_rlc_cpu_baseline_matches_transcripts():
    """bench.py's randomized-batch CPU leg (orc_tpke_verify_batch_rlc: the GPU's k_batch.hip algorithm on the host)
    reproduces every decision of the committed TPKE transcripts (wrong-player, reversed, off-subgroup and infinity
    shares), tiled 1x and 3x, under two exponent seeds"""
    import ctypes
    import json
    import os
    import numpy as np
    from helpers import GOLDEN
    lib = o.lib()
    T = json.load(open(os.path.join(GOLDEN, "transcripts.json")))
    p = lambda arr: arr.ctypes.data_as(ctypes.c_void_p)
    H = bytes.fromhex
    for key in ("tpke_n4", "tpke_n22"):
        t = T[key]
        cs = t["ciphertexts"]
        n = len(t["y_i"])
        assert all(len(H(c["v"])) == len(H(cs[0]["v"])) for c in cs)
        shares = [H(s) for c in cs for s in c["shares"]]
        for rep in (1, 3):                      # a 3-fold tiling puts several runs of one ciphertext in a row
            sh = shares * rep
            m = len(sh)
            ct = np.tile(np.repeat(np.arange(len(cs), dtype=np.uint32), n), rep)
            dec = np.tile(np.arange(n, dtype=np.uint32), len(cs) * rep)
            expect = bytes([a for c in cs for a in c["accept"]] * rep)
            for seed in (1, 0xDEADBEEF):
                acc = ctypes.create_string_buffer(m)
                assert lib.orc_tpke_verify_batch_rlc(
                    acc, ctypes.c_size_t(m), b"".join(H(y) for y in t["y_i"]), ctypes.c_size_t(n),
                    b"".join(H(c["u"]) for c in cs), b"".join(H(c["v"]) for c in cs), ctypes.c_size_t(len(H(cs[0]["v"]))),
                    b"".join(H(c["w"]) for c in cs), ctypes.c_size_t(len(cs)), p(ct), p(dec), b"".join(sh),
                    ctypes.c_uint64(seed), 2) == 0
                assert acc.raw == expect, (key, rep, seed)


def test_rlc_cpu_ts_baseline_and_psi_membership():
    """the batched threshold-signature CPU leg (orc_ts_validate_batch_rlc) reproduces the N=7 / N=100 transcripts
    (wrong-signer, reversed, off-subgroup, infinity shares), and the psi membership test it shares with the GPU
    (psi(P) == [z] P) agrees with the definition ([r] P == O) on in- and off-subgroup points"""
    import ctypes
    import json
    import os
    import numpy as np
    from helpers import GOLDEN, Drbg
    lib = o.lib()
    d = Drbg(b"oracle-psi-membership")
    for k in range(6):
        if k % 2:
            p = o.g2_mul(o.g2_gen(), o.fr(d.fr_int()))
        else:
            while True:
                xa = int.from_bytes(d.bytes(48), "little") % o.P
                xb = int.from_bytes(d.bytes(48), "little") % o.P
                enc = bytearray(xa.to_bytes(48, "little") + xb.to_bytes(48, "little"))
                enc[95] |= 0x80 * (d.bytes(1)[0] & 1)
                p = bytes(enc)
                if o.g2_valid(p):
                    break
        assert lib.orc_g2_in_subgroup_psi(p) == o.g2_in_subgroup(p) == (k % 2 == 1)
    T = json.load(open(os.path.join(GOLDEN, "transcripts.json")))
    pp = lambda arr: arr.ctypes.data_as(ctypes.c_void_p)
    H = bytes.fromhex
    for key in ("ts_n7", "ts_n100"):
        t = T[key]
        rs = t["rounds"]
        n = len(t["pk_i"])
        msgs = [H(r["msg"]) for r in rs]
        mo = np.cumsum([0] + [len(m) for m in msgs]).astype(np.uint32)
        sigs = b"".join(H(s) for r in rs for s in r["sigs"])
        m = len(rs) * n
        mi = np.repeat(np.arange(len(rs), dtype=np.uint32), n)
        pi = np.tile(np.arange(n, dtype=np.uint32), len(rs))
        acc = ctypes.create_string_buffer(m)
        assert lib.orc_ts_validate_batch_rlc(acc, ctypes.c_size_t(m), b"".join(H(x) for x in t["pk_i"]),
                                             ctypes.c_size_t(n), sigs, b"".join(msgs), pp(mo),
                                             ctypes.c_size_t(len(rs)), pp(mi), pp(pi), ctypes.c_uint64(7), 2) == 0
        assert acc.raw == bytes(a for r in rs for a in r["accept"]), key


def test_cpu_pippenger_msm_matches_plain_msm():
    """bench.py's MSM CPU leg (orc_g1_msm_pippenger: signed-digit bucket method over pre-decompressed points) equals the
    plain sum of scalar multiplications (orc_g1_msm), with infinity, repeated and negated points, scalars 0, 1, r - 1
    and every window width the bench may pick"""
    import ctypes
    lib = o.lib()
    d = Drbg(b"cpu-pippenger")
    g = o.g1_gen()
    base = [o.g1_mul(g, o.fr(d.fr_int())) for _ in range(40)]
    pts = base + [base[0], o.g1_neg(base[1]), o.g1_mul(g, o.fr(0)), base[2]]
    scal = [d.fr_int() for _ in range(40)] + [0, 1, R - 1, 12345]
    pts, scal = pts * 3, scal * 3
    n = len(pts)
    pb = b"".join(pts)
    sb = b"".join(s.to_bytes(32, "little") for s in scal)
    want = ctypes.create_string_buffer(48)
    assert lib.orc_g1_msm(want, pb, sb, ctypes.c_size_t(n)) == 0
    lib.orc_g1_affine_bytes.restype = ctypes.c_size_t
    aff = ctypes.create_string_buffer(lib.orc_g1_affine_bytes() * n)
    assert lib.orc_g1_affine_batch(aff, pb, ctypes.c_size_t(n), 4) == 0
    for c in (2, 5, 8, 13, 16):
        got = ctypes.create_string_buffer(48)
        assert lib.orc_g1_msm_pippenger(got, aff, sb, ctypes.c_size_t(n), c, 4) == 0
        assert got.raw == want.raw, c
