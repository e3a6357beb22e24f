"""CPU tests of the secp256k1 ECDSA oracle (oracle/secp.c) against the reference's known answers
(tests/golden/secp256k1_kats.json from test/Lachain.CryptoTest/CryptographyTest.cs) and the libsecp256k1 rules
DefaultCrypto.VerifySignatureHashed (src/Lachain.Crypto/DefaultCrypto.cs:79-101) inherits."""
import json
import os
import random

import pytest

import oracle as o

HERE = os.path.dirname(os.path.abspath(__file__))
K = json.load(open(os.path.join(HERE, "golden", "secp256k1_kats.json")))
PRIV = bytes.fromhex(K["priv_address"]["priv"])


def test_keccak_and_header_kats():
    kk = K["keccak256"]
    assert o.keccak256(kk["msg_ascii"].encode()).hex() == kk["hex"]
    h = K["header_keccak"]
    got = o.header_keccak(bytes.fromhex(h["prev"]), bytes.fromhex(h["state"]), bytes.fromhex(h["merkle"]), h["index"],
                          h["nonce"])
    assert got.hex() == h["hex"]


def test_private_key_to_address():
    c33, c65 = o.ecdsa_pubkey(PRIV)
    assert o.keccak256(c65[1:])[12:].hex() == K["priv_address"]["address"].lower()
    assert c33[1:] == c65[1:33] and c33[0] == 2 + (c65[64] & 1)


@pytest.mark.parametrize("i", range(4))
def test_reference_signatures_verify(i):
    s = K["signatures"][i]
    c33, c65 = o.ecdsa_pubkey(PRIV)
    h = o.keccak256(bytes.fromhex(s["msg_rlp"]))
    sig = bytes.fromhex(s["sig"])
    new, chain = s["use_new_chain_id"], s["chain_id"]
    assert o.ecdsa_verify_hashed(h, sig, c33, new, chain)
    assert o.ecdsa_verify_hashed(h, sig, c65, new, chain)
    if "full_hash" in s:
        assert o.keccak256(bytes.fromhex(s["signed_rlp"])).hex() == s["full_hash"]
    # recover-to-address (Test_External_Signature's assertion) with the reference's recId arithmetic
    enc = sig[64] * 256 + sig[65] if new else sig[64]
    rec = _csdiv(_csdiv(enc - 36, 2), chain)
    pk = o.ecdsa_recover(h, sig[:64], rec)
    assert pk == c33
    # wrong flag / chain id / hash
    assert not o.ecdsa_verify_hashed(h, sig, c33, not new, chain)
    assert not o.ecdsa_verify_hashed(h, sig, c33, new, 0)
    assert not o.ecdsa_verify_hashed(bytes([h[0] ^ 1]) + h[1:], sig, c33, new, chain)


def _csdiv(a, b):
    """C# int division (truncation toward zero)"""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b > 0) else -q


def _sig(rng, h, priv, chain, new):
    while True:
        k = rng.randrange(1, o.SECP_N).to_bytes(32, "big")
        try:
            c, rid = o.ecdsa_sign_compact(h, priv, k)
            return o.ecdsa_encode(c, rid, chain, new)
        except ValueError:
            continue


def test_recid_arithmetic_matches_csharp():
    rng = random.Random(3)
    for _ in range(2000):
        chain = rng.choice([1, 2, 25, 225, 1000, -7, 0])
        new = rng.random() < 0.5
        tail = rng.randrange(0, 65536 if new else 256)
        sig = bytes(64) + (tail.to_bytes(2, "big") if new else bytes([tail]))
        lib = o.lib()
        got = lib.orc_ecdsa_recid_ok(sig, len(sig), chain)
        if chain == 0:
            want = False
        else:
            r = _csdiv(_csdiv(tail - 36, 2), chain)
            want = 0 <= r <= 3
        assert bool(got) == want, (chain, new, tail)


def test_round_trip_and_rejections():
    rng = random.Random(7)
    n = o.SECP_N
    for it in range(40):
        priv = rng.randrange(1, n).to_bytes(32, "big")
        c33, c65 = o.ecdsa_pubkey(priv)
        h = rng.randbytes(32) if it else b"\xff" * 32           # a hash >= n is reduced mod n
        chain, new = rng.choice([(25, False), (225, True), (1, False)])
        sig = _sig(rng, h, priv, chain, new)
        assert o.ecdsa_verify_hashed(h, sig, c33, new, chain)
        r = int.from_bytes(sig[:32], "big")
        s = int.from_bytes(sig[32:64], "big")
        tail = sig[64:]
        assert s <= n // 2
        hi = sig[:32] + (n - s).to_bytes(32, "big") + tail                   # high-s twin: rejected
        assert not o.ecdsa_verify_hashed(h, hi, c33, new, chain)
        assert not o.ecdsa_verify_hashed(h, bytes(32) + sig[32:], c33, new, chain)      # r = 0
        assert not o.ecdsa_verify_hashed(h, sig[:32] + bytes(32) + tail, c33, new, chain)  # s = 0
        if r + n < 2 ** 256:                                                     # r >= n: parse overflow
            assert not o.ecdsa_verify_hashed(h, (r + n).to_bytes(32, "big") + sig[32:], c33, new, chain)
        other = o.ecdsa_pubkey(rng.randrange(1, n).to_bytes(32, "big"))[0]
        assert not o.ecdsa_verify_hashed(h, sig, other, new, chain)
        assert not o.ecdsa_verify_hashed(h, sig[:-1], c33, new, chain)
        # hybrid encodings (0x06 / 0x07) parse when the tag matches y's parity
        odd = c65[64] & 1
        assert o.ecdsa_verify_hashed(h, sig, bytes([6 + odd]) + c65[1:], new, chain)
        assert not o.ecdsa_verify_hashed(h, sig, bytes([7 - odd]) + c65[1:], new, chain)
        assert not o.ecdsa_verify_hashed(h, sig, bytes([5]) + c65[1:], new, chain)
        assert not o.ecdsa_verify_hashed(h, sig, c65[:64] + bytes([c65[64] ^ 1]), new, chain)  # off the curve
        assert not o.ecdsa_verify_hashed(h, sig, bytes([c33[0] ^ 1]) + c33[1:], new, chain)    # other y


def test_bad_keys():
    rng = random.Random(9)
    priv = rng.randrange(1, o.SECP_N).to_bytes(32, "big")
    h = rng.randbytes(32)
    sig = _sig(rng, h, priv, 25, False)
    p = o.SECP_P
    assert not o.ecdsa_verify_hashed(h, sig, b"\x02" + p.to_bytes(32, "big"), False, 25)          # x = p
    # x with no point: find one
    x = 5
    while o.ecdsa_recover(h, x.to_bytes(32, "big") + sig[32:64], 0) is not None:
        x += 1
    assert not o.ecdsa_verify_hashed(h, sig, b"\x02" + x.to_bytes(32, "big"), False, 25)
    assert not o.ecdsa_verify_hashed(h, sig, b"\x04" + bytes(64), False, 25)
    assert not o.ecdsa_verify_hashed(h, sig, bytes(33), False, 25)


def test_x_of_R_at_least_n_branch():
    """x(R) in [n, p): r = x(R) - n; verified through the (r + n) Z^2 comparison (recovery id bit 1)"""
    rng = random.Random(11)
    found = 0
    while found < 3:
        r = rng.randrange(1, o.SECP_P - o.SECP_N)
        s = rng.randrange(1, o.SECP_N // 2)
        h = rng.randbytes(32)
        sig64 = r.to_bytes(32, "big") + s.to_bytes(32, "big")
        pk = o.ecdsa_recover(h, sig64, 2)
        if pk is None:
            continue
        found += 1
        sig = o.ecdsa_encode(sig64, 2, 25, False)
        assert o.ecdsa_verify_hashed(h, sig, pk, False, 25)
        other = o.ecdsa_recover(h, sig64, 0)      # R' with x = r (if it exists) gives a different key
        if other is not None:
            assert other != pk and o.ecdsa_verify_hashed(h, sig, other, False, 25)


def test_batch_matches_single():
    rng = random.Random(13)
    keys = [rng.randrange(1, o.SECP_N).to_bytes(32, "big") for _ in range(5)]
    pks = b"".join(o.ecdsa_pubkey(k)[0] for k in keys)
    hs, ss, idx, want = [], [], [], []
    for i in range(60):
        j = rng.randrange(5)
        h = rng.randbytes(32)
        sig = _sig(rng, h, keys[j], 225, True)
        if i % 7 == 3:
            j = (j + 1) % 5
        hs.append(h); ss.append(sig); idx.append(j if i != 11 else 99)
        want.append(i % 7 != 3 and i != 11)
    got = o.ecdsa_verify_batch(b"".join(hs), b"".join(ss), 66, pks, 33, idx, 60, True, 225)
    assert [bool(b) for b in got] == want


# ---------------------------------------------------------------- independent pure-Python restatement (affine, pow)
_P, _N = o.SECP_P, o.SECP_N
_G = (0x79BE667EF9DCBBAC55A06295CE870B07029BFCDB2DCE28D959F2815B16F81798,
      0x483ADA7726A3C4655DA4FBFC0E1108A8FD17B448A68554199C47D08FFB10D4B8)


def _add(a, b):
    if a is None:
        return b
    if b is None:
        return a
    if a[0] == b[0]:
        if (a[1] + b[1]) % _P == 0:
            return None
        lam = 3 * a[0] * a[0] * pow(2 * a[1], -1, _P) % _P
    else:
        lam = (b[1] - a[1]) * pow(b[0] - a[0], -1, _P) % _P
    x = (lam * lam - a[0] - b[0]) % _P
    return x, (lam * (a[0] - x) - a[1]) % _P


def _mul(k, a):
    r = None
    while k:
        if k & 1:
            r = _add(r, a)
        a = _add(a, a)
        k >>= 1
    return r


def _py_verify(h, sig64, pk33):
    x = int.from_bytes(pk33[1:], "big")
    if pk33[0] not in (2, 3) or x >= _P:
        return False
    y = pow((x ** 3 + 7) % _P, (_P + 1) // 4, _P)
    if y * y % _P != (x ** 3 + 7) % _P:
        return False
    if y & 1 != pk33[0] & 1:
        y = _P - y
    r, s = int.from_bytes(sig64[:32], "big"), int.from_bytes(sig64[32:], "big")
    if not (0 < r < _N and 0 < s <= _N // 2):
        return False
    z = int.from_bytes(h, "big") % _N
    w = pow(s, -1, _N)
    R = _add(_mul(z * w % _N, _G), _mul(r * w % _N, (x, y)))
    return R is not None and R[0] % _N == r


def test_generator_on_curve():
    assert (_G[1] ** 2 - _G[0] ** 3 - 7) % _P == 0 and _mul(_N, _G) is None


def test_python_restatement_cross_check():
    rng = random.Random(17)
    for i in range(24):
        priv = rng.randrange(1, _N)
        c33 = o.ecdsa_pubkey(priv.to_bytes(32, "big"))[0]
        P = _mul(priv, _G)
        assert c33 == bytes([2 + (P[1] & 1)]) + P[0].to_bytes(32, "big")
        h = rng.randbytes(32)
        sig = _sig(rng, h, priv.to_bytes(32, "big"), 25, False)
        if i % 3 == 1:
            sig = sig[:5] + bytes([sig[5] ^ 0x10]) + sig[6:]
        if i % 3 == 2:
            h = rng.randbytes(32)
        assert _py_verify(h, sig[:64], c33) == o.ecdsa_verify_hashed(h, sig, c33, False, 25) == (i % 3 == 0)
