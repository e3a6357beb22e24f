#!/usr/bin/env python3
"""tests/golden/make_transcripts.py — writes tests/golden/transcripts.json: fixed-seed TPKE and threshold-signature
transcripts made by the C oracle and cross-checked, item by item where affordable, by the independent
pure-Python restatement tests/pyref/bls12_381.py.  Needs no /root/reference (the protocol rules are restated in the
oracle, with the reference lines cited there); rerun with `python tests/golden/make_transcripts.py`.

TPKE (src/Lachain.Crypto/TPKE/*.cs): N = 4, F = 1 and N = 22, F = 7; keys from a degree-F polynomial (x_i = f(i + 1),
Y = f(0) G1, Y_i = x_i G1); two ciphertexts of 32-byte payloads; every player's decryption share, with malicious ones
as the reference's tests make them:
  * "reversed": the share's 48 bytes reversed (test/Lachain.ConsensusTest/HoneyBadgerMalicious.cs:23);
  * "random_g1": random bytes that decode as a G1 point, almost surely off the r-subgroup
    (HoneyBadgerSmartMalicious.cs:28-48);
  * "other_player": a valid share of another player; "infinity": 48 zero bytes.
Expected per-share decisions (VerifyShare), and FullDecrypt of the first F + 1 valid shares (PublicKey.cs:59-80).
Threshold signatures (ThresholdSigner / PublicKeySet): N = 7, F = 2 and N = 100, F = 33 over CommonCoin messages
(CoinId bytes), shares x_i H(m) with the same kinds of malicious shares in G2; expected ValidateSignature decisions
and the signature assembled from the first F + 1 valid shares, which equals x H(m).
"""
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import oracle as o                       # noqa: E402
from pyref import bls12_381 as B         # noqa: E402

R = o.R


def coin_id(era, agreement, epoch):
    m64 = (1 << 64) - 1                  # CoinId.ToBytes(): int64 LE each (CoinId.cs:21-24)
    return b"".join((v & m64).to_bytes(8, "little") for v in (era, agreement, epoch))


def random_valid(rng, size, valid):
    while True:
        b = bytes(rng.getrandbits(8) for _ in range(size))
        if valid(b):
            return b


def keys(rng, n, f):
    coeffs = [rng.randrange(R) for _ in range(f + 1)]
    poly = lambda x: sum(c * pow(x, i, R) for i, c in enumerate(coeffs)) % R
    return [poly(i + 1) for i in range(n)], poly(0)


def tpke(rng, n, f, n_ct, bad):
    xs, x = keys(rng, n, f)
    g = o.g1_gen()
    y = o.g1_mul(g, o.fr(x))
    ys = [o.g1_mul(g, o.fr(xi)) for xi in xs]
    cts = []
    for c in range(n_ct):
        data = bytes(rng.getrandbits(8) for _ in range(32))
        u, v, w = o.tpke_encrypt(y, data, o.fr(rng.randrange(1, R)))
        shares, kinds = [], []
        for i in range(n):
            s = o.tpke_decrypt(u, v, w, o.fr(xs[i]))
            kind = bad.get((c, i), "honest")
            if kind == "reversed":
                s = s[::-1]
            elif kind == "random_g1":
                s = random_valid(rng, 48, o.g1_valid)
            elif kind == "other_player":
                s = o.tpke_decrypt(u, v, w, o.fr(xs[(i + 1) % n]))
            elif kind == "infinity":
                s = bytes(48)
            shares.append(s)
            kinds.append(kind)
        accept = [o.tpke_verify_share(ys[i], u, v, w, shares[i]) == 1 for i in range(n)]
        assert accept == [k == "honest" for k in kinds], (accept, kinds)
        ids = [i for i in range(n) if accept[i]][: f + 1]
        plain = o.tpke_full_decrypt(v, ids, [shares[i] for i in ids])
        assert plain == data
        cts.append(dict(u=u.hex(), v=v.hex(), w=w.hex(), data=data.hex(), shares=[s.hex() for s in shares],
                        kinds=kinds, accept=accept, combine_ids=ids, plaintext=plain.hex()))
    return dict(n=n, f=f, y=y.hex(), y_i=[b.hex() for b in ys], x_i=[o.fr(v).hex() for v in xs], ciphertexts=cts)


def ts(rng, n, f, msgs, bad):
    xs, x = keys(rng, n, f)
    g = o.g1_gen()
    pks = [o.g1_mul(g, o.fr(xi)) for xi in xs]
    pk = o.g1_mul(g, o.fr(x))
    rounds = []
    for c, m in enumerate(msgs):
        sigs, kinds = [], []
        for i in range(n):
            s = o.ts_sign(o.fr(xs[i]), m)
            kind = bad.get((c, i), "honest")
            if kind == "reversed":
                s = s[::-1]
            elif kind == "random_g2":
                s = random_valid(rng, 96, o.g2_valid)
            elif kind == "other_player":
                s = o.ts_sign(o.fr(xs[(i + 1) % n]), m)
            elif kind == "infinity":
                s = bytes(96)
            sigs.append(s)
            kinds.append(kind)
        accept = [o.ts_validate(pks[i], sigs[i], m) == 1 for i in range(n)]
        assert accept == [k == "honest" for k in kinds], (accept, kinds)
        ids = [i for i in range(n) if accept[i]][: f + 1]
        combined = o.g2_lagrange([o.fr(i + 1) for i in ids], [sigs[i] for i in ids])
        assert combined == o.ts_sign(o.fr(x), m)
        rounds.append(dict(msg=m.hex(), h=o.g2_hash(m).hex(), sigs=[s.hex() for s in sigs], kinds=kinds,
                           accept=accept, assemble_ids=ids, combined=combined.hex()))
    return dict(n=n, f=f, pk=pk.hex(), pk_i=[b.hex() for b in pks], x_i=[o.fr(v).hex() for v in xs], rounds=rounds)


def pyref_check(t):
    """independent re-derivation of a sample: hash-to-G2, shares x_i H, pairing decisions, Lagrange combination"""
    a = t["tpke_n4"]["ciphertexts"][0]
    u, v, w = (bytes.fromhex(a[k]) for k in ("u", "v", "w"))
    h = B.hash_to_g2(u + v)
    assert B.g2_to_bytes(h) == o.g2_hash(u + v)
    for i in range(4):
        s = bytes.fromhex(a["shares"][i])
        try:
            ui = B.g1_from_bytes(s)
        except ValueError:
            ok = False
        else:
            ok = B.pairing_check(ui, h, B.g1_from_bytes(bytes.fromhex(t["tpke_n4"]["y_i"][i])), B.g2_from_bytes(w))
        assert ok == a["accept"][i], i
    ids = a["combine_ids"]
    lam = B.lagrange_coeffs([i + 1 for i in ids])
    acc = None
    for li, i in zip(lam, ids):
        acc = B.g1_add(acc, B.g1_mul(B.g1_from_bytes(bytes.fromhex(a["shares"][i])), li))
    assert B.g1_to_bytes(acc) == o.g1_lagrange([o.fr(i + 1) for i in ids], [bytes.fromhex(a["shares"][i]) for i in ids])
    r = t["ts_n7"]["rounds"][0]
    m = bytes.fromhex(r["msg"])
    h = B.hash_to_g2(m)
    assert B.g2_to_bytes(h).hex() == r["h"]
    xs = [int.from_bytes(bytes.fromhex(x), "little") for x in t["ts_n7"]["x_i"]]
    for i in range(7):
        if r["kinds"][i] == "honest":
            assert B.g2_to_bytes(B.g2_mul(h, xs[i])).hex() == r["sigs"][i]
    for i in (0, 1, 2):
        s = bytes.fromhex(r["sigs"][i])
        try:
            sg = B.g2_from_bytes(s)
        except ValueError:
            ok = False
        else:
            g1 = B.g1_from_bytes(o.g1_gen())
            ok = B.pairing_check(B.g1_from_bytes(bytes.fromhex(t["ts_n7"]["pk_i"][i])), h, g1, sg)
        assert ok == r["accept"][i], i
    ids = r["assemble_ids"]
    lam = B.lagrange_coeffs([i + 1 for i in ids])
    acc = None
    for li, i in zip(lam, ids):
        acc = B.g2_add(acc, B.g2_mul(B.g2_from_bytes(bytes.fromhex(r["sigs"][i])), li))
    assert B.g2_to_bytes(acc).hex() == r["combined"]


def main(out):
    rng = random.Random(0x4C61636861696E)
    t = {}
    t["tpke_n4"] = tpke(rng, 4, 1, 2, {(0, 1): "reversed", (1, 2): "random_g1", (1, 0): "other_player"})
    t["tpke_n22"] = tpke(rng, 22, 7, 2, {(0, 0): "reversed", (0, 3): "random_g1", (0, 5): "infinity",
                                         (1, 1): "other_player", (1, 2): "random_g1", (1, 20): "reversed"})
    t["ts_n7"] = ts(rng, 7, 2, [coin_id(1, 0, 5), coin_id(1, 3, 7)],
                    {(0, 0): "reversed", (0, 2): "random_g2", (1, 1): "other_player", (1, 3): "infinity"})
    bad100 = {(0, i): k for i, k in zip((0, 4, 9, 17, 30, 33), ("random_g2", "reversed", "other_player", "infinity",
                                                                 "random_g2", "other_player"))}
    t["ts_n100"] = ts(rng, 100, 33, [coin_id(0, 2, 5)], bad100)
    pyref_check(t)
    with open(out, "w") as fo:
        json.dump(t, fo, indent=0, sort_keys=True)
    print("wrote", out)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else os.path.join(HERE, "transcripts.json"))
