"""CPU checks of the committed TPKE / threshold-signature transcripts (tests/golden/transcripts.json, made by
tests/golden/make_transcripts.py): the oracle reproduces every decision and output, and the independent
pure-Python restatement (tests/pyref/bls12_381.py: flat Fp12, affine Miller loop, plain final exponentiation, its own
hash-to-G2) re-derives a sample: hash-to-G2 of a ciphertext and a coin message, the pairing decisions of 4 TPKE and 3
threshold-signature shares (honest and malicious), and both Lagrange combinations."""
import json
import os
import sys

import oracle as o

HERE = os.path.dirname(os.path.abspath(__file__))
T = json.load(open(os.path.join(HERE, "golden", "transcripts.json")))
H = bytes.fromhex


def test_oracle_reproduces_tpke():
    for key in ("tpke_n4", "tpke_n22"):
        t = T[key]
        for c in t["ciphertexts"]:
            u, v, w = H(c["u"]), H(c["v"]), H(c["w"])
            got = [o.tpke_verify_share(H(t["y_i"][i]), u, v, w, H(s)) == 1 for i, s in enumerate(c["shares"])]
            assert got == c["accept"]
            assert sum(got) < t["n"]                     # every transcript carries malicious shares
            ids = c["combine_ids"]
            assert ids == [i for i in range(t["n"]) if c["accept"][i]][: t["f"] + 1]
            assert o.tpke_full_decrypt(v, ids, [H(c["shares"][i]) for i in ids]).hex() == c["plaintext"] == c["data"]


def test_oracle_reproduces_ts():
    for key in ("ts_n7", "ts_n100"):
        t = T[key]
        for r in t["rounds"]:
            m = H(r["msg"])
            assert o.g2_hash(m).hex() == r["h"]
            got = [o.ts_validate(H(t["pk_i"][i]), H(s), m) == 1 for i, s in enumerate(r["sigs"])]
            assert got == r["accept"] and sum(got) < t["n"]
            ids = r["assemble_ids"]
            comb = o.g2_lagrange([o.fr(i + 1) for i in ids], [H(r["sigs"][i]) for i in ids])
            assert comb.hex() == r["combined"]
            assert o.ts_validate(H(t["pk"]), comb, m) == 1


def test_independent_python_restatement():
    sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tests", "golden"))
    sys.path.insert(0, os.path.join(HERE, "golden"))
    from make_transcripts import pyref_check
    pyref_check(T)
