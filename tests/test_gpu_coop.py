"""The cooperative pairing check (coop.hpp / k_coop.hip: nine lanes per check) against the one-lane kernels and the
oracle.  Its final exponentiation must give the same GT element, bit for bit, as the one-lane k_final_exp_check and as
the oracle's final_exp (pairing.hpp's mcl expHardPartBLS12 shape, GT = e^3) on arbitrary Fp12 inputs; its Miller loop
is checked through the decisions of the randomized batch check, with every level forced onto the cooperative kernels
and with them disabled (a wrong Miller value rejects valid groups)."""
import json
import os
import random

import numpy as np
import pytest

import oracle as o
from helpers import gpu_native

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
T = json.load(open(os.path.join(HERE, "golden", "transcripts.json")))
H = bytes.fromhex
RM = 1 << 384


@pytest.fixture(scope="module")
def nat():
    return gpu_native()


def raw_to_words(raw: bytes):
    """GT bytes (12 canonical Fp, 48 B LE each) -> 144 u32 words in Montgomery form"""
    out = []
    for k in range(12):
        v = int.from_bytes(raw[48 * k:48 * k + 48], "little") * RM % o.P
        out += [(v >> (32 * i)) & 0xFFFFFFFF for i in range(12)]
    return out


def words_to_raw(words):
    rinv = pow(RM, -1, o.P)
    b = b""
    for k in range(12):
        v = sum(words[12 * k + i] << (32 * i) for i in range(12))
        b += (v * rinv % o.P).to_bytes(48, "little")
    return b


OPS = {0: "sqr12", 1: "cyc_sqr", 2: "mul12", 3: "mul12_conj", 4: "frob1", 5: "frob2", 6: "frob3", 7: "inv",
       8: "conj", 9: "line", 10: "final_exp"}


def test_coop_ops_match_one_lane(nat):
    """every cooperative Fp12 operation on 16 random values (and one unitary value for the cyclotomic square) equals
    the one-lane field.hpp / pairing.hpp routine, word for word"""
    rng = random.Random(99)
    rnd = lambda: raw_to_words(b"".join(rng.randrange(o.P).to_bytes(48, "little") for _ in range(12)))
    a = [rnd() for _ in range(16)]
    b = [rnd() for _ in range(16)]
    # a unitary value (final exponentiation output) for the cyclotomic square
    u = raw_to_words(o.pairing(o.g1_gen(), o.g2_gen()))
    bad = []
    for op, name in OPS.items():
        aa = [u] * 16 if op == 1 else a
        out, ref = nat.debug_coop_op(op, aa, b)
        if out != ref:
            bad.append((name, [i for i in range(16) if out[i] != ref[i]][:4],
                        [w // 24 for w in range(144) if out[0][w] != ref[0][w]][:6]))
    assert not bad, bad


def test_coop_final_exp_bit_exact(nat):
    """39 random Fp12 values, 1 and a real Miller value: nine-lane == one-lane == oracle"""
    rng = random.Random(20261017)
    raws = [b"".join(rng.randrange(o.P).to_bytes(48, "little") for _ in range(12)) for _ in range(39)]
    one = (1).to_bytes(48, "little") + bytes(48 * 11)
    raws.append(one)
    raws.append(o.miller_loop(o.g1_mul(o.g1_gen(), o.fr(5)), o.g2_gen()))
    vals = [raw_to_words(r) for r in raws]
    coop = nat.debug_final_exp(vals, coop=True)
    lane = nat.debug_final_exp(vals, coop=False)
    assert coop == lane
    for k in (0, 1, 17, len(raws) - 2, len(raws) - 1):
        assert words_to_raw(coop[k]) == o.final_exp(raws[k]), k
    assert words_to_raw(coop[len(raws) - 2]) == one
    # e(5 G1, G2) = e(G1, G2)^5
    assert words_to_raw(coop[-1]) == o.gt_pow(o.pairing(o.g1_gen(), o.g2_gen()), o.fr(5))


def test_coop_final_exp_many_items(nat):
    """more items than one wave holds (7 per wave, 64-lane workgroups): every item its own result"""
    rng = random.Random(7)
    base = [raw_to_words(b"".join(rng.randrange(o.P).to_bytes(48, "little") for _ in range(12))) for _ in range(5)]
    vals = [base[i % 5] for i in range(100)]
    coop = nat.debug_final_exp(vals, coop=True)
    lane = nat.debug_final_exp(base, coop=False)
    for i in range(100):
        assert coop[i] == lane[i % 5], i


@pytest.fixture(params=["coop_all", "coop_off"])
def coop_mode(nat, request):
    nat.set_coop_max((1 << 30) if request.param == "coop_all" else 0)
    yield request.param
    nat.set_coop_max(32768)


@pytest.mark.parametrize("key", ["tpke_n4", "tpke_n22", "ts_n7", "ts_n100"])
def test_batched_transcripts_coop(nat, coop_mode, key):
    t = T[key]
    if key.startswith("tpke"):
        cts = [(H(c["u"]), H(c["v"]), H(c["w"])) for c in t["ciphertexts"]]
        shares = [(ci, i, H(s)) for ci, c in enumerate(t["ciphertexts"]) for i, s in enumerate(c["shares"])]
        got = nat.tpke_verify_shares([H(y) for y in t["y_i"]], cts, shares, batched=True)
        assert got == [a for c in t["ciphertexts"] for a in c["accept"]]
    else:
        msgs = [H(r["msg"]) for r in t["rounds"]]
        items = [(ri, i, H(s)) for ri, r in enumerate(t["rounds"]) for i, s in enumerate(r["sigs"])]
        got = nat.ts_verify_shares([H(p) for p in t["pk_i"]], msgs, items, batched=True)
        assert got == [a for r in t["rounds"] for a in r["accept"]]


def test_batched_density_coop(nat, coop_mode):
    """22 decryptors, 30 % wrong shares: every level (groups, search, singles) on the selected kernels"""
    from test_gpu_batched import Batch
    b = Batch(b"gpu-coop-density", 22, 7, 5)
    rng = np.random.default_rng(3)
    n = 5 * 22 * 4
    bad = rng.random(n) < 0.3
    ct = [i // 22 % 5 for i in range(n)]
    dec = [i % 22 for i in range(n)]
    shares = [(ct[i], dec[i], (b.bad if bad[i] else b.good)[ct[i]][dec[i]]) for i in range(n)]
    got = nat.tpke_verify_shares(b.yi, b.cts, shares, batched=True)
    assert got == [not x for x in bad]


@pytest.mark.parametrize("general_lines", [False, True])
@pytest.mark.parametrize("key", ["tpke_n4", "tpke_n22"])
def test_exact_transcripts_coop(nat, coop_mode, key, general_lines):
    """The exact per-share check (lcb_tpke_verify_shares) on the nine-lane kernels (small batches) and on the one-lane
    kernels: the transcripts' decisions either way, with normalised line sets and with every set forced onto the
    on-the-fly fallback (k_rlc_miller_fallback)"""
    nat.set_line_mode(general_lines)
    try:
        t = T[key]
        cts = [(H(c["u"]), H(c["v"]), H(c["w"])) for c in t["ciphertexts"]]
        shares = [(ci, i, H(s)) for ci, c in enumerate(t["ciphertexts"]) for i, s in enumerate(c["shares"])]
        want = [a for c in t["ciphertexts"] for a in c["accept"]]
        assert nat.tpke_verify_shares([H(y) for y in t["y_i"]], cts, shares) == want
        # a malformed share (bytes reversed, HoneyBadgerMalicious.cs:23) and a valid point that is not the share
        ys = [H(y) for y in t["y_i"]]
        bad = [(0, 0, shares[0][2][::-1]), (0, 1, shares[0][2])]
        exp = [o.g1_valid(ui) and o.tpke_verify_share(ys[d], *cts[c], ui) == 1 for c, d, ui in bad]
        assert exp[1] is False
        assert nat.tpke_verify_shares(ys, cts, bad + shares[:3]) == exp + want[:3]
    finally:
        nat.set_line_mode(False)
